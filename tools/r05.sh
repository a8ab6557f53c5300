#!/bin/bash
# Round-5 GPU experiments, one mode per gpurun call; output under gpurun_out/r05/<mode>.
#   driver  the driver's exact bench command (--steps 20 --warmup 5) as the box's first GPU
#           process, with per-launch times; the same under rocprofv3 kernel traces (every
#           dispatch, warm-ups included) for the gathered loader and stream mode; 400-launch
#           traces from cold; rotated vs one-buffer; the rotated streaming-read ceiling
set -e
mode=${1:?mode}
out=gpurun_out/r05/$mode
mkdir -p "$out"
export TMPDIR=/tmp

bench() {  # bench NAME ARGS... -> $out/NAME.json (appended)
  name=$1; shift
  timeout -k 10 300 python3 bench.py "$@" >> "$out/$name.json" 2>> "$out/$name.err"
}
trace() {  # trace NAME ARGS...: kernel trace + stats of one bench command (env passes through)
  name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/$name" -o run \
      -- python3 bench.py "$@" > "$out/$name.log" 2>&1
}

case $mode in
driver)
  bench n1_default --gpus 1 --steps 20 --warmup 5 --per-launch
  AIPSTACK_CHKSUM_GATHER=-1 bench n1_stream --gpus 1 --steps 20 --warmup 5 --per-launch --no-cpu-baseline
  bench n1_rot1 --gpus 1 --steps 20 --warmup 5 --per-launch --no-cpu-baseline --rotate 1
  trace tr_default --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-ceiling
  AIPSTACK_CHKSUM_GATHER=-1 trace tr_stream --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-ceiling
  trace long_default --steps 400 --warmup 0 --no-cpu-baseline --no-ceiling
  AIPSTACK_CHKSUM_GATHER=-1 trace long_stream --steps 400 --warmup 0 --no-cpu-baseline --no-ceiling
  trace long_rot1 --steps 400 --warmup 0 --no-cpu-baseline --no-ceiling --rotate 1
  timeout -k 10 120 tools/build/hbm_peak ceiling > "$out/ceiling.jsonl"
  timeout -k 10 120 tools/build/hbm_peak ceiling >> "$out/ceiling.jsonl"
  ;;
short)  # round-5 short runs (gather 1, the strided default) vs the round-4 gathered stream (0)
  bench n1_short --gpus 1 --steps 20 --warmup 5 --per-launch
  AIPSTACK_CHKSUM_GATHER=0 bench n1_gath --gpus 1 --steps 20 --warmup 5 --per-launch --no-cpu-baseline
  bench n1_short --gpus 1 --steps 20 --warmup 5 --per-launch --no-cpu-baseline
  AIPSTACK_CHKSUM_GATHER=0 bench n1_gath --gpus 1 --steps 20 --warmup 5 --per-launch --no-cpu-baseline
  trace long_short --steps 400 --warmup 0 --no-cpu-baseline --no-ceiling
  AIPSTACK_CHKSUM_GATHER=0 trace long_gath --steps 400 --warmup 0 --no-cpu-baseline --no-ceiling
  trace tr_short --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-ceiling
  for cp in 0 2 4; do
    AIPSTACK_CHKSUM_CHUNK_PACKETS=$cp bench B_cp$cp --config B --steps 20 --warmup 5 --per-launch --no-cpu-baseline
  done
  AIPSTACK_CHKSUM_GATHER=0 bench B_gath --config B --steps 20 --warmup 5 --per-launch --no-cpu-baseline
  bench C_gath --config C --steps 20 --warmup 5 --per-launch --no-cpu-baseline
  for cp in 0 8 32; do
    AIPSTACK_CHKSUM_GATHER=2 AIPSTACK_CHKSUM_CHUNK_PACKETS=$cp bench C_short$cp --config C --steps 20 --warmup 5 --per-launch --no-cpu-baseline
  done
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
      -k "every_read_form or short_runs or full_size or config_d or stream_mode or ragged or lengths" \
      > "$out/pytest.log" 2>&1
  ;;
shape)  # A's loaders at steady state, interleaved in one process (tools/ab.py), occupancy via
        # lds_pad; their instruction mix; TX2K's line stores (tx_store 2) against 2-byte stores
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
      -k "slotted_tx or tx_line or random_frames or every_read_form or short_runs" \
      > "$out/pytest.log" 2>&1
  timeout -k 10 300 python3 tools/ab.py --config A --variants \
      "gather=0;gather=1;gather=1,lds_pad=33792;gather=1,lds_pad=41984;gather=0,lds_pad=33000;gather=1,chunk_packets=4;gather=1,chunk_packets=16;gather=-1" \
      > "$out/ab_A.jsonl" 2> "$out/ab_A.err"
  for g in 0 1; do
    AIPSTACK_CHKSUM_GATHER=$g timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv \
        -d "$out/pmc_A_g$g" -o run --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD \
        SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES -- python3 bench.py --config A \
        --no-cpu-baseline --no-parity --no-ceiling --steps 5 --warmup 2 > "$out/pmc_A_g$g.log" 2>&1
  done
  for i in 1 2; do
    for st in 0 2; do
      AIPSTACK_CHKSUM_TX_STORE=$st bench TX2K_st$st --config TX2K --steps 20 --warmup 5 --per-launch --no-cpu-baseline
    done
  done
  for st in 0 2; do
    AIPSTACK_CHKSUM_TX_STORE=$st timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv \
        -d "$out/pmc_TX2K_st$st" -o run --pmc WRITE_SIZE GRBM_GUI_ACTIVE -- python3 bench.py \
        --config TX2K --no-cpu-baseline --no-parity --steps 5 --warmup 2 > "$out/pmc_TX2K_st$st.log" 2>&1
    AIPSTACK_CHKSUM_TX_STORE=$st timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv \
        -d "$out/pmcf_TX2K_st$st" -o run --pmc FETCH_SIZE -- python3 bench.py \
        --config TX2K --no-cpu-baseline --no-parity --steps 5 --warmup 2 > "$out/pmcf_TX2K_st$st.log" 2>&1
  done
  ;;
occ)  # A at fewer waves per CU (lds_pad), short runs' chunk sizes and load forms
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
      -k "every_read_form or short_runs" > "$out/pytest.log" 2>&1
  AIPSTACK_CHKSUM_SHORT_LOADS=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 \
      --timeout-method thread -k "every_read_form or short_runs or full_size" > "$out/pytest_gl.log" 2>&1
  timeout -k 10 600 python3 tools/ab.py --config A --rounds 16 --variants \
      "gather=0;gather=1,lds_pad=41984;gather=1,lds_pad=54000;gather=1,chunk_packets=4,lds_pad=41984;gather=1,chunk_packets=16,lds_pad=41984;gather=1,chunk_packets=16,lds_pad=54000;gather=1,short_loads=1;gather=1,short_loads=1,lds_pad=41984;gather=0,lds_pad=54000;gather=1,chunk_packets=32,lds_pad=54000;gather=1,chunk_packets=4,lds_pad=54000" \
      > "$out/ab_A.jsonl" 2> "$out/ab_A.err"
  timeout -k 10 120 tools/build/hbm_peak ceiling > "$out/ceiling.jsonl"
  ;;
driver2)  # short runs at 3 waves per SIMD (the default) under the driver's protocol, against
          # the gathered stream; B and C shapes at steady state
  bench n1_def --gpus 1 --steps 20 --warmup 5 --per-launch
  AIPSTACK_CHKSUM_GATHER=0 bench n1_gath --gpus 1 --steps 20 --warmup 5 --per-launch --no-cpu-baseline
  bench n1_def --gpus 1 --steps 20 --warmup 5 --per-launch --no-cpu-baseline
  AIPSTACK_CHKSUM_GATHER=0 AIPSTACK_CHKSUM_LDS_PAD=33000 bench n1_gath3 --gpus 1 --steps 20 --warmup 5 --per-launch --no-cpu-baseline
  trace tr_def --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-ceiling
  trace long_def --steps 400 --warmup 0 --no-cpu-baseline --no-ceiling
  AIPSTACK_CHKSUM_GATHER=0 AIPSTACK_CHKSUM_LDS_PAD=33000 trace long_gath3 --steps 400 --warmup 0 --no-cpu-baseline --no-ceiling
  bench B_def --config B --steps 20 --warmup 5 --per-launch --no-cpu-baseline
  bench C_def --config C --steps 20 --warmup 5 --per-launch --no-cpu-baseline
  timeout -k 10 600 python3 tools/ab.py --config B --rounds 12 --variants \
      "gather=1;gather=1,lds_pad=-1;gather=1,chunk_packets=2;gather=1,chunk_packets=2,lds_pad=-1;gather=0;gather=0,lds_pad=33000" \
      > "$out/ab_B.jsonl" 2> "$out/ab_B.err"
  timeout -k 10 600 python3 tools/ab.py --config C --rounds 12 --variants \
      "gather=1;gather=1,lds_pad=33000;gather=2;gather=2,lds_pad=-1;gather=2,chunk_packets=32;gather=2,chunk_packets=8" \
      > "$out/ab_C.jsonl" 2> "$out/ab_C.err"
  ;;
clock)  # the new defaults under the driver's protocol; per-dispatch clocks (GRBM_GUI_ACTIVE)
        # through the first 60 launches, short runs against the gathered stream
  bench n1_def --gpus 1 --steps 20 --warmup 5 --per-launch
  bench C_def --config C --steps 20 --warmup 5 --per-launch --no-cpu-baseline
  bench B_def --config B --steps 20 --warmup 5 --per-launch --no-cpu-baseline
  bench n1_def --gpus 1 --steps 20 --warmup 5 --per-launch --no-cpu-baseline
  for g in 1 0; do
    AIPSTACK_CHKSUM_GATHER=$g timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv \
        -d "$out/clk_g$g" -o run --pmc GRBM_GUI_ACTIVE GRBM_COUNT -- python3 bench.py \
        --config A --no-cpu-baseline --no-parity --no-ceiling --steps 60 --warmup 0 \
        > "$out/clk_g$g.log" 2>&1
  done
  trace long_def --steps 400 --warmup 0 --no-cpu-baseline --no-ceiling
  ;;
col)  # column runs (tunable short_loads 2): parity, steady state against the defaults, the
      # driver's protocol at 4 and 3 waves per SIMD, instruction mix
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
      -k "short_run or every_read_form or full_size" > "$out/pytest.log" 2>&1
  AIPSTACK_CHKSUM_SHORT_LOADS=2 bench n1_col --gpus 1 --steps 20 --warmup 5 --per-launch --no-cpu-baseline
  AIPSTACK_CHKSUM_SHORT_LOADS=2 AIPSTACK_CHKSUM_LDS_PAD=26000 bench n1_col3 --gpus 1 --steps 20 --warmup 5 --per-launch --no-cpu-baseline
  bench n1_def --gpus 1 --steps 20 --warmup 5 --per-launch --no-cpu-baseline
  timeout -k 10 600 python3 tools/ab.py --config A --rounds 12 --variants \
      "short_loads=0;short_loads=2;short_loads=2,lds_pad=26000;short_loads=2,lds_pad=38000;gather=0;short_loads=2,chunk_packets=16" \
      > "$out/ab_A.jsonl" 2> "$out/ab_A.err"
  timeout -k 10 600 python3 tools/ab.py --config C --rounds 8 --variants \
      "short_loads=0;short_loads=2;short_loads=2,lds_pad=26000;short_loads=2,chunk_packets=8" \
      > "$out/ab_C.jsonl" 2> "$out/ab_C.err"
  timeout -k 10 600 python3 tools/ab.py --config B --rounds 8 --variants \
      "short_loads=0;short_loads=2;short_loads=2,lds_pad=26000;short_loads=2,chunk_packets=2" \
      > "$out/ab_B.jsonl" 2> "$out/ab_B.err"
  AIPSTACK_CHKSUM_SHORT_LOADS=2 AIPSTACK_CHKSUM_LDS_PAD=26000 trace long_col3 --steps 300 --warmup 0 --no-cpu-baseline --no-ceiling
  AIPSTACK_CHKSUM_SHORT_LOADS=2 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv \
      -d "$out/pmc_A_col" -o run --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD \
      SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES -- python3 bench.py --config A \
      --no-cpu-baseline --no-parity --no-ceiling --steps 5 --warmup 2 > "$out/pmc_A_col.log" 2>&1
  timeout -k 10 120 tools/build/hbm_peak trace 1 > "$out/read_trace.jsonl"
  ;;
confirm)  # the round-5 defaults: the driver's exact command (first GPU process, then again),
          # its rocprof kernel trace, a 300-launch trace, B and C, PMC traffic for A, B, C
  bench n1 --gpus 1 --steps 20 --warmup 5 --per-launch
  bench n1 --gpus 1 --steps 20 --warmup 5 --per-launch --no-cpu-baseline
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_A" -o run \
      -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$out/prof_A.log" 2>&1
  bench n1 --gpus 1 --steps 20 --warmup 5 --per-launch --no-cpu-baseline
  bench B --config B --steps 20 --warmup 5 --per-launch
  bench C --config C --steps 20 --warmup 5 --per-launch
  trace long_A --steps 300 --warmup 0 --no-cpu-baseline --no-ceiling
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
      -k "short_run or every_read_form or full_size or config_d" > "$out/pytest.log" 2>&1
  for c in A B C; do tools/pmc_run.sh $c "$out/pmc_$c"; done
  ;;
gate)  # the whole GPU suite and smoke() on this tree; the ceiling probe's new shapes; RX and
       # TXREC at 3 workgroups per CU (lds_pad) against their 4
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
      > "$out/pytest_gpu.log" 2>&1
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1
  timeout -k 10 120 tools/build/hbm_peak ceiling > "$out/ceiling.jsonl"
  timeout -k 10 120 tools/build/hbm_peak ceiling >> "$out/ceiling.jsonl"
  for i in 1 2; do
    bench RX --config RX --steps 20 --warmup 5 --per-launch --no-cpu-baseline
    AIPSTACK_CHKSUM_LDS_PAD=4000 bench RX_pad --config RX --steps 20 --warmup 5 --per-launch --no-cpu-baseline
    bench TXREC --config TXREC --steps 20 --warmup 5 --per-launch --no-cpu-baseline
    AIPSTACK_CHKSUM_LDS_PAD=4000 bench TXREC_pad --config TXREC --steps 20 --warmup 5 --per-launch --no-cpu-baseline
  done
  ;;
slot)  # slot windows (tunable slot_windows 1) on ring slots and gaps: parity, steady state
       # against the gathered stream, the driver's protocol, instruction mix
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
      -k "slot_windows or slotted_checksums or slotted_packets or overlapping" > "$out/pytest.log" 2>&1
  timeout -k 10 600 python3 tools/ab.py --config C2K --rounds 10 --variants \
      "slot_windows=0;slot_windows=1;slot_windows=1,chunk_packets=16;slot_windows=1,chunk_packets=4" \
      > "$out/ab_C2K.jsonl" 2> "$out/ab_C2K.err"
  timeout -k 10 600 python3 tools/ab.py --config A2K --rounds 10 --variants \
      "slot_windows=0;slot_windows=1;slot_windows=1,chunk_packets=16" > "$out/ab_A2K.jsonl" 2> "$out/ab_A2K.err"
  for sw in 0 1; do
    AIPSTACK_CHKSUM_SLOT_WINDOWS=$sw bench C2K_sw$sw --config C2K --steps 20 --warmup 5 --per-launch --no-cpu-baseline
    AIPSTACK_CHKSUM_SLOT_WINDOWS=$sw bench A2K_sw$sw --config A2K --steps 20 --warmup 5 --per-launch --no-cpu-baseline
    AIPSTACK_CHKSUM_SLOT_WINDOWS=$sw timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv \
        -d "$out/pmc_C2K_sw$sw" -o run --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD \
        SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES -- python3 bench.py --config C2K \
        --no-cpu-baseline --no-parity --steps 5 --warmup 2 > "$out/pmc_C2K_sw$sw.log" 2>&1
    AIPSTACK_CHKSUM_SLOT_WINDOWS=$sw timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv \
        -d "$out/pmcf_C2K_sw$sw" -o run --pmc FETCH_SIZE -- python3 bench.py --config C2K \
        --no-cpu-baseline --no-parity --steps 5 --warmup 2 > "$out/pmcf_C2K_sw$sw.log" 2>&1
  done
  ;;
segtab)  # segment-table runs (short_loads 3) against column runs and stream prefixes
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
      -k "short_run or every_read_form" > "$out/pytest.log" 2>&1
  timeout -k 10 600 python3 tools/ab.py --config C --rounds 10 --variants \
      "short_loads=0;short_loads=2;short_loads=3;short_loads=3,chunk_packets=32;short_loads=3,chunk_packets=8" \
      > "$out/ab_C.jsonl" 2> "$out/ab_C.err"
  timeout -k 10 600 python3 tools/ab.py --config A --rounds 10 --variants \
      "short_loads=2;short_loads=3;short_loads=3,chunk_packets=16;short_loads=0" > "$out/ab_A.jsonl" 2> "$out/ab_A.err"
  timeout -k 10 600 python3 tools/ab.py --config B --rounds 8 --variants \
      "short_loads=2;short_loads=3;short_loads=3,chunk_packets=2" > "$out/ab_B.jsonl" 2> "$out/ab_B.err"
  for m in 3 0 3 0; do
    AIPSTACK_CHKSUM_SHORT_LOADS=$m bench C_m$m --config C --steps 20 --warmup 5 --per-launch --no-cpu-baseline
  done
  for m in 3 2; do
    AIPSTACK_CHKSUM_SHORT_LOADS=$m bench A_m$m --config A --steps 20 --warmup 5 --per-launch --no-cpu-baseline
    AIPSTACK_CHKSUM_SHORT_LOADS=$m bench B_m$m --config B --steps 20 --warmup 5 --per-launch --no-cpu-baseline
  done
  AIPSTACK_CHKSUM_SHORT_LOADS=3 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv \
      -d "$out/pmc_C_m3" -o run --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD \
      SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES -- python3 bench.py --config C \
      --no-cpu-baseline --no-parity --no-ceiling --steps 5 --warmup 2 > "$out/pmc_C_m3.log" 2>&1
  ;;
shape5)  # chunk sizes of the gathered stream, the chain groups and the frame chunks under the
         # driver's protocol (the round-4 choices were steady-state ones), two passes
  for pass in 1 2; do
    for cp in 0 16 32; do
      AIPSTACK_CHKSUM_CHUNK_PACKETS=$cp bench C2K_cp$cp --config C2K --steps 20 --warmup 5 --per-launch --no-cpu-baseline
    done
    AIPSTACK_CHKSUM_STREAM=8 bench C2K_su8 --config C2K --steps 20 --warmup 5 --per-launch --no-cpu-baseline
    for cp in 0 16; do
      AIPSTACK_CHKSUM_CHUNK_PACKETS=$cp bench A2K_cp$cp --config A2K --steps 20 --warmup 5 --per-launch --no-cpu-baseline
    done
    AIPSTACK_CHKSUM_SLOT_WINDOWS=1 bench A2K_slotwin --config A2K --steps 20 --warmup 5 --per-launch --no-cpu-baseline
    for cp in 0 64; do
      AIPSTACK_CHKSUM_CHUNK_PACKETS=$cp bench CHAIN_cp$cp --config CHAIN --steps 20 --warmup 5 --per-launch --no-cpu-baseline
    done
    for cp in 0 64; do
      AIPSTACK_CHKSUM_CHUNK_PACKETS=$cp bench RX_cp$cp --config RX --steps 20 --warmup 5 --per-launch --no-cpu-baseline
      AIPSTACK_CHKSUM_CHUNK_PACKETS=$cp bench RX2K_cp$cp --config RX2K --steps 20 --warmup 5 --per-launch --no-cpu-baseline
    done
  done
  ;;
tab)  # the gathered stream's segment tables (default build) against the scan (lib_notab,
      # -DAIPSTACK_GATHER_TAB=0), driver protocol, two passes; the GPU suite first
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
      > "$out/pytest_gpu.log" 2>&1
  for pass in 1 2; do
    for c in C2K A2K; do
      bench ${c}_tab --config $c --steps 20 --warmup 5 --per-launch --no-cpu-baseline
      AIPSTACK_AMD_LIB=tools/build/lib_notab.so bench ${c}_notab --config $c --steps 20 --warmup 5 --per-launch --no-cpu-baseline
    done
  done
  ;;
lanes)  # the read probe's lane-contiguous shapes (LS segments per lane, hbm_peak lanes)
  timeout -k 10 200 tools/build/hbm_peak lanes > "$out/lanes.jsonl"
  timeout -k 10 120 tools/build/hbm_peak ceiling > "$out/ceiling.jsonl"
  ;;
shape6)  # launch shapes of the remaining configs under the driver's protocol (their round-4
         # choices were steady-state ones), two passes
  b() { n=$1; shift; env "$@" timeout -k 10 300 python3 bench.py --config ${n%%_*} --steps 20 \
        --warmup 5 --per-launch --no-cpu-baseline --no-ceiling >> "$out/$n.json" 2>> "$out/$n.err"; }
  for pass in 1 2; do
    b RX_def X=0;            b RX_su4 AIPSTACK_CHKSUM_STREAM=4;  b RX_cp16 AIPSTACK_CHKSUM_CHUNK_PACKETS=16
    b RX_cp24 AIPSTACK_CHKSUM_CHUNK_PACKETS=24;  b RX_wpc64 AIPSTACK_CHKSUM_WAVES_PER_CU=64
    b TXREC_def X=0;         b TXREC_su4 AIPSTACK_CHKSUM_STREAM=4
    b TXREC_cp24 AIPSTACK_CHKSUM_CHUNK_PACKETS=24
    b TX_def X=0;            b TX_su4 AIPSTACK_CHKSUM_STREAM=4;  b TX_g0 AIPSTACK_CHKSUM_TX_GATHER=0
    b RX2K_def X=0;          b RX2K_cp16 AIPSTACK_CHKSUM_CHUNK_PACKETS=16
    b TX2K_def X=0;          b TX2K_cp16 AIPSTACK_CHKSUM_CHUNK_PACKETS=16
    b CHAIN_def X=0;         b CHAIN_cp16 AIPSTACK_CHKSUM_CHUNK_PACKETS=16;  b CHAIN_su2 AIPSTACK_CHKSUM_STREAM=2
    b A2K_def X=0;           b A2K_su4 AIPSTACK_CHKSUM_STREAM=4;  b A2K_cp4 AIPSTACK_CHKSUM_CHUNK_PACKETS=4
    b C2K_def X=0;           b C2K_su2 AIPSTACK_CHKSUM_STREAM=2
    b C_def X=0;             b C_cp8 AIPSTACK_CHKSUM_CHUNK_PACKETS=8;  b C_cp32 AIPSTACK_CHKSUM_CHUNK_PACKETS=32
    b B_def X=0;             b B_cp2 AIPSTACK_CHKSUM_CHUNK_PACKETS=2
  done
  ;;
rx5)  # frame shapes after the round-5 changes (4 stream windows, 32-frame capture); Rx verify
      # at 5 waves per SIMD (lib_rx5) against 4; the frame tests first
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
      -k "frame or rx or tx or slotted or gathered" > "$out/pytest.log" 2>&1
  b() { n=$1; shift; env "$@" timeout -k 10 300 python3 bench.py --config ${n%%_*} --steps 20 \
        --warmup 5 --per-launch --no-cpu-baseline --no-ceiling >> "$out/$n.json" 2>> "$out/$n.err"; }
  for pass in 1 2 3; do
    b RX_def X=0;  b RX_rx5 AIPSTACK_AMD_LIB=tools/build/lib_rx5.so
    b RX2K_def X=0;  b RX2K_rx5 AIPSTACK_AMD_LIB=tools/build/lib_rx5.so
    b TXREC_def X=0;  b TX_def X=0;  b A2K_def X=0
  done
  ;;
edge)  # short runs' stream prefixes with packet starts' edge segments loaded up front (default
       # build) against partial segments from the stream (lib_noedge), driver protocol
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
      -k "read_form or short_runs or csr or lengths or random_packet or full_size or golden or config" \
      > "$out/pytest.log" 2>&1
  b() { n=$1; shift; env "$@" timeout -k 10 300 python3 bench.py --config ${n%%_*} --steps 20 \
        --warmup 5 --per-launch --no-cpu-baseline --no-ceiling >> "$out/$n.json" 2>> "$out/$n.err"; }
  for pass in 1 2 3; do
    b C_edge X=0;  b C_noedge AIPSTACK_AMD_LIB=tools/build/lib_noedge.so
    b A_m0edge AIPSTACK_CHKSUM_SHORT_LOADS=0
    b A_m0noedge AIPSTACK_CHKSUM_SHORT_LOADS=0 AIPSTACK_AMD_LIB=tools/build/lib_noedge.so
  done
  ;;
gapcol)  # gapped column runs (the new default for strides that are multiples of 16) against the
         # gathered stream (gather 0), driver protocol; the strided/gapped tests first
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
      -k "strided or slotted or lengths or overlapping or read_form or random_packet or golden or engine_host" \
      > "$out/pytest.log" 2>&1
  b() { n=$1; shift; env "$@" timeout -k 10 300 python3 bench.py --config ${n%%_*} --steps 20 \
        --warmup 5 --per-launch --no-cpu-baseline --no-ceiling >> "$out/$n.json" 2>> "$out/$n.err"; }
  for pass in 1 2 3; do
    b A2K_cols X=0;  b A2K_gath AIPSTACK_CHKSUM_GATHER=0
  done
  ;;
txsplit)  # the send ring's split fill (records pass + scatter) against its one-pass fill, and
          # the CSR fill's one pass against its split, driver protocol
  b() { n=$1; shift; env X=0 timeout -k 10 300 python3 bench.py --config ${n%%_*} --steps 20 \
        --warmup 5 --per-launch --no-cpu-baseline --no-ceiling "$@" >> "$out/$n.json" 2>> "$out/$n.err"; }
  for pass in 1 2 3; do
    b TX2K_one;  b TX2K_split --tx-split;  b TX_split;  b TX_one --tx-inplace
  done
  ;;
txmodes)  # the one-pass fills' header and store forms, the gapped column chunk size, under
          # the driver's protocol
  b() { n=$1; shift; env "$@" timeout -k 10 300 python3 bench.py --config ${n%%_*} --steps 20 \
        --warmup 5 --per-launch --no-cpu-baseline --no-ceiling >> "$out/$n.json" 2>> "$out/$n.err"; }
  for pass in 1 2; do
    b TX_def X=0;  b TX_g1 AIPSTACK_CHKSUM_TX_GATHER=1;  b TX_st1 AIPSTACK_CHKSUM_TX_STORE=1
    b TX_st1g2 AIPSTACK_CHKSUM_TX_STORE=1 AIPSTACK_CHKSUM_TX_GATHER=2
    b TX2K_def X=0;  b TX2K_st1 AIPSTACK_CHKSUM_TX_STORE=1
    b A2K_def X=0;  b A2K_cp4 AIPSTACK_CHKSUM_CHUNK_PACKETS=4;  b A2K_cp16 AIPSTACK_CHKSUM_CHUNK_PACKETS=16
  done
  ;;
edgeafter)  # the gathered stream's / gapped columns' edge segments read after the last group is
            # issued (default) against before the stream (lib_edgebefore); FETCH_SIZE of each
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
      -k "slotted or gathered or chain or strided or random or frame" > "$out/pytest.log" 2>&1
  b() { n=$1; shift; env "$@" timeout -k 10 300 python3 bench.py --config ${n%%_*} --steps 20 \
        --warmup 5 --per-launch --no-cpu-baseline --no-ceiling >> "$out/$n.json" 2>> "$out/$n.err"; }
  for pass in 1 2; do
    for c in C2K A2K CHAIN RX2K; do
      b ${c}_after X=0;  b ${c}_before AIPSTACK_AMD_LIB=tools/build/lib_edgebefore.so
    done
  done
  for c in C2K CHAIN; do
    for v in after before; do
      lib=""; [ $v = before ] && lib=tools/build/lib_edgebefore.so
      AIPSTACK_AMD_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv \
          -d "$out/pmc_${c}_$v" -o run --pmc FETCH_SIZE -- python3 bench.py --config $c \
          --no-cpu-baseline --no-parity --no-ceiling --steps 5 --warmup 2 > "$out/pmc_${c}_$v.log" 2>&1
    done
  done
  ;;
colu)  # column runs' windows per group: 8 (default) against 6 and 4 (lib_col6 / lib_col4)
  b() { n=$1; shift; env "$@" timeout -k 10 300 python3 bench.py --config ${n%%_*} --steps 20 \
        --warmup 5 --per-launch --no-cpu-baseline --no-ceiling >> "$out/$n.json" 2>> "$out/$n.err"; }
  for pass in 1 2 3; do
    for c in A B; do
      b ${c}_u8 X=0;  b ${c}_u6 AIPSTACK_AMD_LIB=tools/build/lib_col6.so
      b ${c}_u4 AIPSTACK_AMD_LIB=tools/build/lib_col4.so
    done
  done
  ;;
colb)  # B's 6-window column runs in the product build: the strided tests, then B and A
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
      -k "strided or lengths or read_form or short_runs or full_size or golden or random_packet" \
      > "$out/pytest.log" 2>&1
  for pass in 1 2; do
    bench B --config B --steps 20 --warmup 5 --per-launch --no-cpu-baseline --no-ceiling
    bench A --config A --steps 20 --warmup 5 --per-launch --no-cpu-baseline --no-ceiling
  done
  ;;
sru)  # short runs' (stream prefixes, config C) windows per group: 8 against 6 and 4
  b() { n=$1; shift; env "$@" timeout -k 10 300 python3 bench.py --config ${n%%_*} --steps 20 \
        --warmup 5 --per-launch --no-cpu-baseline --no-ceiling >> "$out/$n.json" 2>> "$out/$n.err"; }
  for pass in 1 2 3; do
    b C_u8 X=0;  b C_u6 AIPSTACK_AMD_LIB=tools/build/lib_sr6.so;  b C_u4 AIPSTACK_AMD_LIB=tools/build/lib_sr4.so
  done
  ;;
gcu)  # gapped column runs' windows per group (8 against 6, lib_gc6); C with the 6-window
      # short runs (product) and its tests
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
      -k "csr or read_form or short_runs or random_packet or config" > "$out/pytest.log" 2>&1
  b() { n=$1; shift; env "$@" timeout -k 10 300 python3 bench.py --config ${n%%_*} --steps 20 \
        --warmup 5 --per-launch --no-cpu-baseline --no-ceiling >> "$out/$n.json" 2>> "$out/$n.err"; }
  for pass in 1 2 3; do
    b A2K_u8 X=0;  b A2K_u6 AIPSTACK_AMD_LIB=tools/build/lib_gc6.so;  b C_def X=0
  done
  ;;
slotmask)  # ring slots' edges masked in the stream (lib_slotmask) against edge loads (default);
           # C2K time and FETCH_SIZE
  b() { n=$1; shift; env "$@" timeout -k 10 300 python3 bench.py --config ${n%%_*} --steps 20 \
        --warmup 5 --per-launch --no-cpu-baseline --no-ceiling >> "$out/$n.json" 2>> "$out/$n.err"; }
  for pass in 1 2 3; do
    b C2K_edge X=0;  b C2K_mask AIPSTACK_AMD_LIB=tools/build/lib_slotmask.so
  done
  for v in edge mask; do
    lib=""; [ $v = mask ] && lib=tools/build/lib_slotmask.so
    AIPSTACK_AMD_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv \
        -d "$out/pmc_C2K_$v" -o run --pmc FETCH_SIZE -- python3 bench.py --config C2K \
        --no-cpu-baseline --no-parity --no-ceiling --steps 5 --warmup 2 > "$out/pmc_C2K_$v.log" 2>&1
  done
  ;;
confirm2)  # the driver's exact command, three processes in a row, on the final device code
  for i in 1 2 3; do
    timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 >> "$out/n1.json" 2>> "$out/n1.err"
  done
  ;;
hcap)  # frames' H(A0) from the header capture (default) against a stream boundary (lib_nohcap)
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
      -k "frame or rx or tx" > "$out/pytest.log" 2>&1
  b() { n=$1; shift; env "$@" timeout -k 10 300 python3 bench.py --config ${n%%_*} --steps 20 \
        --warmup 5 --per-launch --no-cpu-baseline --no-ceiling >> "$out/$n.json" 2>> "$out/$n.err"; }
  for pass in 1 2 3; do
    for c in RX TXREC TX; do
      b ${c}_hcap X=0;  b ${c}_nohcap AIPSTACK_AMD_LIB=tools/build/lib_nohcap.so
    done
  done
  ;;
gtab)  # the gathered stream's chunk starts stored in LDS (default) against a ds_bpermute per
       # window (lib_nogtab); the GPU suite first
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
      > "$out/pytest_gpu.log" 2>&1
  b() { n=$1; shift; env "$@" timeout -k 10 300 python3 bench.py --config ${n%%_*} --steps 20 \
        --warmup 5 --per-launch --no-cpu-baseline --no-ceiling >> "$out/$n.json" 2>> "$out/$n.err"; }
  for pass in 1 2 3; do
    for c in C2K CHAIN RX2K TX2K; do
      b ${c}_gtab X=0;  b ${c}_nogtab AIPSTACK_AMD_LIB=tools/build/lib_nogtab.so
    done
  done
  ;;
fr6)  # frames' stream in groups of 6 windows (lib_fr6) against 4 (default); frame tests on fr6
  AIPSTACK_AMD_LIB=tools/build/lib_fr6.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -v \
      --timeout 120 --timeout-method thread -k "frame or rx or tx" > "$out/pytest.log" 2>&1
  b() { n=$1; shift; env "$@" timeout -k 10 300 python3 bench.py --config ${n%%_*} --steps 20 \
        --warmup 5 --per-launch --no-cpu-baseline --no-ceiling >> "$out/$n.json" 2>> "$out/$n.err"; }
  for pass in 1 2 3; do
    for c in RX TXREC TX; do
      b ${c}_su4 X=0;  b ${c}_su6 AIPSTACK_AMD_LIB=tools/build/lib_fr6.so
    done
  done
  ;;
fnt0)  # frames' stream loads at the default cache policy (lib_fnt0) against nontemporal
  b() { n=$1; shift; env "$@" timeout -k 10 300 python3 bench.py --config ${n%%_*} --steps 20 \
        --warmup 5 --per-launch --no-cpu-baseline --no-ceiling >> "$out/$n.json" 2>> "$out/$n.err"; }
  for pass in 1 2; do
    for c in TX TX2K RX; do
      b ${c}_nt X=0;  b ${c}_def AIPSTACK_AMD_LIB=tools/build/lib_fnt0.so
    done
  done
  ;;
retouch)  # in-place Tx fills loading the field dwords again right before the stores (lib_retouch)
  b() { n=$1; shift; env "$@" timeout -k 10 300 python3 bench.py --config ${n%%_*} --steps 20 \
        --warmup 5 --per-launch --no-cpu-baseline --no-ceiling >> "$out/$n.json" 2>> "$out/$n.err"; }
  for pass in 1 2; do
    for c in TX TX2K; do
      b ${c}_def X=0;  b ${c}_retouch AIPSTACK_AMD_LIB=tools/build/lib_retouch.so
    done
  done
  ;;
splitg)  # the split Tx fill's read pass without the field-line touches (tx_gather 1)
  b() { n=$1; shift; env "$@" timeout -k 10 300 python3 bench.py --config TX --steps 20 \
        --warmup 5 --per-launch --no-cpu-baseline --no-ceiling --tx-split >> "$out/$n.json" 2>> "$out/$n.err"; }
  for pass in 1 2 3; do
    b TXs_touch X=0;  b TXs_g1 AIPSTACK_CHKSUM_TX_GATHER=1
  done
  AIPSTACK_CHKSUM_TX_GATHER=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_g1" -o run \
      -- python3 bench.py --config TX --tx-split --steps 20 --warmup 5 --no-cpu-baseline --no-ceiling \
      > "$out/prof_g1.log" 2>&1
  ;;
frot)  # frame and ring-slot batches rotated over 3 copies (the new default) against one buffer
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
      -k "bench" > "$out/pytest.log" 2>&1
  b() { n=$1; shift; timeout -k 10 300 python3 bench.py --config ${n%%_*} --steps 20 \
        --warmup 5 --per-launch --no-cpu-baseline --no-ceiling "$@" >> "$out/$n.json" 2>> "$out/$n.err"; }
  for pass in 1 2; do
    for c in RX TXREC TX RX2K TX2K C2K; do
      b ${c}_rot3;  b ${c}_rot1 --rotate 1
    done
  done
  ;;
txrot)  # the Tx fill forms under rotation (3 copies): one pass against split, touches
  b() { n=$1; shift; env X=0 timeout -k 10 300 python3 bench.py --config ${n%%_*} --steps 20 \
        --warmup 5 --per-launch --no-cpu-baseline --no-ceiling "$@" >> "$out/$n.json" 2>> "$out/$n.err"; }
  for pass in 1 2; do
    b TX_one;  b TX_split --tx-split;  b TX2K_one;  b TX2K_split --tx-split
  done
  for pass in 1 2; do
    AIPSTACK_CHKSUM_TX_GATHER=1 timeout -k 10 300 python3 bench.py --config TX --steps 20 --warmup 5 \
        --per-launch --no-cpu-baseline --no-ceiling >> "$out/TX_g1.json" 2>> "$out/TX_g1.err"
    AIPSTACK_CHKSUM_TX_STORE=1 timeout -k 10 300 python3 bench.py --config TX --steps 20 --warmup 5 \
        --per-launch --no-cpu-baseline --no-ceiling >> "$out/TX_st1.json" 2>> "$out/TX_st1.err"
    AIPSTACK_CHKSUM_TX_STORE=2 timeout -k 10 300 python3 bench.py --config TX2K --steps 20 --warmup 5 \
        --per-launch --no-cpu-baseline --no-ceiling >> "$out/TX2K_st2.json" 2>> "$out/TX2K_st2.err"
    AIPSTACK_CHKSUM_TX_STORE=1 timeout -k 10 300 python3 bench.py --config TX2K --steps 20 --warmup 5 \
        --per-launch --no-cpu-baseline --no-ceiling >> "$out/TX2K_st1.json" 2>> "$out/TX2K_st1.err"
  done
  ;;
acp)  # A's column-run chunk size under the driver's protocol: 8 packets (default) against 16 and 4
  b() { n=$1; shift; env "$@" timeout -k 10 300 python3 bench.py --config A --steps 20 \
        --warmup 5 --per-launch --no-cpu-baseline --no-ceiling >> "$out/$n.json" 2>> "$out/$n.err"; }
  for pass in 1 2 3; do
    b A_cp8 X=0;  b A_cp16 AIPSTACK_CHKSUM_CHUNK_PACKETS=16;  b A_cp4 AIPSTACK_CHKSUM_CHUNK_PACKETS=4
  done
  ;;
ccp)  # C and C2K chunk sizes between the powers of two under the driver's protocol
  b() { n=$1; shift; env "$@" timeout -k 10 300 python3 bench.py --config ${n%%_*} --steps 20 \
        --warmup 5 --per-launch --no-cpu-baseline --no-ceiling >> "$out/$n.json" 2>> "$out/$n.err"; }
  for pass in 1 2; do
    b C_cp16 X=0;  b C_cp12 AIPSTACK_CHKSUM_CHUNK_PACKETS=12;  b C_cp24 AIPSTACK_CHKSUM_CHUNK_PACKETS=24
    b C2K_cp16 X=0;  b C2K_cp12 AIPSTACK_CHKSUM_CHUNK_PACKETS=12;  b C2K_cp24 AIPSTACK_CHKSUM_CHUNK_PACKETS=24
  done
  ;;
chrot)  # chains rotated over 3 rebased copies (the new default) against one buffer; the fill too
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
      -k "bench or chain" > "$out/pytest.log" 2>&1
  b() { n=$1; shift; timeout -k 10 300 python3 bench.py --config CHAIN --steps 20 \
        --warmup 5 --per-launch --no-cpu-baseline --no-ceiling "$@" >> "$out/$n.json" 2>> "$out/$n.err"; }
  for pass in 1 2; do
    b CHAIN_rot3;  b CHAIN_rot1 --rotate 1;  b CHAINF_rot3 --chain-fill
  done
  ;;
hdrt)  # ring slots' header blocks read 8 lanes per frame (lib_hdrt) against per-lane loads
  AIPSTACK_AMD_LIB=tools/build/lib_hdrt.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -v \
      --timeout 120 --timeout-method thread -k "slotted or frame" > "$out/pytest.log" 2>&1
  b() { n=$1; shift; env "$@" timeout -k 10 300 python3 bench.py --config ${n%%_*} --steps 20 \
        --warmup 5 --per-launch --no-cpu-baseline --no-ceiling >> "$out/$n.json" 2>> "$out/$n.err"; }
  for pass in 1 2 3; do
    for c in RX2K TX2K; do
      b ${c}_def X=0;  b ${c}_hdrt AIPSTACK_AMD_LIB=tools/build/lib_hdrt.so
    done
  done
  ;;
final_bench)  # every config under the driver's protocol (A first, as the box's first GPU
              # process), the ceiling probe, the slot-read probes (RX2K / C2K lines)
  for c in A B C A2K C2K CHAIN RX RX2K TXREC TX TX2K; do
    bench bench_$c --config $c --steps 20 --warmup 5 --per-launch
  done
  timeout -k 10 120 tools/build/hbm_peak ceiling > "$out/ceiling.jsonl"
  timeout -k 10 120 tools/build/hbm_peak > "$out/hbm_peak.jsonl"
  ;;
final_bench2)  # the same set again on another box (the spread between boxes)
  for c in A B C A2K C2K CHAIN RX RX2K TXREC TX TX2K; do
    bench bench_$c --config $c --steps 20 --warmup 5 --per-launch --no-ceiling
  done
  ;;
final_prof)  # rocprofv3 --kernel-trace --stats of each config's driver-protocol command
  for c in A B C A2K C2K CHAIN RX RX2K TXREC TX TX2K; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_$c" -o run \
        -- python3 bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-ceiling \
        > "$out/prof_$c.log" 2>&1
  done
  ;;
final_pmc)  # PMC passes for every config on this device code (tools/pmc_summary.py after)
  for c in A B C A2K C2K CHAIN RX RX2K TXREC TX TX2K; do tools/pmc_run.sh $c "$out/pmc_$c"; done
  ;;
final_pmc_frames)  # PMC of the frame and ring-slot configs, rotated as bench.py now runs them
  for c in C2K RX RX2K TXREC TX TX2K; do tools/pmc_run.sh $c "$out/pmc_$c"; done
  ;;
final_chain)  # CHAIN's final line and rocprof with its batch rotated
  bench bench_CHAIN --config CHAIN --steps 20 --warmup 5 --per-launch
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_CHAIN" -o run \
      -- python3 bench.py --config CHAIN --steps 20 --warmup 5 --no-cpu-baseline --no-ceiling \
      > "$out/prof_CHAIN.log" 2>&1
  ;;
final_misc)  # small batches, end to end, the 8-rank launch rehearsed on one GPU
  for n in 64 4096; do
    for c in A RX TX; do
      timeout -k 10 120 python3 bench.py --config $c --small $n >> "$out/small.jsonl" 2>> "$out/small.err"
    done
  done
  for c in A C RX TX C2K; do
    timeout -k 10 300 python3 bench.py --e2e --config $c --steps 5 --warmup 1 >> "$out/e2e.jsonl" 2>> "$out/e2e.err"
  done
  AIPSTACK_BENCH_FORCE_DEVICE=0 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 \
      --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 8 \
      --steps 20 --warmup 5 --cpu-reps 3 > "$out/bench8_A.json" 2> "$out/bench8_A.err"
  ;;
final_test)  # the round-end gate on this tree
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
      > "$out/pytest_gpu.log" 2>&1
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1
  ;;
*)
  echo "unknown mode $mode"; exit 2 ;;
esac
echo "r05 $mode done"
