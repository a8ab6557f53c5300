#!/bin/bash
# Round-4 GPU experiments, one mode per gpurun call; output under gpurun_out/r04/<mode>.
#   txsect  the Tx fill forms (2-byte vs whole-sector field stores, split slotted fill):
#           their GPU tests, then tools/tx_sweep.py on TX2K and TX, interleaved
#   kern    chained batches with short chunks first (chain_short 0 vs 128): GPU tests,
#           alternating CHAIN bench lines, FETCH_SIZE / VALU per variant; C2K launch shapes
#   engine  the engine's host path (pool, locking) and the async engine group: their GPU
#           tests, the fault program, e2e RX / TX with host-time stats, ring_loop latency
#           (engine vs group of 2) and the descriptor-driven loop (-s)
set -e
mode=${1:?mode}
out=gpurun_out/r04/$mode
mkdir -p "$out"
export TMPDIR=/tmp

pyt() {  # pyt NAME PYTEST-ARGS... -> $out/NAME.log
  name=$1; shift
  timeout -k 10 900 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread "$@" \
      > "$out/$name.log" 2>&1
}
sweep() {  # sweep NAME ARGS... -> $out/NAME.jsonl (appended)
  name=$1; shift
  timeout -k 10 300 python tools/tx_sweep.py "$@" >> "$out/$name.jsonl" 2>> "$out/$name.err"
}

engine_e2e() {
  export AIPSTACK_ENGINE_STATS=1
  for c in RX TX; do
    for i in 1 2; do
      timeout -k 10 300 python bench.py --e2e --config $c --steps 5 --warmup 1 \
          >> "$out/e2e_$c.jsonl" 2>> "$out/e2e_$c.err"
    done
  done
  unset AIPSTACK_ENGINE_STATS
  timeout -k 10 300 python bench.py --e2e --config TX --e2e-pageable --steps 3 --warmup 1 \
      >> "$out/e2e_TX_pageable.jsonl" 2>> "$out/e2e_TX_pageable.err"
  # the group's engines all on the box's one device
  AIPSTACK_BENCH_FORCE_DEVICE=0 timeout -k 10 300 python bench.py --e2e --engines 2 --config C \
      --steps 3 --warmup 1 >> "$out/e2e_group2_C.jsonl" 2>> "$out/e2e_group2_C.err"
  AIPSTACK_BENCH_FORCE_DEVICE=0 timeout -k 10 300 python bench.py --e2e --engines 2 --config C \
      --e2e-pageable --steps 3 --warmup 1 >> "$out/e2e_group2_C_pageable.jsonl" \
      2>> "$out/e2e_group2_C_pageable.err"
}

engine_loops() {
  for i in 1 2; do
    timeout -k 10 120 tools/build/ring_loop -r 1 64 256 >> "$out/lat_engine.jsonl"
    timeout -k 10 120 tools/build/ring_loop -g 2 -r 1 64 256 >> "$out/lat_group2.jsonl"
    timeout -k 10 120 tools/build/ring_loop -r 8 64 1024 4096 >> "$out/loop_engine.jsonl"
    timeout -k 10 120 tools/build/ring_loop -g 2 -r 8 64 1024 4096 >> "$out/loop_group2.jsonl"
  done
  timeout -k 10 200 tools/build/ring_loop -s -r 8 64 256 1024 4096 >> "$out/socket_engine.jsonl"
  timeout -k 10 200 tools/build/ring_loop -s -r 1 64 >> "$out/socket_engine_r1.jsonl"
  timeout -k 10 200 tools/build/ring_loop -s -g 2 -r 8 64 1024 >> "$out/socket_group2.jsonl"
}

bench() {  # bench NAME ARGS... -> $out/NAME.jsonl (appended)
  name=$1; shift
  timeout -k 10 300 python bench.py "$@" >> "$out/$name.jsonl" 2>> "$out/$name.err"
}
pmc1() {  # pmc1 NAME CONFIG COUNTERS...: one PMC pass of a bench config (env passes through)
  name=$1; cfg=$2; shift 2
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$out/pmc_$name" -o run \
      --pmc "$@" -- python3 bench.py --config "$cfg" --no-cpu-baseline --no-parity \
      --steps 5 --warmup 2 > "$out/pmc_$name.log" 2>&1
}

case $mode in
calib)  # FETCH_SIZE by access width (tools/width_calib.hip), 3 dispatches per kernel;
        # CHAIN at 4 stream windows (no spill since round 4) against the default 2
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$out/width" -o run \
      --pmc FETCH_SIZE -- tools/build/width_calib > "$out/width.log" 2>&1
  for i in 1 2 3; do
    bench chain_su2 --config CHAIN --per-launch --no-cpu-baseline
    AIPSTACK_CHKSUM_STREAM=4 bench chain_su4 --config CHAIN --per-launch --no-cpu-baseline
  done
  sweep tx2k_frames --config TX2K --variants "frames=4;frames=2;frames=8;frames=4,split=1;frames=8,split=1"
  ;;
chain)  # CHAIN at its round-4 defaults (4 stream windows, group-bounded table reads): tests,
        # bench lines, rocprof stats, PMC; tools/chain_probe.py's layouts under FETCH_SIZE
  pyt pytest_chain -m gpu -k "chain or native_library"
  for i in 1 2; do bench chain --config CHAIN --per-launch; done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_CHAIN" -o run \
      -- python3 bench.py --config CHAIN --no-cpu-baseline --no-parity > "$out/prof_CHAIN.log" 2>&1
  tools/pmc_run.sh CHAIN "$out/pmc_CHAIN"
  ;&
probe)  # tools/chain_probe.py's layouts under FETCH_SIZE, then timed, per launch variant
        # (VARIANTS: space-separated, each a comma-separated list of AIPSTACK_CHKSUM_ settings)
  for v in ${VARIANTS:-base CHAIN_SHORT=128}; do
    name=${v//=/}; name=${name//,/_}
    (
      if [ "$v" != base ]; then
        for kv in ${v//,/ }; do export "AIPSTACK_CHKSUM_$kv"; done
      fi
      timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$out/probe_$name" -o run \
          --pmc FETCH_SIZE -- python3 tools/chain_probe.py > "$out/probe_$name.jsonl" \
          2> "$out/probe_$name.err"
      python3 tools/chain_probe.py --summarize "$out/probe_$name/run_counter_collection.csv" \
          "$out/probe_$name.jsonl" > "$out/probe_${name}_fetch.jsonl"
      timeout -k 10 240 python3 tools/chain_probe.py --reps 30 > "$out/probe_${name}_timing.jsonl" \
          2>> "$out/probe_$name.err"
    )
  done
  ;;
short)  # neighbour-aware short chunks first in chained batches: GPU tests, CHAIN A/B, the probe
  pyt pytest_short -m gpu -k "chain or native_library"
  for i in 1 2 3; do
    bench chain_table --config CHAIN --per-launch --no-cpu-baseline
    AIPSTACK_CHKSUM_CHAIN_SHORT=128 bench chain_short128 --config CHAIN --per-launch --no-cpu-baseline
    AIPSTACK_CHKSUM_CHAIN_SHORT=32 bench chain_short32 --config CHAIN --per-launch --no-cpu-baseline
  done
  VARIANTS="base CHAIN_SHORT=128 CHAIN_SHORT=32" "$0" probe
  ;;
skip)  # gathered streams skip the scans of windows past the stream: tests, A/B vs the
        # previous library (tools/build/lib_noskip.so), VALU per variant
  pyt pytest_skip -m gpu -k "chain or slotted or native_library"
  for i in 1 2 3; do
    for c in C2K CHAIN; do
      AIPSTACK_AMD_LIB=tools/build/lib_noskip.so bench ${c}_noskip --config $c --per-launch --no-cpu-baseline
      bench ${c}_skip --config $c --per-launch --no-cpu-baseline
    done
  done
  for c in C2K CHAIN; do
    AIPSTACK_AMD_LIB=tools/build/lib_noskip.so pmc1 ${c}_noskip_sq $c SQ_INSTS_VALU SQ_INSTS_SALU
    pmc1 ${c}_skip_sq $c SQ_INSTS_VALU SQ_INSTS_SALU
  done
  ;;
edge)  # gathered streams: AIPSTACK_GATHER_MODE 2 (edge segments copied from the stream,
        # the product) against 0 (per-segment masks, tools/build/lib_masked.so) and 1 (edge
        # segments re-read, tools/build/lib_edgeload.so): tests, A/B, VALU and FETCH
  pyt pytest_edge -m gpu -k "chain or slotted or native_library or random"
  for i in 1 2 3; do
    for c in C2K CHAIN; do
      AIPSTACK_AMD_LIB=tools/build/lib_masked.so bench ${c}_masked --config $c --per-launch --no-cpu-baseline
      AIPSTACK_AMD_LIB=tools/build/lib_edgeload.so bench ${c}_edgeload --config $c --per-launch --no-cpu-baseline
      bench ${c}_edge --config $c --per-launch --no-cpu-baseline
    done
  done
  for c in C2K CHAIN; do
    pmc1 ${c}_edge_sq $c SQ_INSTS_VALU SQ_INSTS_SALU
    pmc1 ${c}_edge_fetch $c FETCH_SIZE
  done
  ;;
shape)  # launch shapes again after the edge form (fewer VGPRs): full GPU suite, C2K shapes,
         # CHAIN at 2 / 4 windows
  pyt pytest_all -m gpu
  timeout -k 10 300 python tools/slot_sweep.py --config C2K --rounds 6 --variants \
      "chunk_packets=16;stream=8,chunk_packets=16;stream=2,chunk_packets=16;chunk_packets=32;stream=8,chunk_packets=32;chunk_packets=8;stream=8,chunk_packets=8" \
      > "$out/c2k_sweep.jsonl" 2> "$out/c2k_sweep.err"
  for i in 1 2 3; do
    bench chain_su4 --config CHAIN --per-launch --no-cpu-baseline
    AIPSTACK_CHKSUM_STREAM=2 bench chain_su2 --config CHAIN --per-launch --no-cpu-baseline
    # edge loads only where a chunk has foreign bytes (product) vs always (lib_edgeall.so)
    AIPSTACK_AMD_LIB=tools/build/lib_edgeall.so bench chain_edgeall --config CHAIN --per-launch --no-cpu-baseline
    AIPSTACK_AMD_LIB=tools/build/lib_edgeall.so bench c2k_edgeall --config C2K --per-launch --no-cpu-baseline
    bench c2k --config C2K --per-launch --no-cpu-baseline
  done
  pmc1 chain_fetch CHAIN FETCH_SIZE
  ;;
shape2)  # slot chunk sizes for C2K and A2K after the conditional edge loads; CHAIN chains per group
  timeout -k 10 300 python tools/slot_sweep.py --config C2K --rounds 6 --variants \
      "chunk_packets=8;chunk_packets=4;stream=2,chunk_packets=8;chunk_packets=16;stream=2,chunk_packets=4;stream=8,chunk_packets=4" \
      > "$out/c2k_sweep.jsonl" 2> "$out/c2k_sweep.err"
  timeout -k 10 300 python tools/slot_sweep.py --config A2K --rounds 6 --variants \
      "chunk_packets=16;chunk_packets=8;chunk_packets=4;stream=2,chunk_packets=8;stream=8,chunk_packets=8" \
      > "$out/a2k_sweep.jsonl" 2> "$out/a2k_sweep.err"
  for i in 1 2 3; do
    bench chain_g64 --config CHAIN --per-launch --no-cpu-baseline
    AIPSTACK_CHKSUM_CHUNK_PACKETS=32 bench chain_g32 --config CHAIN --per-launch --no-cpu-baseline
    AIPSTACK_CHKSUM_CHUNK_PACKETS=16 bench chain_g16 --config CHAIN --per-launch --no-cpu-baseline
  done
  ;;
gatherA)  # back-to-back strided batches (A, B) through the gathered stream, chunk sizes
  for i in 1 2 3; do
    bench A_stream --config A --per-launch --no-cpu-baseline
    AIPSTACK_CHKSUM_GATHER=1 bench A_g8 --config A --per-launch --no-cpu-baseline
    AIPSTACK_CHKSUM_GATHER=1 AIPSTACK_CHKSUM_CHUNK_PACKETS=16 bench A_g16 --config A --per-launch --no-cpu-baseline
    AIPSTACK_CHKSUM_GATHER=1 AIPSTACK_CHKSUM_CHUNK_PACKETS=4 bench A_g4 --config A --per-launch --no-cpu-baseline
    bench B_stream --config B --per-launch --no-cpu-baseline
    AIPSTACK_CHKSUM_GATHER=1 bench B_g8 --config B --per-launch --no-cpu-baseline
    AIPSTACK_CHKSUM_GATHER=1 AIPSTACK_CHKSUM_CHUNK_PACKETS=2 bench B_g2 --config B --per-launch --no-cpu-baseline
  done
  ;;
gather2)  # the gathered stream as the default for strided and CSR checksum batches: the GPU
          # suite, then A / B / C against stream mode (gather = -1), small batches
  pyt pytest_all -m gpu
  for i in 1 2 3; do
    for c in A B C; do
      AIPSTACK_CHKSUM_GATHER=-1 bench ${c}_stream --config $c --per-launch --no-cpu-baseline
      bench ${c}_gather --config $c --per-launch --no-cpu-baseline
    done
  done
  for n in 1024 4096 16384; do
    AIPSTACK_CHKSUM_GATHER=-1 timeout -k 10 120 python bench.py --config A --small $n >> "$out/small_stream.jsonl" 2>> "$out/small.err"
    timeout -k 10 120 python bench.py --config A --small $n >> "$out/small_gather.jsonl" 2>> "$out/small.err"
  done
  pmc1 A_fetch A FETCH_SIZE
  pmc1 C_fetch C FETCH_SIZE
  ;;
chunks)  # chunk sizes: stream mode for A (what made the gathered form faster?), frames for RX / TX
  for i in 1 2; do
    for k in 64 32 16 8; do
      AIPSTACK_CHKSUM_GATHER=-1 AIPSTACK_CHKSUM_CHUNK_PACKETS=$k bench A_stream_$k --config A --per-launch --no-cpu-baseline
    done
    for k in 64 32 16; do
      AIPSTACK_CHKSUM_CHUNK_PACKETS=$k bench RX_$k --config RX --per-launch --no-cpu-baseline
      AIPSTACK_CHKSUM_CHUNK_PACKETS=$k bench TX_$k --config TX --per-launch --no-cpu-baseline
    done
    for k in 16 8 32; do
      AIPSTACK_CHKSUM_CHUNK_PACKETS=$k bench C_g$k --config C --per-launch --no-cpu-baseline
    done
  done
  ;;
e2eh)  # the engine's zero-copy strided / CSR pieces back in stream mode: engine tests, e2e A / C
  pyt pytest_engine -m gpu -k "engine or group or slotted or chain or ring_loop"
  for c in ${E2E_CONFIGS:-A C C2K}; do
    timeout -k 10 300 python bench.py --e2e --config $c --steps 5 --warmup 1 >> "$out/e2e.jsonl" 2>> "$out/e2e.err"
  done
  ;;
fdb)  # double-buffered stream mode (tools/build/lib_fdb.so: frames' captured stream and the
      # batches' stream mode issue the next group before summing the current one)
  for i in 1 2 3; do
    for c in RX TX TXREC; do
      bench ${c}_base --config $c --per-launch --no-cpu-baseline
      AIPSTACK_AMD_LIB=tools/build/lib_fdb.so bench ${c}_db8 --config $c --per-launch --no-cpu-baseline
      AIPSTACK_AMD_LIB=tools/build/lib_fdb.so AIPSTACK_CHKSUM_STREAM=4 bench ${c}_db4 --config $c --per-launch --no-cpu-baseline
    done
    AIPSTACK_CHKSUM_GATHER=-1 bench A_stream --config A --per-launch --no-cpu-baseline
    AIPSTACK_AMD_LIB=tools/build/lib_fdb.so AIPSTACK_CHKSUM_GATHER=-1 bench A_streamdb --config A --per-launch --no-cpu-baseline
  done
  AIPSTACK_AMD_LIB=tools/build/lib_fdb.so timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 \
      --timeout-method thread -m gpu -k "rx_verify or tx_fill or frames or random" > "$out/pytest_fdb.log" 2>&1
  ;;
slotg)  # ring-slot frames: the L4 bytes past the header blocks as one gathered stream (product)
        # vs one frame per wave instruction pair (tools/build/lib_noslot.so)
  pyt pytest_slotg -m gpu -k "slotted or frames or rx_verify or tx_fill or random or engine"
  for i in 1 2 3; do
    for c in RX2K TX2K; do
      AIPSTACK_AMD_LIB=tools/build/lib_noslot.so bench ${c}_wave --config $c --per-launch --no-cpu-baseline
      bench ${c}_gather --config $c --per-launch --no-cpu-baseline
    done
  done
  for i in 1 2; do
    sweep tx2k --config TX2K --variants "split=0;split=1;split=0,frames=4"
  done
  ;;
slotg2)  # slotted frames' chunk size with the gathered L4 stream
  timeout -k 10 300 python tools/slot_sweep.py --config RX2K --rounds 6 --variants \
      "chunk_packets=32;chunk_packets=16;chunk_packets=64;chunk_packets=8" > "$out/rx2k_sweep.jsonl" 2> "$out/rx2k_sweep.err"
  sweep tx2k --config TX2K --variants "split=0,chunk_packets=32;split=0,chunk_packets=16;split=0,chunk_packets=64;split=0,chunk_packets=8"
  ;;
su8)  # the gathered stream at 8 windows per group (SU = 8) against 4
  for i in 1 2 3; do
    for c in A C C2K; do
      bench ${c}_su4 --config $c --per-launch --no-cpu-baseline
      AIPSTACK_CHKSUM_STREAM=8 bench ${c}_su8 --config $c --per-launch --no-cpu-baseline
    done
  done
  ;;
su8b)  # A2K and B at 8 windows (the new default for fixed lengths >= 1 KiB) against 4
  for i in 1 2 3; do
    for c in A2K B A; do
      bench ${c}_su8 --config $c --per-launch --no-cpu-baseline
      AIPSTACK_CHKSUM_STREAM=4 bench ${c}_su4 --config $c --per-launch --no-cpu-baseline
    done
  done
  ;;
chain8)  # chains at 8 windows per group against 4
  pyt pytest_chain8 -m gpu -k "chain_bench_shape or chain_golden"
  for i in 1 2 3; do
    bench chain_su4 --config CHAIN --per-launch --no-cpu-baseline
    AIPSTACK_CHKSUM_STREAM=8 bench chain_su8 --config CHAIN --per-launch --no-cpu-baseline
  done
  ;;
kern)
  pyt pytest_kern -m gpu -k "chain or contract_violations or native_library"
  for i in 1 2 3; do
    AIPSTACK_CHKSUM_CHAIN_SHORT=0 bench chain_table --config CHAIN --per-launch --no-cpu-baseline
    bench chain_short --config CHAIN --per-launch --no-cpu-baseline
  done
  AIPSTACK_CHKSUM_CHAIN_SHORT=0 pmc1 chain_table_fetch CHAIN FETCH_SIZE
  pmc1 chain_short_fetch CHAIN FETCH_SIZE
  AIPSTACK_CHKSUM_CHAIN_SHORT=0 pmc1 chain_table_sq CHAIN SQ_INSTS_VALU SQ_INSTS_SALU
  pmc1 chain_short_sq CHAIN SQ_INSTS_VALU SQ_INSTS_SALU
  timeout -k 10 300 python tools/slot_sweep.py --config C2K --rounds 6 --variants \
      "chunk_packets=16;stream=2,chunk_packets=16;stream=8,chunk_packets=16;chunk_packets=32;stream=2,chunk_packets=32;stream=8,chunk_packets=32;chunk_packets=8" \
      > "$out/c2k_sweep.jsonl" 2> "$out/c2k_sweep.err"
  pmc1 c2k_sq C2K SQ_INSTS_VALU SQ_INSTS_SALU
  AIPSTACK_CHKSUM_CHUNK_PACKETS=32 pmc1 c2k_32_sq C2K SQ_INSTS_VALU SQ_INSTS_SALU
  ;;
txsect)
  pyt pytest_tx -m gpu -k "tx_fill or slotted or random_frames"
  for i in 1 2; do
    sweep tx2k --config TX2K --variants "split=0,store=0;split=0,store=1;split=1,store=0"
    sweep tx --config TX --variants "split=1;split=0,store=0;split=0,store=1;split=0,store=1,gather=2;split=1,gather=1"
  done
  ;;
engine)
  pyt pytest_engine -m gpu -k "engine or ring_loop or group"
  engine_e2e
  engine_loops
  ;;
engine2)  # the engine mode's measurements after its tests
  engine_e2e
  engine_loops
  ;;
*)
  echo "unknown mode $mode" >&2; exit 2 ;;
esac
