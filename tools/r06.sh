#!/bin/bash
# Round-6 GPU experiments, one mode per gpurun call; output under gpurun_out/r06/<mode>.
#   fresh   tools/fresh.py: the first read of a freshly written batch, by writer, reader,
#           granularity and age; plus the counters this box's rocprofv3 offers
set -e
mode=${1:?mode}
out=gpurun_out/r06/$mode
mkdir -p "$out"
export TMPDIR=/tmp

case $mode in
fresh)
  (timeout -k 10 60 rocprofv3 -L > "$out/avail.txt" 2>&1 || true)
  timeout -k 10 600 python3 -u tools/fresh.py > "$out/fresh.jsonl" 2> "$out/fresh.err"
  ;;
fresh2)  # which reader pays (pure-read modes, the checksum, the edge loads nontemporal), and
         # per-dispatch counters of the driver's command: launches 1-3 (each batch's first
         # read) against 4-25
  timeout -k 10 300 python3 -u tools/fresh.py readers base fresh_kcopy > "$out/readers.jsonl" 2> "$out/readers.err"
  AIPSTACK_AMD_LIB=$PWD/tools/build/lib_edgent.so timeout -k 10 300 python3 -u tools/fresh.py \
      readers base fresh_kcopy > "$out/readers_edgent.jsonl" 2> "$out/readers_edgent.err"
  pmc() {  # pmc NAME COUNTERS...
    name=$1; shift
    timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d "$out/pmc_$name" -o run \
        --pmc "$@" -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ceiling \
        --no-parity > "$out/pmc_$name.log" 2>&1
  }
  pmc fetch FETCH_SIZE
  pmc ea TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum
  pmc probe TCC_PROBE_sum TCC_PROBE_ALL_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum
  pmc tcp TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum
  pmc sq SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE
  ;;
col6)  # round-6 column runs (partial segments from the stream) against round 5's edge loads:
       # parity of the forms, fresh-data and steady-state reads, the driver's command
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
      -k "every_read_form or short_runs or full_size or config_d or ragged or lengths or empty_chunks or all_zero" \
      > "$out/pytest.log" 2>&1
  for lib in product coledge product coledge; do
    if [ $lib = product ]; then L=$PWD/aipstack_amd/lib/libaipstack_chksum.so; else L=$PWD/tools/build/lib_$lib.so; fi
    AIPSTACK_AMD_LIB=$L timeout -k 10 300 python3 -u tools/fresh.py base fresh_synth fresh_d2d \
        fresh_kcopy fresh_h2d steady >> "$out/fresh_$lib.jsonl" 2>> "$out/fresh_$lib.err"
    AIPSTACK_AMD_LIB=$L timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 \
        --per-launch --no-cpu-baseline --no-ceiling >> "$out/bench_$lib.json" 2>> "$out/bench_$lib.err"
  done
  ;;
col6b)  # the same after the window prefixes were shared with the partial segments; occupancy
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
      -k "every_read_form or short_runs or full_size or config_d or ragged or lengths or empty_chunks or all_zero" \
      > "$out/pytest.log" 2>&1
  timeout -k 10 300 python3 -u tools/fresh.py base fresh_synth fresh_d2d fresh_kcopy fresh_h2d steady \
      > "$out/fresh.jsonl" 2> "$out/fresh.err"
  timeout -k 10 300 python3 tools/ab.py --config A --variants \
      "gather=1;gather=1,lds_pad=20000;gather=1,lds_pad=30000" > "$out/ab_A.jsonl" 2> "$out/ab_A.err"
  for i in 1 2; do
    timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --per-launch --no-cpu-baseline \
        --no-ceiling >> "$out/bench_A.json" 2>> "$out/bench.err"
  done
  timeout -k 10 300 python3 bench.py --config B --steps 20 --warmup 5 --per-launch --no-cpu-baseline \
      --no-ceiling >> "$out/bench_B.json" 2>> "$out/bench.err"
  ;;
col6c)  # column runs capturing the boundary segments from the stream (AIPSTACK_COL_PARTIAL 0)
        # against round 5's edge loads (lib_colp1), alternating processes
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
      -k "every_read_form or short_runs or full_size or config_d or ragged or lengths or empty_chunks or all_zero" \
      > "$out/pytest.log" 2>&1
  timeout -k 10 300 python3 tools/ab.py --config A --variants \
      "gather=1;gather=1,lds_pad=20000" > "$out/ab_A.jsonl" 2> "$out/ab_A.err"
  for lib in product colp1 product colp1; do
    if [ $lib = product ]; then L=$PWD/aipstack_amd/lib/libaipstack_chksum.so; else L=$PWD/tools/build/lib_$lib.so; fi
    AIPSTACK_AMD_LIB=$L timeout -k 10 300 python3 -u tools/fresh.py base fresh_synth fresh_d2d \
        fresh_h2d steady >> "$out/fresh_$lib.jsonl" 2>> "$out/fresh_$lib.err"
    AIPSTACK_AMD_LIB=$L timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 \
        --per-launch --no-cpu-baseline --no-ceiling >> "$out/bench_$lib.json" 2>> "$out/bench_$lib.err"
  done
  timeout -k 10 300 python3 bench.py --config B --steps 20 --warmup 5 --per-launch --no-cpu-baseline \
      --no-ceiling >> "$out/bench_B.json" 2>> "$out/bench.err"
  ;;
pf6)  # column runs: capture (product) / round-5 edge loads (colp1) / capture + scalar touches of
      # the boundary lines (spf) / capture + default-policy vector touches after group 0 (vpf)
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
      -k "every_read_form or short_runs or full_size" > "$out/pytest.log" 2>&1
  for r in 1 2; do
    for lib in ${LIBS:-product spf vpf}; do
      if [ $lib = product ]; then L=$PWD/aipstack_amd/lib/libaipstack_chksum.so; else L=$PWD/tools/build/lib_$lib.so; fi
      AIPSTACK_AMD_LIB=$L timeout -k 10 300 python3 -u tools/fresh.py fresh_synth fresh_d2d steady \
          >> "$out/fresh_$lib.jsonl" 2>> "$out/fresh_$lib.err"
      AIPSTACK_AMD_LIB=$L timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 \
          --per-launch --no-cpu-baseline --no-ceiling >> "$out/bench_$lib.json" 2>> "$out/bench_$lib.err"
    done
  done
  ;;
pmc6)  # per-dispatch counters, column runs with and without the round-5 edge loads
  pmc() {  # pmc LIB NAME COUNTERS...
    lib=$1; name=$2; shift 2
    if [ $lib = product ]; then L=$PWD/aipstack_amd/lib/libaipstack_chksum.so; else L=$PWD/tools/build/lib_$lib.so; fi
    AIPSTACK_AMD_LIB=$L timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv \
        -d "$out/${lib}_$name" -o run --pmc "$@" -- python3 bench.py --steps 20 --warmup 5 \
        --no-cpu-baseline --no-ceiling --no-parity > "$out/${lib}_$name.log" 2>&1
  }
  for lib in ${LIBS:-product colp1}; do
    pmc $lib fetch FETCH_SIZE
    pmc $lib ea TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_HIT_sum TCC_MISS_sum
    pmc $lib req TCC_REQ_sum TCC_STREAMING_REQ_sum TCC_READ_sum TCC_EA0_RDREQ_DRAM_sum
    pmc $lib sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE
    pmc $lib tcp TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_NC_READ_REQ_sum
  done
  ;;
abp0)  # shapes of the capture form (product) at steady state, interleaved in one process
  timeout -k 10 120 tests/cpp/build/engine_fault_test > "$out/engine_fault.log" 2>&1
  timeout -k 10 300 tests/cpp/build/engine_fault_test_asan > "$out/engine_fault_asan.log" 2>&1
  timeout -k 10 400 python3 tools/ab.py --config A --variants \
      "gather=1;gather=1,chunk_packets=16;gather=1,chunk_packets=4;gather=1,lds_pad=30000;gather=1,short_loads=0;gather=0" \
      > "$out/ab_A.jsonl" 2> "$out/ab_A.err"
  AIPSTACK_AMD_LIB=$PWD/tools/build/lib_colp1.so timeout -k 10 400 python3 tools/ab.py --config A --variants \
      "gather=1;gather=1,chunk_packets=16;gather=1,lds_pad=30000" > "$out/ab_A_colp1.jsonl" 2> "$out/ab_A_colp1.err"
  ;;
fresh6)  # fresh-data lines per writer (with and without the JUST_WRITTEN hint) for A, C, A2K,
         # CHAIN, RX; Tx fill ceiling; the driver's command; then the GPU suite
  b() {  # b NAME ARGS...
    name=$1; shift
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ceiling "$@" \
        >> "$out/$name.json" 2>> "$out/$name.err"
  }
  b driver_A --gpus 1 --per-launch
  timeout -k 10 300 python3 -u tools/tx_ceiling.py > "$out/tx_ceiling.jsonl" 2> "$out/tx_ceiling.err"
  AIPSTACK_AMD_LIB=$PWD/tools/build/lib_txnt.so timeout -k 10 300 python3 -u tools/tx_ceiling.py \
      > "$out/tx_ceiling_txnt.jsonl" 2> "$out/tx_ceiling_txnt.err"
  # in-place Tx fills: field stores plain / nontemporal (lib_txnt), field-line touches on / off
  for i in 1 2; do
    b tx_plain --config TX --per-launch
    AIPSTACK_CHKSUM_TX_GATHER=1 b tx_plain_notouch --config TX --per-launch
    AIPSTACK_AMD_LIB=$PWD/tools/build/lib_txnt.so b tx_nt --config TX --per-launch
    AIPSTACK_AMD_LIB=$PWD/tools/build/lib_txnt.so AIPSTACK_CHKSUM_TX_GATHER=1 b tx_nt_notouch --config TX --per-launch
    b tx2k_plain --config TX2K --per-launch
    AIPSTACK_AMD_LIB=$PWD/tools/build/lib_txnt.so b tx2k_nt --config TX2K --per-launch
  done
  for w in dma nt plain d2d; do
    b fresh_A --fresh $w
    b fresh_A --fresh $w --just-written
  done
  for cfg in C A2K CHAIN RX B; do
    for w in dma plain; do b fresh_$cfg --config $cfg --fresh $w; done
  done
  b driver_A --gpus 1 --per-launch
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
      > "$out/pytest_gpu.log" 2>&1
  ;;
check6)  # NT-written synthetic batches and DMA-written copies: the driver's command, its rocprof
         # average over all 25 launches, the Tx lines with their fill ceiling
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
      -k "synth or full_size or header_capture or tx_fill_matches or rx_verify_matches or chain_many" \
      > "$out/pytest.log" 2>&1
  b() {  # b NAME ARGS...
    name=$1; shift
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 "$@" >> "$out/$name.json" 2>> "$out/$name.err"
  }
  b A --gpus 1 --per-launch
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/rocprof_A" -o run \
      -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$out/rocprof_A.log" 2>&1
  for cfg in TX TX2K C CHAIN RX; do b $cfg --config $cfg --per-launch --no-cpu-baseline; done
  b A --gpus 1 --per-launch --no-cpu-baseline
  ;;
txrec6)  # the records pass against Rx verify on the same frames: times, the records' price
         # (lib_norec: no record stores, wrong output), counters
  b() {  # b NAME ARGS...
    name=$1; shift
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" >> "$out/$name.json" 2>> "$out/$name.err"
  }
  for i in 1 2; do
    b RX --config RX --per-launch
    b TXREC --config TXREC --per-launch
    AIPSTACK_AMD_LIB=$PWD/tools/build/lib_norec.so b TXREC_norec --config TXREC --per-launch --no-parity
  done
  pmc() {  # pmc CFG NAME COUNTERS...
    cfg=$1; name=$2; shift 2
    timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d "$out/${cfg}_$name" -o run \
        --pmc "$@" -- python3 bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline \
        --no-parity > "$out/${cfg}_$name.log" 2>&1
  }
  for cfg in RX TXREC; do
    pmc $cfg sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES
    pmc $cfg sq2 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS
    pmc $cfg tcc FETCH_SIZE TCC_EA0_WRREQ_sum
  done
  ;;
rank8)  # the multi-rank flow rehearsed on this one GPU (every rank on device 0): the solo phase
        # and scaling_efficiency; the records pass with its ceiling; the Tx probe sweep
  for N in 2 8; do
    AIPSTACK_BENCH_FORCE_DEVICE=0 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 \
        --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29600 + N)) bench.py \
        --gpus $N --steps 20 --warmup 5 --no-cpu-baseline --no-ceiling > "$out/bench${N}_A.json" \
        2> "$out/bench${N}_A.err"
  done
  timeout -k 10 300 python3 bench.py --config TXREC --steps 20 --warmup 5 --no-cpu-baseline \
      --per-launch > "$out/TXREC.json" 2> "$out/TXREC.err"
  timeout -k 10 300 python3 -u tools/tx_ceiling.py TX > "$out/tx_ceiling.jsonl" 2> "$out/tx_ceiling.err"
  ;;
recnt)  # the records pass with nontemporal record stores (lib_recnt) against ordinary ones
  b() {  # b NAME ARGS...
    name=$1; shift
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" >> "$out/$name.json" 2>> "$out/$name.err"
  }
  for i in 1 2 3; do
    b TXREC --config TXREC --per-launch --no-ceiling
    AIPSTACK_AMD_LIB=$PWD/tools/build/lib_recnt.so b TXREC_nt --config TXREC --per-launch --no-ceiling
  done
  ;;
chain6)  # chain runs (long chunks back to back as one stream-prefix run, short ones per lane)
         # against the gathered stream (lib_chain0): the chain tests, then alternating benches
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
      -k "chain" > "$out/pytest.log" 2>&1
  b() {  # b NAME ARGS...
    name=$1; shift
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" >> "$out/$name.json" 2>> "$out/$name.err"
  }
  for i in 1 2; do
    b CHAIN --config CHAIN --per-launch
    AIPSTACK_AMD_LIB=$PWD/tools/build/lib_chain0.so b CHAIN0 --config CHAIN --per-launch
  done
  b CHAINFILL --config CHAIN --chain-fill
  AIPSTACK_AMD_LIB=$PWD/tools/build/lib_chain0.so b CHAINFILL0 --config CHAIN --chain-fill
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d "$out/pmc_CHAIN" -o run \
      --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES -- python3 bench.py --config CHAIN \
      --steps 20 --warmup 5 --no-cpu-baseline --no-parity > "$out/pmc_CHAIN.log" 2>&1
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d "$out/fetch_CHAIN" -o run \
      --pmc FETCH_SIZE -- python3 bench.py --config CHAIN --steps 20 --warmup 5 --no-cpu-baseline \
      --no-parity > "$out/fetch_CHAIN.log" 2>&1
  ;;
ccols)  # chain column runs (lib_chaincols: run chunks as column runs of <= 32, lib_chaincols16:
        # <= 16; lone short ones per lane) against the gathered stream (product): the chain tests
        # on the variants, then alternating benches, the chain fill, fresh plain-written data
  for v in ${VARS:-chaincols chaincols16}; do
    AIPSTACK_AMD_LIB=$PWD/tools/build/lib_$v.so timeout -k 10 600 python -u -m pytest tests \
        -m gpu -x -v --timeout 120 --timeout-method thread -k "chain" > "$out/pytest_$v.log" 2>&1
  done
  b() {  # b LIB NAME ARGS...
    lib=$1; name=$2; shift 2
    if [ $lib = product ]; then L=$PWD/aipstack_amd/lib/libaipstack_chksum.so; else L=$PWD/tools/build/lib_$lib.so; fi
    AIPSTACK_AMD_LIB=$L timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline \
        "$@" >> "$out/${name}_$lib.json" 2>> "$out/${name}_$lib.err"
  }
  for i in 1 2; do
    for v in product ${VARS:-chaincols chaincols16}; do b $v CHAIN --config CHAIN --per-launch --no-ceiling; done
  done
  for v in product ${VARS:-chaincols chaincols16}; do
    b $v CHAINFILL --config CHAIN --chain-fill --no-ceiling
    b $v CHAIN_plain --config CHAIN --fresh plain --no-ceiling
    b $v CHAIN_plain_hint --config CHAIN --fresh plain --just-written --no-ceiling
    b $v CHAIN_dma --config CHAIN --fresh dma --no-ceiling
  done
  for v in ${VARS:-chaincols}; do
    AIPSTACK_AMD_LIB=$PWD/tools/build/lib_$v.so timeout -s KILL 120 rocprofv3 --kernel-trace \
        --output-format csv -d "$out/pmc_$v" -o run --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU \
        SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY -- python3 bench.py --config CHAIN --steps 20 --warmup 5 \
        --no-cpu-baseline --no-parity --no-ceiling > "$out/pmc_$v.log" 2>&1
  done
  ;;
ccols2)  # the column-run chain kernel for AIPSTACK_CHKSUM_JUST_WRITTEN in the product build:
         # chain tests (the Tx-shaped random chains included), the hint's fresh-data rates
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
      -k "chain or just_written" > "$out/pytest.log" 2>&1
  b() {  # b NAME ARGS...
    name=$1; shift
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ceiling "$@" \
        >> "$out/$name.json" 2>> "$out/$name.err"
  }
  b CHAIN --config CHAIN --per-launch
  b CHAIN_hint --config CHAIN --per-launch --just-written
  b CHAIN_plain --config CHAIN --fresh plain
  b CHAIN_plain_hint --config CHAIN --fresh plain --just-written
  b CHAIN_dma_hint --config CHAIN --fresh dma --just-written
  b CHAINFILL --config CHAIN --chain-fill
  b CHAINFILL_hint --config CHAIN --chain-fill --just-written
  b CHAINFILL_plain_hint --config CHAIN --chain-fill --fresh plain --just-written
  ;;
chshape)  # chain groups per wave (AIPSTACK_CHKSUM_CHUNKS_PER_WAVE; default: one group of 32
          # chains per wave) at steady state, alternating processes
  for i in 1 2; do
    for w in 0 2 4 8; do
      AIPSTACK_CHKSUM_CHUNKS_PER_WAVE=$w timeout -k 10 300 python3 bench.py --config CHAIN --steps 20 \
          --warmup 5 --no-cpu-baseline --no-ceiling >> "$out/CHAIN_cpw$w.json" 2>> "$out/CHAIN_cpw$w.err"
    done
  done
  ;;
final_bench)  # every config under the driver's protocol (A first, as the box's first GPU
              # process), with the CPU baseline, the read probe and the Tx / records / slot ceilings
  for c in A B C A2K C2K CHAIN RX RX2K TXREC TX TX2K; do
    timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 5 --per-launch \
        >> "$out/bench_$c.json" 2>> "$out/bench_$c.err"
  done
  timeout -k 10 120 tools/build/hbm_peak ceiling > "$out/ceiling.jsonl"
  ;;
final_prof)  # rocprofv3 --kernel-trace --stats of each config's driver-protocol command
  for c in A B C A2K C2K CHAIN RX RX2K TXREC TX TX2K; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_$c" -o run \
        -- python3 bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-ceiling \
        > "$out/prof_$c.log" 2>&1
  done
  ;;
final_pmc1)  # PMC passes (tools/pmc_run.sh), first half of the configs
  for c in A B C A2K C2K CHAIN; do tools/pmc_run.sh $c "$out/pmc_$c"; done
  ;;
final_pmc2)
  for c in RX RX2K TXREC TX TX2K; do tools/pmc_run.sh $c "$out/pmc_$c"; done
  ;;
final_misc)  # small batches, end to end, the chain fill, fresh A, the 8-rank launch rehearsed
  for n in 64 4096; do
    for c in A RX TX; do
      timeout -k 10 120 python3 bench.py --config $c --small $n >> "$out/small.jsonl" 2>> "$out/small.err"
    done
  done
  for c in A C RX TX C2K; do
    timeout -k 10 300 python3 bench.py --e2e --config $c --steps 5 --warmup 1 >> "$out/e2e.jsonl" 2>> "$out/e2e.err"
  done
  timeout -k 10 300 python3 bench.py --config CHAIN --chain-fill --steps 20 --warmup 5 \
      --no-cpu-baseline > "$out/bench_CHAINFILL.json" 2> "$out/bench_CHAINFILL.err"
  for w in dma plain; do
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --fresh $w \
        >> "$out/fresh_A.json" 2>> "$out/fresh_A.err"
  done
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --fresh plain \
      --just-written >> "$out/fresh_A.json" 2>> "$out/fresh_A.err"
  for h in "" --just-written; do
    timeout -k 10 300 python3 bench.py --config CHAIN --steps 20 --warmup 5 --no-cpu-baseline \
        --fresh plain $h >> "$out/fresh_CHAIN.json" 2>> "$out/fresh_CHAIN.err"
  done
  AIPSTACK_BENCH_FORCE_DEVICE=0 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 \
      --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29631 bench.py --gpus 8 \
      --steps 20 --warmup 5 --cpu-reps 3 > "$out/bench8_A.json" 2> "$out/bench8_A.err"
  ;;
final_test)  # the round-end gate on this tree
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
      > "$out/pytest_gpu.log" 2>&1
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1
  timeout -k 10 120 tests/cpp/build/engine_fault_test > "$out/engine_fault.log" 2>&1
  ;;
hint6)  # the JUST_WRITTEN hint in the gathered and gapped forms and the chains (nontemporal
        # edge loads): parity, fresh plain-written data with and without it; the chain fill with
        # nontemporal field stores (lib_fieldnt)
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
      -k "just_written or chain or gapped or slotted or short_runs" > "$out/pytest.log" 2>&1
  b() {  # b NAME ARGS...
    name=$1; shift
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ceiling "$@" >> "$out/$name.json" 2>> "$out/$name.err"
  }
  for c in A2K C2K CHAIN; do
    b fresh_$c --config $c --fresh plain
    b fresh_$c --config $c --fresh plain --just-written
    b fresh_$c --config $c --fresh dma --just-written
    b steady_$c --config $c
  done
  for i in 1 2; do
    b chainfill --config CHAIN --chain-fill
    AIPSTACK_AMD_LIB=$PWD/tools/build/lib_fieldnt.so b chainfill_nt --config CHAIN --chain-fill
  done
  ;;
hint6b)  # the hint on batches read before (steady state): chains and ring slots, alternating
  b() {  # b NAME ARGS...
    name=$1; shift
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ceiling "$@" >> "$out/$name.json" 2>> "$out/$name.err"
  }
  for i in 1 2; do
    for c in CHAIN C2K; do
      b steady_$c --config $c
      b steady_hint_$c --config $c --just-written
    done
  done
  b chainfill --config CHAIN --chain-fill
  b chainfill_hint --config CHAIN --chain-fill --just-written
  ;;
txsplit6)  # the split Tx fills with nontemporal field stores in the scatter pass (lib_txnt:
           # every field store nontemporal) against ordinary ones, and the one-pass fills
  b() {  # b NAME ARGS...
    name=$1; shift
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ceiling "$@" >> "$out/$name.json" 2>> "$out/$name.err"
  }
  for i in 1 2; do
    for c in TX TX2K; do
      b ${c}_split --config $c --tx-split
      AIPSTACK_AMD_LIB=$PWD/tools/build/lib_txnt.so b ${c}_split_nt --config $c --tx-split
      b ${c}_one --config $c
      AIPSTACK_AMD_LIB=$PWD/tools/build/lib_txnt.so b ${c}_one_nt --config $c
    done
  done
  ;;
driver)  # the driver's exact command on a fresh box, twice, and the N = 2 rehearsal
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$out/n1_a.json" 2> "$out/n1_a.err"
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$out/n1_b.json" 2> "$out/n1_b.err"
  ;;
*)
  echo "unknown mode $mode"; exit 2 ;;
esac
