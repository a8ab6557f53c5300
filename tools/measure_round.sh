#!/bin/bash
# One round's GPU measurements, written under gpurun_out/$1 (e.g. r03). Phases (arg 2,
# default "all"; each fits one gpurun call on its own):
#   test   pytest -m gpu (the round-end gate) and smoke()
#   bench  hbm_peak.jsonl (streaming-read ceiling + slotted-read ceiling, tools/hbm_peak.hip);
#          bench_<CFG>.json for every config in $CONFIGS (default: all; CPU baselines;
#          RX2K / C2K with their slot-read ceilings)
#   e2e    e2e.jsonl: host memory in and out (single engine, and an engine group of 2)
#   prof   prof_<CFG>/: rocprofv3 --kernel-trace --stats of the bench command
#   pmc    pmc_<CFG>/: PMC passes (FETCH_SIZE, WRITE_SIZE, SQ instruction mix); summarise
#          with tools/pmc_summary.py on the same tree (entries record the kernel digest)
#   sweep  sweep_{A,B,C,RX,TX}.jsonl: launch-parameter sweeps (tools/sweep.py)
#   rank8  the driver's 8-rank launch rehearsed on a 1-GPU box (all ranks on device 0):
#          control plane, per-rank parity and device ids (throughput is shared)
#   small  small batches (bench.py --small) for A, RX and TX, eager vs graph replay
set -e
tag=${1:-r02}
phase=${2:-all}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp

if [ "$phase" = test ] || [ "$phase" = all ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$out/pytest_gpu.log" 2>&1
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1
fi
CONFIGS=${CONFIGS:-A B C A2K C2K RX RX2K TX TX2K TXREC CHAIN}
if [ "$phase" = bench ] || [ "$phase" = all ]; then
  timeout -k 10 120 tools/build/hbm_peak > "$out/hbm_peak.jsonl"
  for c in $CONFIGS; do
    timeout -k 10 300 python bench.py --config $c --per-launch \
        > "$out/bench_$c.json" 2> "$out/bench_$c.err"
  done
fi
if [ "$phase" = e2e ] || [ "$phase" = all ]; then
  : > "$out/e2e.jsonl"
  for c in A C RX TX RX2K TX2K C2K; do
    timeout -k 10 300 python bench.py --e2e --config $c --steps 5 --warmup 1 >> "$out/e2e.jsonl" 2>> "$out/e2e.err"
    timeout -k 10 300 python bench.py --e2e --e2e-pageable --config $c --steps 3 --warmup 1 >> "$out/e2e.jsonl" 2>> "$out/e2e.err"
  done
  AIPSTACK_BENCH_FORCE_DEVICE=0 timeout -k 10 300 python bench.py --e2e --engines 2 --config C \
      --steps 5 --warmup 1 >> "$out/e2e.jsonl" 2>> "$out/e2e.err"
fi
if [ "$phase" = prof ] || [ "$phase" = all ]; then
  for c in $CONFIGS; do
    [ "$c" = B ] && continue
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_$c" -o run \
        -- python3 bench.py --config $c --no-cpu-baseline --no-parity > "$out/prof_$c.log" 2>&1
  done
fi
if [ "$phase" = pmc ] || [ "$phase" = all ]; then
  for c in $CONFIGS; do tools/pmc_run.sh $c "$out/pmc_$c"; done
fi
if [ "$phase" = sweep ] || [ "$phase" = all ]; then
  for c in A B C A2K RX TX; do
    timeout -k 10 200 python tools/sweep.py --config $c > "$out/sweep_$c.jsonl" 2> "$out/sweep_$c.err"
  done
fi
if [ "$phase" = rank8 ]; then
  for c in A C; do
    AIPSTACK_BENCH_FORCE_DEVICE=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 8 \
        --config $c --steps 5 --warmup 2 --cpu-reps 3 > "$out/bench8_$c.json" 2> "$out/bench8_$c.err"
  done
fi
if [ "$phase" = small ]; then
  for n in 64 1024 4096 16384; do
    for c in A RX TX; do
      timeout -k 10 120 python bench.py --config $c --small $n >> "$out/small.jsonl" 2>> "$out/small.err"
    done
  done
fi
echo "measure_round: $phase done"
