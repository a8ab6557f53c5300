#!/bin/bash
# One round's GPU measurements, written under gpurun_out/$1 (e.g. r01). Phases (arg 2,
# default "all"; each fits one gpurun call on its own):
#   bench  hbm_peak.jsonl (streaming-read ceiling, tools/hbm_peak.hip);
#          bench_{A,B,C,RX,TX,CHAIN}.json (A with the CPU baseline); e2e.jsonl;
#          prof_A/ and prof_C/: rocprofv3 --kernel-trace --stats of the bench command
#   pmc    pmc_{A,B,C,RX,TX,CHAIN}/: PMC passes (FETCH_SIZE, WRITE_SIZE, SQ instruction mix)
#   sweep  sweep_{A,B,C,RX,TX}.jsonl: launch-parameter sweeps (tools/sweep.py)
set -e
tag=${1:-r01}
phase=${2:-all}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp

if [ "$phase" = bench ] || [ "$phase" = all ]; then
  timeout -k 10 120 tools/build/hbm_peak > "$out/hbm_peak.jsonl"
  timeout -k 10 300 python bench.py > "$out/bench_A.json" 2> "$out/bench_A.err"
  for c in B C; do
    timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --per-launch \
        > "$out/bench_$c.json" 2> "$out/bench_$c.err"
  done
  for c in RX TX CHAIN; do
    timeout -k 10 300 python bench.py --config $c --steps 10 --per-launch \
        > "$out/bench_$c.json" 2> "$out/bench_$c.err"
  done
  : > "$out/e2e.jsonl"
  for c in A C; do
    timeout -k 10 300 python bench.py --e2e --config $c --steps 5 --warmup 1 >> "$out/e2e.jsonl" 2>> "$out/e2e.err"
    timeout -k 10 300 python bench.py --e2e --e2e-pageable --config $c --steps 3 --warmup 1 >> "$out/e2e.jsonl" 2>> "$out/e2e.err"
  done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_A" -o run \
      -- python3 bench.py --no-cpu-baseline > "$out/prof_A.log" 2>&1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_C" -o run \
      -- python3 bench.py --config C --no-cpu-baseline > "$out/prof_C.log" 2>&1
fi
if [ "$phase" = pmc ] || [ "$phase" = all ]; then
  for c in A B C RX TX CHAIN; do tools/pmc_run.sh $c "$out/pmc_$c"; done
fi
if [ "$phase" = sweep ] || [ "$phase" = all ]; then
  for c in A B C RX TX; do
    timeout -k 10 200 python tools/sweep.py --config $c > "$out/sweep_$c.jsonl" 2> "$out/sweep_$c.err"
  done
fi
echo "measure_round: $phase done"
