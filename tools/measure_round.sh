#!/bin/bash
# One round's GPU measurements, written under gpurun_out/$1 (e.g. r01):
#   hbm_peak.jsonl         streaming-read ceiling of this MI355X (tools/hbm_peak.hip)
#   bench_{A,B,C}.json     bench.py lines (A with the CPU baseline)
#   prof_A/                rocprofv3 --kernel-trace --stats of the default bench command
#   pmc_{A,B,C}/           PMC passes (FETCH_SIZE, WRITE_SIZE+GRBM, SQ instruction mix)
set -e
tag=${1:-r01}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 120 tools/build/hbm_peak > "$out/hbm_peak.jsonl"
timeout -k 10 300 python bench.py > "$out/bench_A.json" 2> "$out/bench_A.err"
timeout -k 10 300 python bench.py --config B --no-cpu-baseline > "$out/bench_B.json" 2> "$out/bench_B.err"
timeout -k 10 300 python bench.py --config C --no-cpu-baseline > "$out/bench_C.json" 2> "$out/bench_C.err"
timeout -k 10 300 python bench.py --config RX --steps 10 > "$out/bench_RX.json" 2> "$out/bench_RX.err"
timeout -k 10 300 python bench.py --config TX --steps 10 > "$out/bench_TX.json" 2> "$out/bench_TX.err"
: > "$out/e2e.jsonl"
for c in A C; do
  timeout -k 10 300 python bench.py --e2e --config $c --steps 5 --warmup 1 >> "$out/e2e.jsonl" 2>> "$out/e2e.err"
  timeout -k 10 300 python bench.py --e2e --e2e-pageable --config $c --steps 3 --warmup 1 >> "$out/e2e.jsonl" 2>> "$out/e2e.err"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_A" -o run \
    -- python3 bench.py --no-cpu-baseline > "$out/prof_A.log" 2>&1
for c in A B C RX TX; do tools/pmc_run.sh $c "$out/pmc_$c"; done
for c in A B C; do timeout -k 10 200 python tools/sweep.py --config $c > "$out/sweep_$c.jsonl" 2> "$out/sweep_$c.err"; done
echo "measure_round: done"
