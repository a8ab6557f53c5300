#!/bin/bash
# Round 2, first GPU pass: GPU tests, bench A (new cpu_baseline fields), the slotted A2K
# config (per-packet wave mode) and CHAIN (gathered stream), with rocprof kernel traces.
set -e
out=gpurun_out/r02a
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$out/pytest_gpu.log" 2>&1
timeout -k 10 300 python bench.py > "$out/bench_A.json" 2> "$out/bench_A.err"
timeout -k 10 300 python bench.py --config A2K --per-launch > "$out/bench_A2K.json" 2> "$out/bench_A2K.err"
timeout -k 10 300 python bench.py --config CHAIN --steps 10 --per-launch > "$out/bench_CHAIN.json" 2> "$out/bench_CHAIN.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_A2K" -o run \
    -- python3 bench.py --config A2K --no-cpu-baseline > "$out/prof_A2K.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_CHAIN" -o run \
    -- python3 bench.py --config CHAIN --no-parity > "$out/prof_CHAIN.log" 2>&1
echo done
