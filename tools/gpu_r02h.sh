#!/bin/bash
# Chain kernel, cleaned-segment gathered stream: parity + windows-in-flight sweep.
set -e
out=gpurun_out/r02h
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k chain -x -q --timeout 120 --timeout-method thread > "$out/pytest_chain.log" 2>&1
: > "$out/bench_CHAIN_sweep.jsonl"
for su in 2 4 8 4 2; do
  AIPSTACK_CHKSUM_STREAM=$su timeout -k 10 300 python bench.py --config CHAIN --steps 20 --per-launch --no-parity >> "$out/bench_CHAIN_sweep.jsonl" 2>> "$out/bench_CHAIN.err"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_CHAIN" -o run -- python3 bench.py --config CHAIN --no-parity > "$out/prof_CHAIN.log" 2>&1
echo done
