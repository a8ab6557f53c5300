#!/bin/bash
# Chain kernel, gathered stream (pipelined): parity + windows-in-flight sweep.
set -e
out=gpurun_out/r02b
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k chain -x -v --timeout 120 --timeout-method thread > "$out/pytest_chain.log" 2>&1
for su in 2 4 8 4 2 8; do
  AIPSTACK_CHKSUM_STREAM=$su timeout -k 10 300 python bench.py --config CHAIN --steps 20 --per-launch --no-parity >> "$out/bench_CHAIN_sweep.jsonl" 2>> "$out/bench_CHAIN.err"
done
echo done
