#!/bin/bash
# Small-batch shapes: full GPU suite, small-batch eager/graph rates, and the big configs
# (unchanged shape) against lib_prev.
set -e
out=gpurun_out/r02sb2
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$out/pytest_gpu.log" 2>&1
for c in A RX; do for n in 1 64 256 1024 4096 16384; do
  timeout -k 10 120 python bench.py --config $c --small $n >> "$out/small.jsonl" 2>> "$out/err"
  AIPSTACK_AMD_LIB=$PWD/tools/build/lib_prev.so timeout -k 10 120 python bench.py --config $c --small $n >> "$out/small_prev.jsonl" 2>> "$out/err"
done; done
for c in A C RX TX CHAIN; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --per-launch >> "$out/big.jsonl" 2>> "$out/err"
done
echo done
