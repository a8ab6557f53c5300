#!/bin/bash
# Tx fill per batch size: split (read + scatter pass) vs one-pass in-place.
set -e
out=gpurun_out/r02tx
mkdir -p "$out"
export TMPDIR=/tmp
for n in 64 1024 4096 16384 65536 262144; do
  timeout -k 10 120 python bench.py --config TX --small $n >> "$out/tx_small.jsonl" 2>> "$out/err"
  timeout -k 10 120 python bench.py --config TX --small $n --tx-inplace >> "$out/tx_small.jsonl" 2>> "$out/err"
done
timeout -k 10 200 python bench.py --config TX --no-cpu-baseline --per-launch >> "$out/tx_big.jsonl" 2>> "$out/err"
timeout -k 10 200 python bench.py --config TX --no-cpu-baseline --per-launch --tx-inplace >> "$out/tx_big.jsonl" 2>> "$out/err"
echo done
