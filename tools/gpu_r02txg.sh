#!/bin/bash
# One-pass in-place Tx fill with headers captured from the stream (AIPSTACK_FRAME_GATHER_TX=1
# variant) vs the product's per-lane header loads; split fill of both for reference.
set -e
out=gpurun_out/r02txg
mkdir -p "$out"
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 200 python bench.py --config TX --no-cpu-baseline --per-launch --tx-inplace >> "$out/inplace_product.jsonl" 2>> "$out/err"
  AIPSTACK_AMD_LIB=$PWD/tools/build/lib_txg.so timeout -k 10 200 python bench.py --config TX --no-cpu-baseline --per-launch --tx-inplace >> "$out/inplace_txg.jsonl" 2>> "$out/err"
  timeout -k 10 200 python bench.py --config TX --no-cpu-baseline --per-launch >> "$out/split_product.jsonl" 2>> "$out/err"
  AIPSTACK_AMD_LIB=$PWD/tools/build/lib_txg.so timeout -k 10 200 python bench.py --config TX --no-cpu-baseline --per-launch >> "$out/split_txg.jsonl" 2>> "$out/err"
done
echo done
