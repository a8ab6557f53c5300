#!/bin/bash
# Batch-shape transition: A and RX at 8K..512K packets per batch, automatic shape vs forced
# (64 packets per chunk with the family's default windows, 64 with 8 windows, 16 and 32
# with 8 windows).
set -e
out=gpurun_out/r02sb3
mkdir -p "$out"
export TMPDIR=/tmp
for c in A RX; do for n in 8192 32768 65536 131072 262144 524288; do
  timeout -k 10 120 python bench.py --config $c --small $n >> "$out/shape.jsonl" 2>> "$out/err"
  AIPSTACK_CHKSUM_CHUNK_PACKETS=64 timeout -k 10 120 python bench.py --config $c --small $n >> "$out/shape.jsonl" 2>> "$out/err"
  AIPSTACK_CHKSUM_CHUNK_PACKETS=64 AIPSTACK_CHKSUM_STREAM=8 timeout -k 10 120 python bench.py --config $c --small $n >> "$out/shape.jsonl" 2>> "$out/err"
  AIPSTACK_CHKSUM_CHUNK_PACKETS=32 AIPSTACK_CHKSUM_STREAM=8 timeout -k 10 120 python bench.py --config $c --small $n >> "$out/shape.jsonl" 2>> "$out/err"
  AIPSTACK_CHKSUM_CHUNK_PACKETS=16 AIPSTACK_CHKSUM_STREAM=8 timeout -k 10 120 python bench.py --config $c --small $n >> "$out/shape.jsonl" 2>> "$out/err"
done; done
echo done
