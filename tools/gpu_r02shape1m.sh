#!/bin/bash
# Full-size batches under other chunk shapes (A, C, CHAIN): default vs forced
# chunk_packets / stream windows, two interleaved rounds.
set -e
out=gpurun_out/r02shape1m
mkdir -p "$out"
export TMPDIR=/tmp
run() { tag=$1; shift; env "$@" timeout -k 10 200 python bench.py --config $cfg --no-cpu-baseline --no-parity --per-launch >> "$out/${cfg}_$tag.jsonl" 2>> "$out/err"; }
for r in 1 2; do
  cfg=A; run default X=1; run c64s8 AIPSTACK_CHKSUM_STREAM=8; run c32s8 AIPSTACK_CHKSUM_CHUNK_PACKETS=32 AIPSTACK_CHKSUM_STREAM=8; run c32s2 AIPSTACK_CHKSUM_CHUNK_PACKETS=32 AIPSTACK_CHKSUM_STREAM=2; run c16s8 AIPSTACK_CHKSUM_CHUNK_PACKETS=16 AIPSTACK_CHKSUM_STREAM=8
  cfg=C; run default X=1; run c32s8 AIPSTACK_CHKSUM_CHUNK_PACKETS=32
  cfg=CHAIN; run default X=1; run c32 AIPSTACK_CHKSUM_CHUNK_PACKETS=32
done
echo done
