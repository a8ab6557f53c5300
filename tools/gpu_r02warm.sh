#!/bin/bash
# Cold-box effect: config A in fresh processes with 5, 2000, 5 and 200 warm-up launches.
set -e
out=gpurun_out/${OUT:-r02warm}
mkdir -p "$out"
export TMPDIR=/tmp
for w in ${WARMS:-5 2000 5 200 5}; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity --per-launch --warmup $w >> "$out/A_warm.jsonl" 2>> "$out/err"
done
echo done
