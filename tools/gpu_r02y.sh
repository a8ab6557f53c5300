#!/bin/bash
# Order experiment: does the per-launch drift follow the kernel (instructions per byte) or
# the box's warm-up over a measurement script? CHAIN first on a cool chip, then A, then
# CHAIN and A again; 40 launches each under rocprofv3 --kernel-trace.
set -e
out=gpurun_out/r02y
mkdir -p "$out"
export TMPDIR=/tmp
i=0
for c in CHAIN A CHAIN A A2K RX; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $out/p${i}_$c -o run \
      -- python3 bench.py --config $c --steps 40 --warmup 1 --no-cpu-baseline --no-parity > $out/p${i}_$c.log 2>&1
done
echo done
