#!/bin/bash
# Rehearsal of the driver's 8-rank launch on a 1-GPU box: 8 ranks on device 0
# (AIPSTACK_BENCH_FORCE_DEVICE), configs A and C. Throughput is shared by the 8 ranks, so
# only the control plane and parity are what this checks.
set -e
out=gpurun_out/r02rank8
mkdir -p "$out"
export TMPDIR=/tmp AIPSTACK_BENCH_FORCE_DEVICE=0
for c in A C; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
      --master-port 29531 bench.py --gpus 8 --config $c --steps 5 --warmup 2 --cpu-reps 3 \
      > "$out/bench8_$c.json" 2> "$out/bench8_$c.err"
done
echo done
