#!/bin/bash
# Where the gathered TX loses: kernel trace and SQ counters of TX (and RX) on the product lib.
set -e
out=gpurun_out/r02p
mkdir -p "$out"
export TMPDIR=/tmp
for cfg in TX RX; do
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_$cfg -o run -- python3 bench.py --config $cfg --no-cpu-baseline --no-parity > $out/prof_$cfg.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $out/sq_$cfg -o run --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR \
  -- python3 bench.py --config $cfg --no-cpu-baseline --no-parity --steps 5 --warmup 2 > $out/sq_$cfg.log 2>&1
done
echo done
