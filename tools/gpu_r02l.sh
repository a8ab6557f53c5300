#!/bin/bash
# PMC: frame kernels' HBM fetch and instruction mix, holes vs HEAD (prev).
set -e
out=gpurun_out/r02l
mkdir -p "$out"
export TMPDIR=/tmp
for lib in prev holes; do
  export AIPSTACK_AMD_LIB=$PWD/tools/build/lib_$lib.so
  for cfg in RX TX; do
    d=$out/${cfg}_$lib
    mkdir -p $d
    timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $d/fetch -o run --pmc FETCH_SIZE \
      -- python3 bench.py --config $cfg --no-cpu-baseline --no-parity --steps 5 --warmup 2 > $d/fetch.log 2>&1
    timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $d/sq1 -o run --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
      -- python3 bench.py --config $cfg --no-cpu-baseline --no-parity --steps 5 --warmup 2 > $d/sq1.log 2>&1
  done
done
echo done
