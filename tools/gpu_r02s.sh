#!/bin/bash
# Split Tx read pass: gathered vs classic headers, with and without its record stores
# (kernel traces separate the read pass from the scatter pass).
set -e
out=gpurun_out/r02s
mkdir -p "$out"
export TMPDIR=/tmp
for v in product txg txg_norec norec; do
  if [ $v = product ]; then unset AIPSTACK_AMD_LIB; else export AIPSTACK_AMD_LIB=$PWD/tools/build/lib_$v.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_$v -o run -- python3 bench.py --config TX --no-cpu-baseline --no-parity > $out/prof_$v.log 2>&1
done
echo done
