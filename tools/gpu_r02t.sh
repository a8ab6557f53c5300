#!/bin/bash
# Split Tx: stream cache policy (nt vs default) for classic and gathered headers.
set -e
out=gpurun_out/r02t
mkdir -p "$out"
export TMPDIR=/tmp
for v in product nt0 txg txg_nt0; do
  if [ $v = product ]; then unset AIPSTACK_AMD_LIB; else export AIPSTACK_AMD_LIB=$PWD/tools/build/lib_$v.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_TX_$v -o run -- python3 bench.py --config TX --no-cpu-baseline --no-parity > $out/prof_TX_$v.log 2>&1
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_RX_$v -o run -- python3 bench.py --config RX --no-cpu-baseline --no-parity > $out/prof_RX_$v.log 2>&1
done
echo done
