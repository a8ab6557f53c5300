#!/bin/bash
# Frame kernels: occupancy variants (launch bounds 4/5/6 waves per SIMD) x stream windows.
set -e
out=gpurun_out/r02i
mkdir -p "$out"
export TMPDIR=/tmp
for cfg in RX TX; do
  timeout -k 10 200 python tools/sweep.py --config $cfg --rounds 5 --variants "0,0,0;0,0,4" > "$out/sweep_${cfg}_w4.jsonl" 2> "$out/err_${cfg}_w4"
  timeout -k 10 200 python tools/sweep.py --config $cfg --rounds 5 --variants "0,0,0;0,0,4" --lib tools/build/lib_fw5.so > "$out/sweep_${cfg}_w5.jsonl" 2> "$out/err_${cfg}_w5"
  timeout -k 10 200 python tools/sweep.py --config $cfg --rounds 5 --variants "0,0,4;0,0,2" --lib tools/build/lib_fw6.so > "$out/sweep_${cfg}_w6.jsonl" 2> "$out/err_${cfg}_w6"
done
echo done
