#!/bin/bash
# Price of the frame kernels' per-lane header loads: every lane parses the chunk's first
# (L2-hot) header instead (lib_exphdr; wrong output, same stream) vs the product (HEAD).
set -e
out=gpurun_out/r02n
mkdir -p "$out"
export TMPDIR=/tmp
for r in 1 2; do
  for cfg in RX TX; do
    timeout -k 10 200 python tools/sweep.py --config $cfg --rounds 4 --variants "0,0" >> "$out/sweep_${cfg}_head.jsonl" 2>> "$out/err"
    timeout -k 10 200 python tools/sweep.py --config $cfg --rounds 4 --variants "0,0" --lib tools/build/lib_exphdr.so >> "$out/sweep_${cfg}_exphdr.jsonl" 2>> "$out/err"
  done
done
export AIPSTACK_AMD_LIB=$PWD/tools/build/lib_exphdr.so
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $out/pmc_RX_exphdr -o run --pmc FETCH_SIZE \
  -- python3 bench.py --config RX --no-cpu-baseline --no-parity --steps 5 --warmup 2 > $out/pmc.log 2>&1
echo done
