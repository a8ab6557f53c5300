#!/bin/bash
# Split Tx fill: where do the records' 22 us come from? Product vs a build whose scatter
# pass stores statuses but no fields (AIPSTACK_TX_STORE_MODE=2: wrong output, pricing only).
set -e
out=gpurun_out/r02txwb
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_product -o run -- python3 bench.py --config TX --no-cpu-baseline --no-parity > $out/prof_product.log 2>&1
AIPSTACK_AMD_LIB=$PWD/tools/build/lib_nofields.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_nofields -o run -- python3 bench.py --config TX --no-cpu-baseline --no-parity > $out/prof_nofields.log 2>&1
echo done
