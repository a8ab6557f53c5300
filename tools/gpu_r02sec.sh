#!/bin/bash
# Split Tx fill with whole-sector field writes (lib_sectors) vs the product: parity on the
# Tx tests, then rocprof of both over 2,100 launches.
set -e
out=gpurun_out/r02sec
mkdir -p "$out"
export TMPDIR=/tmp
AIPSTACK_AMD_LIB=$PWD/tools/build/lib_sectors.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "tx_fill" -x -q --timeout 120 --timeout-method thread > $out/pytest_sectors.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_product -o run -- python3 bench.py --config TX --no-cpu-baseline --no-parity > $out/prof_product.log 2>&1
AIPSTACK_AMD_LIB=$PWD/tools/build/lib_sectors.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_sectors -o run -- python3 bench.py --config TX --no-cpu-baseline --no-parity > $out/prof_sectors.log 2>&1
AIPSTACK_AMD_LIB=$PWD/tools/build/lib_sectors.so timeout -k 10 200 python bench.py --config TX --no-cpu-baseline --per-launch --steps 20 > $out/bench_TX_sectors.json 2> $out/err
timeout -k 10 200 python bench.py --config TX --no-cpu-baseline --per-launch --steps 20 > $out/bench_TX_product.json 2>> $out/err
echo done
