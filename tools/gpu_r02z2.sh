#!/bin/bash
# Chain pairs: default-policy loads (AIPSTACK_CHKSUM_NT=0) vs nt, and HEAD's one-segment loader.
set -e
out=gpurun_out/r02z2
mkdir -p "$out"
export TMPDIR=/tmp
for nt in 0 1; do
  export AIPSTACK_CHKSUM_NT=$nt
  unset AIPSTACK_AMD_LIB
  timeout -k 10 200 python bench.py --config CHAIN --steps 20 --per-launch --no-cpu-baseline >> "$out/bench_CHAIN_pairs_nt$nt.jsonl" 2>> "$out/err"
  export AIPSTACK_AMD_LIB=$PWD/tools/build/lib_prev.so
  timeout -k 10 200 python bench.py --config CHAIN --steps 20 --per-launch --no-cpu-baseline >> "$out/bench_CHAIN_prev_nt$nt.jsonl" 2>> "$out/err"
done
unset AIPSTACK_AMD_LIB
export AIPSTACK_CHKSUM_NT=0
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $out/fetch_CHAIN_nt0 -o run --pmc FETCH_SIZE \
  -- python3 bench.py --config CHAIN --no-cpu-baseline --no-parity --steps 5 --warmup 2 > $out/fetch_CHAIN.log 2>&1
echo done
