#!/bin/bash
# Chain kernel A/B: product vs lib_prev (HEAD bab2a58).
set -e
out=gpurun_out/${1:-r02z}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "chain" -x -q --timeout 120 --timeout-method thread > "$out/pytest_chain.log" 2>&1
for r in 1 2; do
  unset AIPSTACK_AMD_LIB
  timeout -k 10 200 python bench.py --config CHAIN --steps 20 --per-launch --no-cpu-baseline >> "$out/bench_CHAIN_new.jsonl" 2>> "$out/err"
  export AIPSTACK_AMD_LIB=$PWD/tools/build/lib_prev.so
  timeout -k 10 200 python bench.py --config CHAIN --steps 20 --per-launch --no-cpu-baseline >> "$out/bench_CHAIN_prev.jsonl" 2>> "$out/err"
done
unset AIPSTACK_AMD_LIB
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_CHAIN -o run -- python3 bench.py --config CHAIN --no-cpu-baseline --no-parity --steps 40 --warmup 1 > $out/prof_CHAIN.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $out/sq_CHAIN -o run --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR \
  -- python3 bench.py --config CHAIN --no-cpu-baseline --no-parity --steps 5 --warmup 2 > $out/sq_CHAIN.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $out/fetch_CHAIN -o run --pmc FETCH_SIZE \
  -- python3 bench.py --config CHAIN --no-cpu-baseline --no-parity --steps 5 --warmup 2 > $out/fetch_CHAIN.log 2>&1
echo done
