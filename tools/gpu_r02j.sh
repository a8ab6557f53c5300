#!/bin/bash
# Frame kernels: boundary partials from header registers vs previous (A/B, same call).
set -e
out=gpurun_out/r02j
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "rx_ or tx_ or fill" -x -q --timeout 120 --timeout-method thread > "$out/pytest_frames.log" 2>&1
for cfg in RX TX; do
  for r in 1 2; do
    timeout -k 10 200 python tools/sweep.py --config $cfg --rounds 4 --variants "0,0,0" > "$out/sweep_${cfg}_new_$r.jsonl" 2> "$out/err_${cfg}_new"
    timeout -k 10 200 python tools/sweep.py --config $cfg --rounds 4 --variants "0,0,0" --lib tools/build/lib_prev.so > "$out/sweep_${cfg}_prev_$r.jsonl" 2> "$out/err_${cfg}_prev"
  done
done
echo done
