#!/bin/bash
# StreamRun: the last group's windows past the run are no longer consumed. Full GPU suite on
# the product, then product vs lib_prev (HEAD) on A, C, RX, TX, interleaved.
set -e
out=gpurun_out/r02skip
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/pytest_gpu.log" 2>&1
for r in 1 2; do
  for c in A C; do
    timeout -k 10 200 python tools/sweep.py --config $c --rounds 4 --variants "0,0,1,0" >> "$out/sweep_${c}_new.jsonl" 2>> "$out/err"
    timeout -k 10 200 python tools/sweep.py --config $c --rounds 4 --variants "0,0,1,0" --lib tools/build/lib_prev.so >> "$out/sweep_${c}_prev.jsonl" 2>> "$out/err"
  done
  for c in RX TX; do
    timeout -k 10 200 python tools/sweep.py --config $c --rounds 4 --variants "0,0" >> "$out/sweep_${c}_new.jsonl" 2>> "$out/err"
    timeout -k 10 200 python tools/sweep.py --config $c --rounds 4 --variants "0,0" --lib tools/build/lib_prev.so >> "$out/sweep_${c}_prev.jsonl" 2>> "$out/err"
  done
done
echo done
