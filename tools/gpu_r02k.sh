#!/bin/bash
# Stream scan interleave (il) and frame-stream holes (holes) vs HEAD (prev), same call:
#   product lib = il + holes; lib_il = interleave only; lib_holes = holes only.
set -e
out=gpurun_out/r02k
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > "$out/pytest_parity.log" 2>&1
run() {  # cfg tag variants [lib]
  local cfg=$1 tag=$2 v=$3 lib=$4
  if [ -n "$lib" ]; then
    timeout -k 10 200 python tools/sweep.py --config $cfg --rounds 4 --variants "$v" --lib $lib >> "$out/sweep_${cfg}_$tag.jsonl" 2>> "$out/err_${cfg}_$tag"
  else
    timeout -k 10 200 python tools/sweep.py --config $cfg --rounds 4 --variants "$v" >> "$out/sweep_${cfg}_$tag.jsonl" 2>> "$out/err_${cfg}_$tag"
  fi
}
for r in 1 2; do
  for cfg in RX TX; do
    run $cfg both "0,0"
    run $cfg prev "0,0" tools/build/lib_prev.so
    run $cfg il "0,0" tools/build/lib_il.so
    run $cfg holes "0,0" tools/build/lib_holes.so
  done
  for cfg in A C; do
    run $cfg both "0,0,1,0"
    run $cfg prev "0,0,1,0" tools/build/lib_prev.so
  done
done
echo done
