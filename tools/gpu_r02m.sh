#!/bin/bash
# Frame kernels: CSR offsets one chunk ahead + stores deferred behind the next chunk's loads
# (product lib) vs HEAD cb21732 (lib_prev), same call.
set -e
out=gpurun_out/r02m
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "rx_ or tx_ or fill or frame" -x -q --timeout 120 --timeout-method thread > "$out/pytest_frames.log" 2>&1
for r in 1 2; do
  for cfg in RX TX; do
    timeout -k 10 200 python tools/sweep.py --config $cfg --rounds 4 --variants "0,0" >> "$out/sweep_${cfg}_new.jsonl" 2>> "$out/err"
    timeout -k 10 200 python tools/sweep.py --config $cfg --rounds 4 --variants "0,0" --lib tools/build/lib_prev.so >> "$out/sweep_${cfg}_prev.jsonl" 2>> "$out/err"
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_RX -o run -- python3 bench.py --config RX --no-cpu-baseline --no-parity > $out/prof_RX.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_TX -o run -- python3 bench.py --config TX --no-cpu-baseline --no-parity > $out/prof_TX.log 2>&1
echo done
