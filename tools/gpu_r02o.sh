#!/bin/bash
# Frame stream with the headers captured from the stream into LDS (product lib) vs HEAD
# cb21732 (lib_prev): frame parity tests, interleaved sweeps, FETCH_SIZE.
set -e
out=gpurun_out/r02o
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "rx_ or tx_ or fill or frame" -x -q --timeout 120 --timeout-method thread > "$out/pytest_frames.log" 2>&1
for r in 1 2; do
  for cfg in RX TX; do
    timeout -k 10 200 python tools/sweep.py --config $cfg --rounds 4 --variants "0,0" >> "$out/sweep_${cfg}_new.jsonl" 2>> "$out/err"
    timeout -k 10 200 python tools/sweep.py --config $cfg --rounds 4 --variants "0,0" --lib tools/build/lib_prev.so >> "$out/sweep_${cfg}_prev.jsonl" 2>> "$out/err"
  done
done
for cfg in RX TX; do
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $out/pmc_$cfg -o run --pmc FETCH_SIZE \
  -- python3 bench.py --config $cfg --no-cpu-baseline --no-parity --steps 5 --warmup 2 > $out/pmc_$cfg.log 2>&1
done
echo done
