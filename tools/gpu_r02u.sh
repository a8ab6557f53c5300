#!/bin/bash
# Gathered Rx with per-window SGPR masks + exec-masked capture store vs HEAD cb21732.
set -e
out=gpurun_out/r02u
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "rx_ or tx_ or fill or frame" -x -q --timeout 120 --timeout-method thread > "$out/pytest_frames.log" 2>&1
for r in 1 2; do
  timeout -k 10 200 python tools/sweep.py --config RX --rounds 4 --variants "0,0" >> "$out/sweep_RX_new.jsonl" 2>> "$out/err"
  timeout -k 10 200 python tools/sweep.py --config RX --rounds 4 --variants "0,0" --lib tools/build/lib_prev.so >> "$out/sweep_RX_prev.jsonl" 2>> "$out/err"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_RX -o run -- python3 bench.py --config RX --no-cpu-baseline --no-parity > $out/prof_RX.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $out/sq_RX -o run --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR \
  -- python3 bench.py --config RX --no-cpu-baseline --no-parity --steps 5 --warmup 2 > $out/sq_RX.log 2>&1
echo done
