#!/bin/bash
# Slot mode (A2K) parity + sweep vs wave mode.
set -e
out=gpurun_out/r02d
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "slotted or lengths or ragged or chain" -x -q --timeout 120 --timeout-method thread > "$out/pytest.log" 2>&1
timeout -k 10 300 python tools/sweep.py --config A2K --rounds 6 > "$out/sweep_A2K.jsonl" 2> "$out/sweep_A2K.err"
timeout -k 10 300 python bench.py --config A2K --per-launch > "$out/bench_A2K.json" 2> "$out/bench_A2K.err"
echo done
