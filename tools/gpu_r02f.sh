#!/bin/bash
# Deferred-store frame kernels: parity + RX/TX deferred vs per-chunk stores.
set -e
out=gpurun_out/r02f
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "rx_verify_matches or tx_fill_matches" -x -q --timeout 120 --timeout-method thread > "$out/pytest_frames.log" 2>&1
timeout -k 10 300 python tools/sweep.py --config RX --rounds 6 --variants "0,0,0,1;0,0,0,0;0,0,0,4;0,0,4,1" > "$out/sweep_RX.jsonl" 2> "$out/sweep_RX.err"
timeout -k 10 300 python tools/sweep.py --config TX --rounds 6 --variants "0,0,0,1;0,0,0,0;0,0,0,4;0,0,4,1" > "$out/sweep_TX.jsonl" 2> "$out/sweep_TX.err"
echo done
