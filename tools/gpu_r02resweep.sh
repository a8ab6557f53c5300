#!/bin/bash
# Final-code launch re-sweeps: CHAIN with 2 vs 4 windows per group; A2K packets in flight;
# C stream windows.
set -e
out=gpurun_out/r02resweep
mkdir -p "$out"
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 200 python bench.py --config CHAIN --steps 20 --per-launch --no-cpu-baseline --no-parity >> "$out/chain_su2.jsonl" 2>> "$out/err"
  AIPSTACK_CHKSUM_STREAM=4 timeout -k 10 200 python bench.py --config CHAIN --steps 20 --per-launch --no-cpu-baseline --no-parity >> "$out/chain_su4.jsonl" 2>> "$out/err"
done
timeout -k 10 300 python tools/sweep.py --config A2K --rounds 4 > "$out/sweep_A2K.jsonl" 2>> "$out/err"
timeout -k 10 300 python tools/sweep.py --config C --rounds 4 --variants "0,0,1,0;0,0,1,0,2;0,0,1,0,4;0,0,1,64;0,0,1,256" > "$out/sweep_C.jsonl" 2>> "$out/err"
echo done
