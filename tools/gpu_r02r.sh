#!/bin/bash
# Full GPU suite + smoke on the gathered-Rx code; Tx one-pass (in place) vs split, same call.
set -e
out=gpurun_out/r02r
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$out/pytest_gpu.log" 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1
for r in 1 2; do
  timeout -k 10 200 python tools/sweep.py --config TX --rounds 4 --variants "0,0" >> "$out/sweep_TX_split.jsonl" 2>> "$out/err"
  timeout -k 10 200 python tools/sweep.py --config TX --rounds 4 --variants "0,0" --tx-inplace >> "$out/sweep_TX_inplace.jsonl" 2>> "$out/err"
done
echo done
