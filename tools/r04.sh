#!/bin/bash
# Round-4 GPU experiments, one mode per gpurun call; output under gpurun_out/r04/<mode>.
#   txsect  the Tx fill forms (2-byte vs whole-sector field stores, split slotted fill):
#           their GPU tests, then tools/tx_sweep.py on TX2K and TX, interleaved
set -e
mode=${1:?mode}
out=gpurun_out/r04/$mode
mkdir -p "$out"
export TMPDIR=/tmp

pyt() {  # pyt NAME PYTEST-ARGS... -> $out/NAME.log
  name=$1; shift
  timeout -k 10 900 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread "$@" \
      > "$out/$name.log" 2>&1
}
sweep() {  # sweep NAME ARGS... -> $out/NAME.jsonl (appended)
  name=$1; shift
  timeout -k 10 300 python tools/tx_sweep.py "$@" >> "$out/$name.jsonl" 2>> "$out/$name.err"
}

case $mode in
txsect)
  pyt pytest_tx -m gpu -k "tx_fill or slotted or random_frames"
  for i in 1 2; do
    sweep tx2k --config TX2K --variants "split=0,store=0;split=0,store=1;split=1,store=0"
    sweep tx --config TX --variants "split=1;split=0,store=0;split=0,store=1;split=0,store=1,gather=2;split=1,gather=1"
  done
  ;;
*)
  echo "unknown mode $mode" >&2; exit 2 ;;
esac
