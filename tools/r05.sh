#!/bin/bash
# Round-5 GPU experiments, one mode per gpurun call; output under gpurun_out/r05/<mode>.
#   driver  the driver's exact bench command (--steps 20 --warmup 5) as the box's first GPU
#           process, with per-launch times; the same under rocprofv3 kernel traces (every
#           dispatch, warm-ups included) for the gathered loader and stream mode; 400-launch
#           traces from cold; rotated vs one-buffer; the rotated streaming-read ceiling
set -e
mode=${1:?mode}
out=gpurun_out/r05/$mode
mkdir -p "$out"
export TMPDIR=/tmp

bench() {  # bench NAME ARGS... -> $out/NAME.json (appended)
  name=$1; shift
  timeout -k 10 300 python3 bench.py "$@" >> "$out/$name.json" 2>> "$out/$name.err"
}
trace() {  # trace NAME ARGS...: kernel trace + stats of one bench command (env passes through)
  name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/$name" -o run \
      -- python3 bench.py "$@" > "$out/$name.log" 2>&1
}

case $mode in
driver)
  bench n1_default --gpus 1 --steps 20 --warmup 5 --per-launch
  AIPSTACK_CHKSUM_GATHER=-1 bench n1_stream --gpus 1 --steps 20 --warmup 5 --per-launch --no-cpu-baseline
  bench n1_rot1 --gpus 1 --steps 20 --warmup 5 --per-launch --no-cpu-baseline --rotate 1
  trace tr_default --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-ceiling
  AIPSTACK_CHKSUM_GATHER=-1 trace tr_stream --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-ceiling
  trace long_default --steps 400 --warmup 0 --no-cpu-baseline --no-ceiling
  AIPSTACK_CHKSUM_GATHER=-1 trace long_stream --steps 400 --warmup 0 --no-cpu-baseline --no-ceiling
  trace long_rot1 --steps 400 --warmup 0 --no-cpu-baseline --no-ceiling --rotate 1
  timeout -k 10 120 tools/build/hbm_peak ceiling > "$out/ceiling.jsonl"
  timeout -k 10 120 tools/build/hbm_peak ceiling >> "$out/ceiling.jsonl"
  ;;
short)  # round-5 short runs (gather 1, the strided default) vs the round-4 gathered stream (0)
  bench n1_short --gpus 1 --steps 20 --warmup 5 --per-launch
  AIPSTACK_CHKSUM_GATHER=0 bench n1_gath --gpus 1 --steps 20 --warmup 5 --per-launch --no-cpu-baseline
  bench n1_short --gpus 1 --steps 20 --warmup 5 --per-launch --no-cpu-baseline
  AIPSTACK_CHKSUM_GATHER=0 bench n1_gath --gpus 1 --steps 20 --warmup 5 --per-launch --no-cpu-baseline
  trace long_short --steps 400 --warmup 0 --no-cpu-baseline --no-ceiling
  AIPSTACK_CHKSUM_GATHER=0 trace long_gath --steps 400 --warmup 0 --no-cpu-baseline --no-ceiling
  trace tr_short --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-ceiling
  for cp in 0 2 4; do
    AIPSTACK_CHKSUM_CHUNK_PACKETS=$cp bench B_cp$cp --config B --steps 20 --warmup 5 --per-launch --no-cpu-baseline
  done
  AIPSTACK_CHKSUM_GATHER=0 bench B_gath --config B --steps 20 --warmup 5 --per-launch --no-cpu-baseline
  bench C_gath --config C --steps 20 --warmup 5 --per-launch --no-cpu-baseline
  for cp in 0 8 32; do
    AIPSTACK_CHKSUM_GATHER=2 AIPSTACK_CHKSUM_CHUNK_PACKETS=$cp bench C_short$cp --config C --steps 20 --warmup 5 --per-launch --no-cpu-baseline
  done
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
      -k "every_read_form or short_runs or full_size or config_d or stream_mode or ragged or lengths" \
      > "$out/pytest.log" 2>&1
  ;;
*)
  echo "unknown mode $mode"; exit 2 ;;
esac
echo "r05 $mode done"
