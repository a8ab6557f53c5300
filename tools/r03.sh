#!/bin/bash
# Round-3 GPU experiments, one mode per gpurun call; output under gpurun_out/r03/<mode>.
# (Round 2 kept one script per call, tools/gpu_r02*.sh; they are folded into the modes of
# this file and tools/measure_round.sh.)
#   txrec   Tx records-only read pass: header capture (default) vs per-lane header loads
#           (AIPSTACK_CHKSUM_TX_GATHER=0), interleaved; the split fill both ways; rocprof
#           stats and FETCH/WRITE passes of TXREC; then pytest -m gpu
#   check   pytest -m gpu, then bench A, C, CHAIN, TXREC, RX (no CPU baseline)
#   txnt    split Tx fill: scatter stores plain vs nontemporal (+ rocprof of each)
#   asweep  launch shapes of configs A and B (robustness across boxes)
#   estats  engine host-time counters, e2e RX / TX / TX2K
#   e2ethreads  host engine Tx: apply/staging threads, piece size, streams
#   tx2k    send ring: device in-place slotted Tx fill (bench + rocprof) and e2e
#   ringloop  the engine as a TAP receive loop from C++, per batch size
#   zc      engine zero-copy (metadata / packet bytes read in place) vs DMA: engine tests +
#           receive loop (round-3 experiment; zero copy is the default since)
#   zc2     e2e from registered memory: DMA vs zero-copy pieces, every config
#   txtouch split Tx fill with captured headers + field lines touched up front (experiment)
#   txmode  split / one-pass Tx fill by header mode, then the GPU suite
#   prows   pageable rings staged frame-bytes-only vs whole slots; a third field-line touch
#   ring    e2e receive rings (RX2K / C2K): 2-D copies of the slots' used prefix vs whole slots
#   slots   pytest -m gpu; ring-slot lines RX2K / C2K (+ their slot-read ceilings) and A2K;
#           a U/P sweep of the slotted checksum; e2e through an engine group of 1/2/4
set -e
mode=${1:?mode}
out=gpurun_out/r03/$mode
mkdir -p "$out"
export TMPDIR=/tmp

bench() {  # bench NAME ARGS... -> $out/NAME.jsonl (appended)
  name=$1; shift
  timeout -k 10 300 python bench.py "$@" >> "$out/$name.jsonl" 2>> "$out/$name.err"
}

case $mode in
txrec)
  for i in 1 2; do
    bench txrec --config TXREC --steps 100 --per-launch --no-cpu-baseline
    AIPSTACK_CHKSUM_TX_GATHER=0 bench txrec_lane --config TXREC --steps 100 --per-launch --no-cpu-baseline
    bench tx --config TX --steps 100 --per-launch --no-cpu-baseline
    AIPSTACK_CHKSUM_TX_GATHER=1 bench tx_gather --config TX --steps 100 --per-launch --no-cpu-baseline
  done
  bench rx --config RX --steps 100 --per-launch --no-cpu-baseline
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_TXREC" -o run \
      -- python3 bench.py --config TXREC --no-cpu-baseline --no-parity > "$out/prof_TXREC.log" 2>&1
  tools/pmc_run.sh TXREC "$out/pmc_TXREC"
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      > "$out/pytest_gpu.log" 2>&1
  ;;
estats)
  # where the engine's host time goes, Tx vs Rx e2e (AIPSTACK_ENGINE_STATS: stderr JSON),
  # after the GPU suite
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      > "$out/pytest_gpu.log" 2>&1
  export AIPSTACK_ENGINE_STATS=1
  for c in RX TX TX2K; do
    bench "e2e_$c" --e2e --config $c --steps 5 --warmup 1
    bench "e2ep_$c" --e2e --e2e-pageable --config $c --steps 3 --warmup 1
  done
  AIPSTACK_ENGINE_HOST_THREADS=16 bench e2ep_TX2K_t16 --e2e --e2e-pageable --config TX2K --steps 3 --warmup 1
  AIPSTACK_ENGINE_HOST_THREADS=16 bench e2ep_RX2K_t16 --e2e --e2e-pageable --config RX2K --steps 3 --warmup 1
  bench e2ep_RX2K --e2e --e2e-pageable --config RX2K --steps 3 --warmup 1
  ;;
check)
  # the GPU suite, then the timed configs the last change could move
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      > "$out/pytest_gpu.log" 2>&1
  for c in A C CHAIN TXREC RX; do
    bench "bench_$c" --config $c --per-launch --no-cpu-baseline
  done
  ;;
slots)
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      > "$out/pytest_gpu.log" 2>&1
  for c in RX2K C2K A2K; do
    bench "bench_$c" --config $c --per-launch
  done
  for u in 1 2 3; do
    for p in 4 8; do
      AIPSTACK_CHKSUM_UNROLL=$u AIPSTACK_CHKSUM_PACKETS=$p bench sweep_C2K --config C2K \
          --per-launch --no-cpu-baseline --no-parity
    done
  done
  for f in 2 4 8; do
    AIPSTACK_CHKSUM_FRAMES=$f bench sweep_RX2K --config RX2K --per-launch --no-cpu-baseline --no-parity
  done
  for e in 1 2 4; do
    AIPSTACK_BENCH_FORCE_DEVICE=0 bench e2e_group --e2e --engines $e --config C --steps 5 --warmup 1
  done
  ;;
gslot)
  # the gathered stream for ring slots (C2K) against the wave mode, interleaved
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      -k "slotted or slot" > "$out/pytest_slots.log" 2>&1
  for i in 1 2; do
    bench c2k --config C2K --per-launch --no-cpu-baseline
    AIPSTACK_CHKSUM_STREAM=4 bench c2k_su4 --config C2K --per-launch --no-cpu-baseline --no-parity
    AIPSTACK_CHKSUM_STREAM=-1 bench c2k_wave --config C2K --per-launch --no-cpu-baseline --no-parity
    AIPSTACK_CHKSUM_WAVES_PER_CU=128 bench c2k_w128 --config C2K --per-launch --no-cpu-baseline --no-parity
  done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_C2K" -o run \
      -- python3 bench.py --config C2K --no-cpu-baseline --no-parity > "$out/prof_C2K.log" 2>&1
  ;;
ssweep)
  # ring slots: chunk size, waves, gathered vs wave mode (tools/slot_sweep.py, interleaved)
  timeout -k 10 400 python tools/slot_sweep.py --config C2K --variants \
"stream=-1;stream=-1,chunk_packets=16,chunks_per_wave=1;stream=-1,chunk_packets=8,chunks_per_wave=1;\
stream=-1,chunk_packets=32,chunks_per_wave=1;stream=-1,chunk_packets=16,chunks_per_wave=1,packets=4;\
stream=-1,chunk_packets=16,chunks_per_wave=1,unroll=1;stream=-1,chunk_packets=16,chunks_per_wave=2;\
stream=4,chunk_packets=16,chunks_per_wave=1;stream=4,chunks_per_wave=1" > "$out/c2k.jsonl" 2> "$out/c2k.err"
  timeout -k 10 400 python tools/slot_sweep.py --config RX2K --variants \
"frames=4;frames=8;frames=4,chunk_packets=16,waves_per_cu=100000;frames=4,chunk_packets=32,waves_per_cu=100000;\
frames=8,chunk_packets=16,waves_per_cu=100000;frames=4,waves_per_cu=100000;frames=2,chunk_packets=16,waves_per_cu=100000;\
frames=4,chunk_packets=8,waves_per_cu=100000" > "$out/rx2k.jsonl" 2> "$out/rx2k.err"
  ;;
coal)
  # ring-slot frames: coalesced header loads + LDS transpose (product) vs per-lane header
  # loads (tools/build/lib_nocoal.so), alternating processes; slot tests first
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      -k "slot" > "$out/pytest_slots.log" 2>&1
  for i in 1 2 3; do
    timeout -k 10 300 python tools/slot_sweep.py --config RX2K --variants "frames=4;frames=8" \
        >> "$out/rx2k_coal.jsonl" 2>> "$out/err"
    timeout -k 10 300 python tools/slot_sweep.py --config RX2K --variants "frames=4;frames=8" \
        --lib tools/build/lib_nocoal.so >> "$out/rx2k_nocoal.jsonl" 2>> "$out/err"
  done
  for c in RX2K C2K; do bench "bench_$c" --config $c --per-launch; done
  # one-pass Tx fill: 2-byte field stores (product) vs whole 16-byte field segments
  # (tools/build/lib_segstore.so), alternating processes; the split fill beside them
  for i in 1 2; do
    bench tx_inplace --config TX --tx-inplace --per-launch --no-cpu-baseline
    AIPSTACK_AMD_LIB=tools/build/lib_segstore.so bench tx_inplace_seg --config TX --tx-inplace \
        --per-launch --no-cpu-baseline
    bench tx_split --config TX --per-launch --no-cpu-baseline
  done
  ;;
fsweep)
  # ring-slot frames: segments per lane up front (unroll 1/2), frames in flight, chunk size
  timeout -k 10 600 python tools/slot_sweep.py --config RX2K --variants \
"frames=4;frames=4,unroll=1;frames=8,unroll=1;frames=2,unroll=1;frames=8;\
frames=4,unroll=1,chunk_packets=64,waves_per_cu=100000;frames=8,unroll=1,chunk_packets=64,waves_per_cu=100000;\
frames=4,unroll=1,chunk_packets=16,waves_per_cu=100000" > "$out/rx2k.jsonl" 2> "$out/rx2k.err"
  bench bench_RX2K --config RX2K --per-launch
  ;;
txnt)
  # split Tx fill: the scatter pass's 2-byte field stores plain (product) vs nontemporal
  # (tools/build/lib_scatter_nt.so, -DAIPSTACK_TX_STORE_MODE=1), alternating processes;
  # then rocprof per pass for both
  for i in 1 2 3; do
    bench tx_split --config TX --steps 100 --per-launch --no-cpu-baseline
    AIPSTACK_AMD_LIB=tools/build/lib_scatter_nt.so bench tx_split_nt --config TX --steps 100 \
        --per-launch --no-cpu-baseline
  done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_TX" -o run \
      -- python3 bench.py --config TX --no-cpu-baseline --no-parity > "$out/prof_TX.log" 2>&1
  AIPSTACK_AMD_LIB=tools/build/lib_scatter_nt.so timeout -k 10 300 rocprofv3 --kernel-trace \
      --stats --output-format csv -d "$out/prof_TX_nt" -o run \
      -- python3 bench.py --config TX --no-cpu-baseline --no-parity > "$out/prof_TX_nt.log" 2>&1
  ;;
ring)
  # receive rings through the host engine (RX2K / C2K, 2048-B slots): each slot's used prefix
  # as a 2-D copy (product) vs whole slots (AIPSTACK_ENGINE_SLOT_ROWS=0), registered and
  # pageable; the CSR RX line beside them (same frames back to back)
  for i in 1 2; do
    for c in RX2K C2K; do
      bench e2e_ring --e2e --config $c --steps 5 --warmup 1
      AIPSTACK_ENGINE_SLOT_ROWS=0 bench e2e_ring_full --e2e --config $c --steps 5 --warmup 1
    done
  done
  bench e2e_ring --e2e --e2e-pageable --config RX2K --steps 3 --warmup 1
  AIPSTACK_ENGINE_SLOT_ROWS=0 bench e2e_ring_full --e2e --e2e-pageable --config RX2K --steps 3 --warmup 1
  bench e2e_rx --e2e --config RX --steps 5 --warmup 1
  ;;
asweep)
  # config A / B launch shapes, interleaved in one process per config (tools/sweep.py): the
  # default against more windows in flight, smaller chunks (more waves), runs of chunks
  v="stream=0;stream=4;stream=8;chunk_packets=32,stream=2;chunk_packets=32,stream=4;\
chunk_packets=16,stream=4;waves_per_cu=32;waves_per_cu=16,stream=4"
  for c in A B; do
    timeout -k 10 300 python tools/sweep.py --config $c --rounds 6 --variants "$v" \
        > "$out/sweep_$c.jsonl" 2> "$out/sweep_$c.err"
  done
  timeout -k 10 120 tools/build/hbm_peak > "$out/hbm_peak.jsonl"
  ;;
e2ethreads)
  # host engine: threads for the Tx record apply / pageable staging (8 = default, 16, 32),
  # and the piece size / stream count for the Tx fill, alternating
  for i in 1 2; do
    for t in 8 16 32; do
      AIPSTACK_ENGINE_HOST_THREADS=$t bench tx_t$t --e2e --config TX --steps 5 --warmup 1
      AIPSTACK_ENGINE_HOST_THREADS=$t bench txp_t$t --e2e --e2e-pageable --config TX --steps 3 --warmup 1
    done
    bench tx_c32 --e2e --config TX --steps 5 --warmup 1 --e2e-chunk-mib 32
    bench tx_s8 --e2e --config TX --steps 5 --warmup 1 --e2e-streams 8
    bench rx --e2e --config RX --steps 5 --warmup 1
  done
  ;;
tx2k)
  # a send ring (TX2K): the in-place slotted fill on the device (+ its rocprof stats), and
  # through the host engine (registered / pageable)
  bench bench_TX2K --config TX2K --per-launch
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_TX2K" -o run \
      -- python3 bench.py --config TX2K --no-cpu-baseline --no-parity > "$out/prof_TX2K.log" 2>&1
  bench e2e_tx2k --e2e --config TX2K --steps 5 --warmup 1
  bench e2e_tx2k --e2e --e2e-pageable --config TX2K --steps 3 --warmup 1
  ;;
ringloop)
  # the engine driven as a TAP receive loop (tools/ring_loop.cpp): 8 regions of B slots, 7
  # batches in flight, per batch size B
  timeout -k 10 400 tools/build/ring_loop 64 256 1024 4096 16384 65536 > "$out/ring_loop.jsonl" \
      2> "$out/ring_loop.err"
  ;;
zc)
  # engine pieces of at most AIPSTACK_ENGINE_ZERO_COPY_SMALL packets: offsets / lengths read and
  # results written by the kernel in the pinned staging (no metadata copies); with
  # AIPSTACK_ENGINE_ZERO_COPY=1 the kernel also reads registered packet bytes in place.
  # The engine tests with every piece zero-copy (both levels), then the receive loop in the
  # three modes, alternating
  AIPSTACK_ENGINE_ZERO_COPY=0 AIPSTACK_ENGINE_ZERO_COPY_SMALL=100000000 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
      -k "engine" --timeout 120 --timeout-method thread > "$out/pytest_engine_zc.log" 2>&1
  AIPSTACK_ENGINE_ZERO_COPY=1 AIPSTACK_ENGINE_ZERO_COPY_SMALL=100000000 timeout -k 10 600 \
      python -u -m pytest tests -m gpu -x -q -k "engine" --timeout 120 --timeout-method thread \
      > "$out/pytest_engine_zcb.log" 2>&1
  for i in 1 2; do
    AIPSTACK_ENGINE_ZERO_COPY=0 AIPSTACK_ENGINE_ZERO_COPY_SMALL=0 timeout -k 10 400 \
        tools/build/ring_loop 64 256 1024 4096 16384 >> "$out/ring_loop.jsonl" 2>> "$out/err"
    AIPSTACK_ENGINE_ZERO_COPY=0 AIPSTACK_ENGINE_ZERO_COPY_SMALL=65536 timeout -k 10 400 tools/build/ring_loop 64 256 1024 4096 16384 \
        >> "$out/ring_loop_zc.jsonl" 2>> "$out/err"
    AIPSTACK_ENGINE_ZERO_COPY=1 AIPSTACK_ENGINE_ZERO_COPY_SMALL=65536 timeout -k 10 400 \
        tools/build/ring_loop 64 256 1024 4096 16384 >> "$out/ring_loop_zcb.jsonl" 2>> "$out/err"
  done
  ;;
zc2)
  # whole batches from registered memory: DMA (default) vs every piece zero-copy (the kernel
  # reads the caller's bytes over the link), alternating
  for i in 1 2; do
    for c in A C RX TX RX2K TX2K C2K; do
      AIPSTACK_ENGINE_ZERO_COPY=0 AIPSTACK_ENGINE_ZERO_COPY_SMALL=0 \
          bench e2e_dma --e2e --config $c --steps 5 --warmup 1
      AIPSTACK_ENGINE_ZERO_COPY=1 AIPSTACK_ENGINE_ZERO_COPY_SMALL=100000000 \
          bench e2e_zcb --e2e --config $c --steps 5 --warmup 1
    done
  done
  ;;
txtouch)
  # split Tx fill: per-lane header loads (product) vs headers captured from the stream with
  # the field lines loaded up front at the default policy (tools/build/lib_txtouch.so,
  # tools/experiments/tx_touch_field_lines.patch) vs captured without them; alternating
  for i in 1 2 3; do
    bench tx_split --config TX --steps 100 --per-launch --no-cpu-baseline
    AIPSTACK_AMD_LIB=tools/build/lib_txtouch.so AIPSTACK_CHKSUM_TX_GATHER=1 bench tx_touch \
        --config TX --steps 100 --per-launch --no-cpu-baseline
    AIPSTACK_CHKSUM_TX_GATHER=1 bench tx_gather --config TX --steps 100 --per-launch --no-cpu-baseline
  done
  AIPSTACK_AMD_LIB=tools/build/lib_txtouch.so AIPSTACK_CHKSUM_TX_GATHER=1 timeout -k 10 300 \
      rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_touch" -o run \
      -- python3 bench.py --config TX --no-cpu-baseline --no-parity > "$out/prof_touch.log" 2>&1
  ;;
txmode)
  # the split fill's header modes (tune tx_gather: 0 per-lane loads = round 2's product,
  # 2 captured + field lines touched = the product now), and the one-pass fill both ways;
  # then the GPU suite
  for i in 1 2 3; do
    bench tx_split --config TX --steps 100 --per-launch --no-cpu-baseline
    AIPSTACK_CHKSUM_TX_GATHER=0 bench tx_split_loads --config TX --steps 100 --per-launch --no-cpu-baseline
    bench tx_inplace --config TX --tx-inplace --steps 100 --per-launch --no-cpu-baseline
    AIPSTACK_CHKSUM_TX_GATHER=2 bench tx_inplace_touch --config TX --tx-inplace --steps 100 \
        --per-launch --no-cpu-baseline
  done
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      > "$out/pytest_gpu.log" 2>&1
  ;;
prows)
  # pageable rings: frame bytes staged and read in place (product) vs whole slots staged and
  # DMA'd (AIPSTACK_ENGINE_PAGEABLE_ROWS=0); then the split Tx fill with a third field-line
  # touch (tools/build/lib_touch3.so) vs the product; the engine tests
  for i in 1 2; do
    for c in RX2K TX2K C2K; do
      bench e2e_prows --e2e --e2e-pageable --config $c --steps 3 --warmup 1
      AIPSTACK_ENGINE_PAGEABLE_ROWS=0 bench e2e_pwhole --e2e --e2e-pageable --config $c --steps 3 --warmup 1
    done
  done
  for i in 1 2 3; do
    bench tx_split --config TX --steps 100 --per-launch --no-cpu-baseline
    AIPSTACK_AMD_LIB=tools/build/lib_touch3.so bench tx_touch3 --config TX --steps 100 --per-launch \
        --no-cpu-baseline
  done
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "engine" --timeout 120 \
      --timeout-method thread > "$out/pytest_engine.log" 2>&1
  ;;
*)
  echo "unknown mode $mode" >&2; exit 2 ;;
esac
echo "r03 $mode done"
