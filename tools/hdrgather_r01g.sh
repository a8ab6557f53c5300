# Header segments gathered from the stream windows (LDS ring) vs loaded before the stream
# (tools/build/lib_old.so = the frame kernel without the patch; the product build = with tools/experiments/hdr_gather_*.patch or hdr_loads_behind_stream.patch applied): parity, time, FETCH_SIZE.
export TMPDIR=/tmp; o=gpurun_out/r01g/${1:-hdrgather}; mkdir -p $o; V="4,128,8"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "tx_fill or rx_verify or fill_then or frame or cpp_capi" --timeout 120 --timeout-method thread > $o/pytest_frames.log 2>&1 || exit 1
for pass in 1 2; do
  for c in RX TX; do
    timeout -k 10 200 python tools/sweep.py --config $c --variants "$V" > $o/${c}_new_$pass.jsonl 2>> $o/err || exit 1
    timeout -k 10 200 python tools/sweep.py --config $c --variants "$V" --lib tools/build/lib_old.so > $o/${c}_old_$pass.jsonl 2>> $o/err || exit 1
  done
done
timeout -k 10 300 tools/pmc_run.sh RX $o/pmc_RX || exit 1
