# FETCH_SIZE calibration of the frame kernels' per-lane header loads (tools/fetch_calib.hip).
export TMPDIR=/tmp; o=gpurun_out/r01g/${1:-fetch_calib}; mkdir -p $o
timeout -k 10 60 tools/build/fetch_calib > $o/times.jsonl 2> $o/times.err &&
timeout -s KILL 60 rocprofv3 --kernel-trace --output-format csv -d $o/fetch -o run --pmc FETCH_SIZE -- tools/build/fetch_calib > $o/fetch.log 2>&1 &&
timeout -s KILL 60 rocprofv3 --kernel-trace --output-format csv -d $o/rdreq -o run --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -- tools/build/fetch_calib > $o/rdreq.log 2>&1
