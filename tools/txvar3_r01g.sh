# Split Tx with the status in the record (one store per frame in the read pass).
export TMPDIR=/tmp; o=gpurun_out/r01g/txvar3; mkdir -p $o
V="4,128,8;4,64,8"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "tx_fill or fill_then" --timeout 120 --timeout-method thread > $o/pytest_tx.log 2>&1 &&
timeout -k 10 200 python tools/sweep.py --config TX --variants "$V" > $o/split.jsonl 2> $o/split.err &&
timeout -k 10 200 python tools/sweep.py --config TX --variants "$V" --tx-inplace > $o/inplace.jsonl 2> $o/inplace.err &&
timeout -k 10 200 python tools/sweep.py --config TX --variants "$V" --lib tools/build/lib_recnone2.so > $o/recnone2.jsonl 2> $o/recnone2.err &&
timeout -k 10 200 python tools/sweep.py --config TX --variants "$V" > $o/split_b.jsonl 2> $o/split_b.err
