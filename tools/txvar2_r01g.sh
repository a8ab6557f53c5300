# Tx split vs in-place across waves per CU (chunks per wave), and the no-record floor.
export TMPDIR=/tmp; o=gpurun_out/r01g/txvar2; mkdir -p $o
V="4,128,8;4,64,8;4,32,8;4,16,8;4,8,8"
timeout -k 10 200 python tools/sweep.py --config TX --variants "$V" > $o/split.jsonl 2> $o/split.err &&
timeout -k 10 200 python tools/sweep.py --config TX --variants "$V" --tx-inplace > $o/inplace.jsonl 2> $o/inplace.err &&
timeout -k 10 200 python tools/sweep.py --config RX --variants "$V" > $o/rx.jsonl 2> $o/rx.err
