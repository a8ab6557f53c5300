# Price split Tx read-pass record stores by their width (8/4/2/1/0 bytes per frame).
export TMPDIR=/tmp; o=gpurun_out/r01g/txvar5; mkdir -p $o; V="4,128,8"
for pass in 1 2; do
  timeout -k 10 200 python tools/sweep.py --config TX --variants "$V" > $o/rec8_$pass.jsonl 2>> $o/err || exit 1
  for m in rec3 rec4 rec5 recnone3; do
    timeout -k 10 200 python tools/sweep.py --config TX --variants "$V" --lib tools/build/lib_$m.so > $o/${m}_$pass.jsonl 2>> $o/err || exit 1
  done
done
