export TMPDIR=/tmp; o=gpurun_out/r01g/txvar; mkdir -p $o
for pass in 1 2; do
  timeout -k 10 200 python bench.py --config TX --steps 20 --no-parity > $o/split_$pass.json 2>>$o/err || exit 1
  timeout -k 10 200 python bench.py --config TX --steps 20 --no-parity --tx-inplace > $o/inplace_$pass.json 2>>$o/err || exit 1
  AIPSTACK_AMD_LIB=$PWD/tools/build/lib_recnt.so timeout -k 10 200 python bench.py --config TX --steps 20 --no-parity > $o/recnt_$pass.json 2>>$o/err || exit 1
  AIPSTACK_AMD_LIB=$PWD/tools/build/lib_recnone.so timeout -k 10 200 python bench.py --config TX --steps 20 --no-parity > $o/recnone_$pass.json 2>>$o/err || exit 1
  AIPSTACK_AMD_LIB=$PWD/tools/build/lib_stnone.so timeout -k 10 200 python bench.py --config TX --steps 20 --no-parity --tx-inplace > $o/stnone_$pass.json 2>>$o/err || exit 1
  timeout -k 10 200 python bench.py --config RX --steps 20 --no-parity > $o/rx_$pass.json 2>>$o/err || exit 1
done
