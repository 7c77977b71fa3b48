for v in "" nodma nomfma; do
  if [ -z "$v" ]; then lib=$PWD/deep-rawburst-sr_amd/libdbsr_hip.so; else lib=$PWD/deep-rawburst-sr_amd/libdbsr_hip_$v.so; fi
  echo "== variant ${v:-base}"
  DBSR_HIP_LIB=$lib timeout -k 10 120 python tools/bench_conv.py --algos 3 --only "enc.res" || exit $?
  DBSR_HIP_LIB=$lib timeout -k 10 120 python tools/bench_conv.py --algos 3 --only "wp.out" || exit $?
  DBSR_HIP_LIB=$lib timeout -k 10 120 python tools/bench_conv.py --algos 3 --only "dec.post" || exit $?
done
