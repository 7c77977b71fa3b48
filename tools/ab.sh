#!/bin/bash
# Interleaved A/B of two library builds on one box: A = libdbsr_hip_base.so, B = libdbsr_hip.so
# usage: bash tools/ab.sh [rounds] [extra bench args]
set -o pipefail
R=${1:-3}; shift
for i in $(seq 1 $R); do
  for v in base cur; do
    lib=deep-rawburst-sr_amd/libdbsr_hip_$v.so; [ $v = cur ] && lib=deep-rawburst-sr_amd/libdbsr_hip.so
    DBSR_HIP_LIB=$PWD/$lib timeout -k 10 150 python bench.py --no-cpu-baseline --steps 40 "$@" > gpurun_out/ab_$v$i.json 2> gpurun_out/ab_$v$i.err || { echo "[ab] $v$i rc=$?"; tail -5 gpurun_out/ab_$v$i.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/ab_$v$i.json $v$i
  done
done
