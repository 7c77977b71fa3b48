#!/bin/bash
# Interleaved A/B of one library build with an environment toggle: A = "$VAR=0", B = default.
# usage: bash tools/ab_env.sh VAR [rounds] [extra bench args]
set -o pipefail
VAR=$1; shift
R=${1:-3}; shift
for i in $(seq 1 $R); do
  for v in off on; do
    if [ $v = off ]; then envs="$VAR=0"; else envs="DBSR_AB_DUMMY=1"; fi
    env $envs timeout -k 10 150 python bench.py --no-cpu-baseline --steps 40 "$@" > gpurun_out/ab_$v$i.json 2> gpurun_out/ab_$v$i.err || { echo "[ab] $v$i rc=$?"; tail -5 gpurun_out/ab_$v$i.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));h=d.get('roofline_hbm',{});print(sys.argv[2], d['value'], d['ms_per_step'], 'fuse_us', h.get('fuse',{}).get('us'), 'warp_us', h.get('warp',{}).get('us'))" gpurun_out/ab_$v$i.json $v$i
  done
done
