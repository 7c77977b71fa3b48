#!/bin/bash
# warp kernel pixels-per-wave sweep (DBSR_WARP_PPW), interleaved
set -o pipefail
for i in 1 2; do
for ppw in 2 4 8; do
  DBSR_WARP_PPW=$ppw timeout -k 10 150 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/sw_$ppw.json 2> gpurun_out/sw_$ppw.err || { echo "[sweep] $ppw failed"; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));h=d['roofline_hbm'];print(sys.argv[2], d['value'], 'warp_us', h['warp']['us'])" gpurun_out/sw_$ppw.json $ppw
done
done
