#!/bin/bash
# per-op times of the generic-conv ops under different DBSR_GENERIC_MIN_BLOCKS targets
set -o pipefail
for mb in 512 1024 2048 4096; do
  DBSR_GENERIC_MIN_BLOCKS=$mb timeout -k 10 150 python bench.py --no-cpu-baseline --steps 20 --kernel-breakdown > gpurun_out/sg_$mb.json 2> gpurun_out/sg_$mb.txt || { echo "[sweep] $mb failed"; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/sg_$mb.json $mb
  grep -E "conv2d_generic|family" gpurun_out/sg_$mb.txt | grep -E "enc.init|ofe.init|proj|family\] conv2d" 
done
