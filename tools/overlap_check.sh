#!/bin/bash
set -o pipefail
j() { python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['value'], d['ms_per_step'])" "$@"; }
timeout -k 10 150 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/ov_a.json 2>gpurun_out/ov_a.err || exit $?; j gpurun_out/ov_a.json default
for k in 32 64 96; do
DBSR_CU_SPLIT=$k timeout -k 10 150 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/ov_s$k.json 2>gpurun_out/ov_s$k.err || exit $?; j gpurun_out/ov_s$k.json cusplit$k
done
