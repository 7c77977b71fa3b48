#!/bin/bash
set -o pipefail
j() { python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['value'], d['ms_per_step'])" "$@"; }
timeout -k 10 150 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/ov_a.json 2>/dev/null || exit $?; j gpurun_out/ov_a.json default
DBSR_NO_SPLITK=1 timeout -k 10 150 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/ov_b.json 2>/dev/null || exit $?; j gpurun_out/ov_b.json nosplitk
DBSR_NO_SPLITK=1 DBSR_MAIN_FIRST=0 timeout -k 10 150 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/ov_c.json 2>/dev/null || exit $?; j gpurun_out/ov_c.json nosplitk_sidefirst
DBSR_NO_SPLITK=1 timeout -k 10 150 python bench.py --no-cpu-baseline --steps 30 --no-graph > gpurun_out/ov_d.json 2>/dev/null || exit $?; j gpurun_out/ov_d.json nosplitk_eager
