#!/bin/bash
# bench.py at several lane-0 CU caps (DBSR_LANE0_CUS) in one GPU call
for c in 0 224 192 160 128; do
  DBSR_LANE0_CUS=$c timeout -k 10 150 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/lane0_$c.json 2> gpurun_out/lane0_$c.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/lane0_$c.json'));print('cap $c', d['value'], d['ms_per_step'])"
done
