#!/bin/bash
# interleaved lane-0 CU cap A/B: DBSR_LANE0_CUS in {0, 192, 224}
set -o pipefail
for i in 1 2 3; do
  for c in 0 192 224; do
    DBSR_LANE0_CUS=$c timeout -k 10 150 python bench.py --no-cpu-baseline --steps 40 > gpurun_out/l0_$c$i.json 2> gpurun_out/l0_$c$i.err || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/l0_$c$i.json'));print('cap $c', d['value'], d['ms_per_step'])"
  done
done
