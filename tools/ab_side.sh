#!/bin/bash
# interleaved side-lane CU cap A/B: DBSR_SIDE_CUS in {0, 64, 128}
set -o pipefail
for i in 1 2 3; do
  for c in 0 64 128; do
    DBSR_SIDE_CUS=$c timeout -k 10 150 python bench.py --no-cpu-baseline --steps 40 > gpurun_out/sc_$c$i.json 2> gpurun_out/sc_$c$i.err || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/sc_$c$i.json'));print('side $c', d['value'], d['ms_per_step'])"
  done
done
