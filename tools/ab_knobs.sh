#!/bin/bash
# interleaved A/B of scheduling knobs: lane-0 CU cap and side-lane stream priority
set -o pipefail
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 150 python bench.py --no-cpu-baseline --steps 40 > gpurun_out/k_$tag.json 2> gpurun_out/k_$tag.err || exit $?
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/k_$tag.json "$tag"
}
for i in 1 2; do
  run cap176_$i DBSR_LANE0_CUS=176
  run cap192_$i DBSR_LANE0_CUS=192
  run cap208_$i DBSR_LANE0_CUS=208
  run prio0_$i DBSR_LANE0_CUS=192 DBSR_SIDE_PRIO=0
done
