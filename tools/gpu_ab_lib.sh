#!/bin/bash
# Same-box A/B of the full bench: the in-tree library against a baseline library (deep-rawburst-sr_amd/libdbsr_hip_base.so,
# built from an earlier commit's sources), alternating, N rounds.  bash tools/gpu.sh 900 'bash tools/gpu_ab_lib.sh 3'
set -o pipefail
export TMPDIR=/tmp
B=deep-rawburst-sr_amd/libdbsr_hip_base.so
for i in $(seq ${1:-2}); do
  DBSR_HIP_LIB=$B timeout -k 10 200 python bench.py --no-cpu-baseline --no-op-timing > gpurun_out/ab_base.json || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab_base.json'));print('bench base', d['value'])"
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-op-timing > gpurun_out/ab_new.json || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab_new.json'));print('bench new ', d['value'])"
done
