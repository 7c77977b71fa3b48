#!/bin/bash
# Per-op in-step / whole-chip breakdown of the inference bench and the training step.
#   bash tools/gpu.sh 900 'bash tools/gpu_r06_breakdown.sh <tag> [train]'
set -o pipefail
tag=${1:-r06b}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 300 python bench.py --kernel-breakdown --no-cpu-baseline > $out/bench.json 2> $out/bench.err || { echo bench failed; tail -20 $out/bench.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench.json'));print('fp16', d['value'], d['ms_per_step'])"
if [ "${2:-}" = train ]; then
  timeout -k 10 300 python bench.py --mode train --kernel-breakdown --no-cpu-baseline > $out/bench_train.json 2> $out/bench_train.err || { echo train failed; tail -20 $out/bench_train.err; exit 1; }
  python -c "import json;d=json.load(open('$out/bench_train.json'));print('train', d['value'], d['ms_per_step'])"
fi
