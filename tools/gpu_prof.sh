#!/bin/bash
# Bench with the per-op breakdown (in-step and whole-chip), then a rocprofv3 kernel trace of graph replays only.
#   bash tools/gpu.sh 900 'bash tools/gpu_prof.sh <tag> [bench args]'
set -o pipefail
tag=${1:-r04}
shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --kernel-breakdown --no-cpu-baseline "$@" > $out/bench.json 2> $out/bench.err || { echo bench failed; tail -20 $out/bench.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench.json'));print('value', d['value'], d['ms_per_step'], 'roof', d['roofline']['kernel'][:20], d['roofline']['frac'], 'chip', d['roofline_whole_chip']['frac'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-op-timing "$@" > $out/trace.log 2>&1 || { echo trace failed; tail -5 $out/trace.log; exit 1; }
echo done
