#!/bin/bash
# Lane timeline of one eager bench-shape forward (tools/lane_events.py) plus a short bench line.
#   bash tools/gpu.sh 600 'bash tools/gpu_r06_timeline.sh <tag>'
set -o pipefail
tag=${1:-r06t}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 240 python -u tools/lane_events.py --reps 3 > $out/lanes.txt 2>&1 || { echo "lanes failed"; tail -20 $out/lanes.txt; exit 1; }
tail -4 $out/lanes.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $out/bench.json 2> $out/bench.err || { echo bench failed; tail -20 $out/bench.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench.json'));print('fp16', d['value'], d['ms_per_step'])"
