#!/bin/bash
# rocprofv3 kernel-trace --stats (csv) of the inference bench and the bench line itself, for profiles/.
#   bash tools/gpu.sh 600 'bash tools/gpu_r05_prof.sh <tag>'
set -o pipefail
tag=${1:-r05y}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > $out/bench.json 2> $out/bench.err || { echo bench failed; tail -5 $out/bench.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench.json'));print('fp16', d['value'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline']['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o bench -- python3 bench.py --steps 20 --warmup 5 \
    --no-cpu-baseline > $out/prof.log 2>&1 || { echo "rocprof failed"; tail -5 $out/prof.log; exit 1; }
echo done
