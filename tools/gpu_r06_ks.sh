#!/bin/bash
# K-split 128-channel kernel: its tests, the microbenchmark against the pipelined kernel, a short bench line.
#   bash tools/gpu.sh 900 'bash tools/gpu_r06_ks.sh <tag>'
set -o pipefail
tag=${1:-r06k}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ks128.py -x -v --timeout 120 --timeout-method thread > $out/pytest_ks.log 2>&1 \
    || { echo "ks tests failed"; grep -E "FAIL|Error|assert" $out/pytest_ks.log | head -20; tail -5 $out/pytest_ks.log; exit 1; }
tail -1 $out/pytest_ks.log
timeout -k 10 200 python -u tools/bench_conv.py --only "128->128" --algos 2,5 > $out/bench_conv.txt 2>&1 || { echo "bench_conv failed"; tail -10 $out/bench_conv.txt; exit 1; }
cat $out/bench_conv.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $out/bench.json 2> $out/bench.err || { echo bench failed; tail -20 $out/bench.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench.json'));print('fp16', d['value'], d['ms_per_step'])"
