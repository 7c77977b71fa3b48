#!/bin/bash
# Split-K tests, the training GPU tests and the training bench with the per-op breakdown.
#   bash tools/gpu.sh 900 'bash tools/gpu_r06_train.sh <tag>'
set -o pipefail
tag=${1:-r06tr}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ks128.py tests/test_gpu_train.py -x -v --timeout 200 \
    --timeout-method thread > $out/pytest.log 2>&1 || { echo "tests failed rc=$?"; grep -E "FAIL|Error|assert" $out/pytest.log | head; tail -3 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 300 python bench.py --mode train --kernel-breakdown --no-cpu-baseline > $out/bench_train.json 2> $out/bench_train.err || { echo train failed; tail -20 $out/bench_train.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench_train.json'));print('train', d['value'], d['ms_per_step'])"
grep "^\[family\]" $out/bench_train.err | head -14
