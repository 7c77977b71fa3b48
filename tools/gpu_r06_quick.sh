#!/bin/bash
# Quick kernel iteration: the K-split / tiled split-K tests and the engine-level tests, then the bench with the
# per-op breakdown.   bash tools/gpu.sh 900 'bash tools/gpu_r06_quick.sh <tag>'
set -o pipefail
tag=${1:-r06q}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ks128.py tests/test_gpu_e2e.py tests/test_gpu_parity.py -x -v --timeout 200 \
    --timeout-method thread > $out/pytest.log 2>&1 || { echo "tests failed rc=$?"; grep -E "FAIL|Error|assert" $out/pytest.log | head; tail -3 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 300 python bench.py --kernel-breakdown --no-cpu-baseline > $out/bench.json 2> $out/bench.err || { echo bench failed; tail -20 $out/bench.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench.json'));print('fp16', d['value'], d['ms_per_step'])"
grep -E "dec.init|dense4|^\[family\]" $out/bench.err | head -12
