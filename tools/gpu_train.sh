#!/bin/bash
# GPU session for the training path: the training / conv-variant GPU tests, then the training bench with its
# per-op breakdown.  Each GPU step has its own time limit; the chain stops at the first failure.
#   bash tools/gpu.sh 900 'bash tools/gpu_train.sh <tag>'
set -o pipefail
tag=${1:-r03t}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_parity.py -x -v --timeout 300 \
    --timeout-method thread -k "${2:-train or ws_conv or pipe_epilogue or warp_backward or chan_sum or dgrad or wgrad}" \
    > $out/pytest.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "FAIL|Error|assert" $out/pytest.log | head -30; tail -5 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 300 python bench.py --mode train --steps 5 --warmup 2 --kernel-breakdown > $out/bench_train.json 2> $out/bench_train.err || { echo bench train failed; tail -20 $out/bench_train.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench_train.json'));print('train', d['value'], d['ms_per_step'], d['step_roofline'])"
grep "^\[family\]" $out/bench_train.err | head -20
echo done
