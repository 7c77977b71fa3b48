#!/bin/bash
# GPU session for an inference-kernel change: the conv-variant / bench-shape / e2e GPU tests, then the bench
# with the per-op breakdown.  Each GPU step has its own time limit; the chain stops at the first failure.
#   bash tools/gpu.sh 900 'bash tools/gpu_infer.sh <tag> [pytest -k expr]'
set -o pipefail
tag=${1:-r03i}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_e2e.py tests/test_gpu_ops.py -x -v --timeout 300 \
    --timeout-method thread -k "${2:-ws_conv or pipe_epilogue or two_lanes or bench_shape or e2e or conv}" \
    > $out/pytest.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "FAIL|Error|assert" $out/pytest.log | head -30; tail -5 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 300 python bench.py --kernel-breakdown --no-cpu-baseline > $out/bench.json 2> $out/bench.err || { echo bench failed; tail -20 $out/bench.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench.json'));print('fp16', d['value'], d['ms_per_step'], {k: v['frac'] for k, v in d['roofline_families'].items()})"
grep "^\[family\]" $out/bench.err | head -12
echo done
