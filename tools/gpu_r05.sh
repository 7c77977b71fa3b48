#!/bin/bash
# Round-5 GPU session: the fused weight-predictor kernel's tests first, then the whole -m gpu suite, then the
# bench with the per-op breakdown.  Each GPU step has its own limit; the chain stops at the first failure.
#   bash tools/gpu.sh 1100 'bash tools/gpu_r05.sh <tag> [extra bench args]'
# FIRST=<test file> replaces the first test file; SUITE=<pytest -k expr> narrows the -m gpu suite (SUITE=none
# skips it).
set -o pipefail
tag=${1:-r05a}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest ${FIRST:-tests/test_gpu_fuse.py} -x -v --timeout 120 --timeout-method thread \
    > $out/pytest_fuse.log 2>&1 || { echo "fuse tests failed rc=$?"; grep -E "FAIL|Error|assert|Mismatch" $out/pytest_fuse.log | head -30; tail -5 $out/pytest_fuse.log; exit 1; }
tail -1 $out/pytest_fuse.log
if [ "${SUITE:-all}" != none ]; then
    kexpr=(); [ "${SUITE:-all}" != all ] && kexpr=(-k "$SUITE")
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread "${kexpr[@]}" \
        > $out/pytest.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "FAIL|Error|assert" $out/pytest.log | head -30; tail -5 $out/pytest.log; exit 1; }
    tail -1 $out/pytest.log; grep "precision vs oracle" $out/pytest.log || true
fi
timeout -k 10 300 python bench.py --kernel-breakdown --no-cpu-baseline ${@:2} > $out/bench.json 2> $out/bench.err || { echo bench failed; tail -20 $out/bench.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench.json'));print('fp16', d['value'], d['ms_per_step'], {k: v['frac'] for k, v in d['roofline_families'].items()})"
grep "^\[family\]" $out/bench.err | head -14
echo done
