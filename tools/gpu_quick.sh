#!/bin/bash
# Quick GPU check: the whole -m gpu suite, then the training bench with the per-op breakdown.
#   bash tools/gpu.sh 900 "bash tools/gpu_quick.sh <tag>"
set -o pipefail
out=gpurun_out/${1:-quick}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $out/pytest.log | head -10; tail -3 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 300 python bench.py --mode train --kernel-breakdown > $out/bench_train.json 2> $out/bench_train.err || { echo bench train failed; tail -20 $out/bench_train.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench_train.json'));print('train', d['value'], d['ms_per_step'], d['step_roofline']['frac'])"
