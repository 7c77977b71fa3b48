#!/bin/bash
# Training-step A/B of the two wgrad kernels on one box: the GPU training tests, then the train bench with the
# LDS-DMA ring kernel (default) and with the register-staged kernel.
#   bash tools/gpu.sh 900 "bash tools/gpu_wgrad_ab.sh <tag>"
set -o pipefail
out=gpurun_out/${1:-wgab}
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread > $out/pytest_train.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $out/pytest_train.log | head; exit 1; }
tail -1 $out/pytest_train.log
for a in 1 0; do
  timeout -k 10 300 python bench.py --mode train --kernel-breakdown --wgrad-algo $a > $out/bench_train_w$a.json 2> $out/bench_train_w$a.err || { echo bench failed; tail -5 $out/bench_train_w$a.err; exit 1; }
  python -c "import json;d=json.load(open('$out/bench_train_w$a.json'));print('wgrad-algo $a', d['value'], d['ms_per_step'])"
  grep "family\] conv_wgrad" $out/bench_train_w$a.err
done
