#!/bin/bash
# One GPU-box session: GPU tests, then the bench legs.  Each GPU step has its own time limit and the chain
# stops at the first failure (no retries).  Usage (from the build container):
#   bash tools/gpu.sh 900 'bash tools/gpu_check.sh <tag> [pytest -k expr]'
set -o pipefail
tag=${1:-r03}
kexpr=${2:-}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
if [ -n "$kexpr" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$kexpr" \
      > $out/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $out/pytest.log; exit 1; }
else
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread \
      > $out/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $out/pytest.log; exit 1; }
fi
tail -3 $out/pytest.log
timeout -k 10 300 python bench.py --kernel-breakdown > $out/bench_fp16.json 2> $out/bench_fp16.err || { echo bench fp16 failed; tail -20 $out/bench_fp16.err; exit 1; }
cat $out/bench_fp16.json
timeout -k 10 300 python bench.py --dtype bf16 --no-cpu-baseline > $out/bench_bf16.json 2> $out/bench_bf16.err || { echo bench bf16 failed; exit 1; }
python -c "import json;d=json.load(open('$out/bench_bf16.json'));print('bf16', d['value'], d['ms_per_step'])"
timeout -k 10 300 python bench.py --mode train --steps 5 --warmup 2 --kernel-breakdown > $out/bench_train.json 2> $out/bench_train.err || { echo bench train failed; tail -20 $out/bench_train.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench_train.json'));print('train', d['value'], d['ms_per_step'], d['step_roofline'])"
echo done
