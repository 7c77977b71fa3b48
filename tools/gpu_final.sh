#!/bin/bash
# Round-end GPU session: every GPU test, the smoke test, the bench legs (fp16 default with the CPU baseline,
# bf16, training).  Each GPU step has its own time limit; the chain stops at the first failure.
#   bash tools/gpu.sh 1100 'bash tools/gpu_final.sh <tag>'
set -o pipefail
tag=${1:-r03z}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread \
    > $out/pytest.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "FAIL|Error" $out/pytest.log | head -20; tail -5 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo smoke failed; tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 300 python bench.py --kernel-breakdown > $out/bench_fp16.json 2> $out/bench_fp16.err || { echo bench fp16 failed; tail -20 $out/bench_fp16.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench_fp16.json'));print('fp16', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic'], d['cpu_baseline']['value'])"
timeout -k 10 300 python bench.py --dtype bf16 --no-cpu-baseline > $out/bench_bf16.json 2> $out/bench_bf16.err || { echo bench bf16 failed; exit 1; }
python -c "import json;d=json.load(open('$out/bench_bf16.json'));print('bf16', d['value'], d['ms_per_step'])"
timeout -k 10 300 python bench.py --mode train --kernel-breakdown > $out/bench_train.json 2> $out/bench_train.err || { echo bench train failed; tail -20 $out/bench_train.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench_train.json'));print('train', d['value'], d['ms_per_step'], d['step_roofline']['frac'])"
echo done
