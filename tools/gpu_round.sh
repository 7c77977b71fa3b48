#!/bin/bash
# Measurement session on one box: GPU tests, smoke, the bench legs (fp16 default with the CPU baseline and the
# per-op breakdown, bf16, training), then the rocprofv3 kernel-trace + PMC profile of the same binary.
#   bash tools/gpu.sh 1150 'bash tools/gpu_round.sh <tag>'
set -o pipefail
tag=${1:-r04}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread \
    > $out/pytest.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "FAIL|Error" $out/pytest.log | head -20; tail -5 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo smoke failed; tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 300 python bench.py --kernel-breakdown > $out/bench_fp16.json 2> $out/bench_fp16.err || { echo bench fp16 failed; tail -20 $out/bench_fp16.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench_fp16.json'));print('fp16', d['value'], d['ms_per_step'], d['roofline']['kernel'][:20], d['roofline']['frac'], d['roofline_whole_chip']['frac'], d['cpu_baseline']['value'])"
timeout -k 10 300 python bench.py --dtype bf16 --no-cpu-baseline --no-op-timing > $out/bench_bf16.json 2> $out/bench_bf16.err || { echo bench bf16 failed; exit 1; }
python -c "import json;d=json.load(open('$out/bench_bf16.json'));print('bf16', d['value'], d['ms_per_step'])"
timeout -k 10 300 python bench.py --mode train --kernel-breakdown > $out/bench_train.json 2> $out/bench_train.err || { echo bench train failed; tail -20 $out/bench_train.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench_train.json'));print('train', d['value'], d['ms_per_step'], d['step_roofline']['frac'])"
bash tools/profile.sh $tag || { echo profile failed; exit 1; }
echo done
