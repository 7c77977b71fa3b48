#!/bin/bash
# Final validation of the shipped build: the whole -m gpu suite, smoke(), the fp16 bench and the training bench.
#   bash tools/gpu.sh 900 'bash tools/gpu_r06_close.sh <tag>'
set -o pipefail
tag=${1:-r06zz}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu --maxfail 5 -v -s --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 \
    || { echo "suite failed rc=$?"; grep -E "FAIL|Error|assert" $out/pytest.log | head -20; tail -3 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log; grep "precision vs oracle" $out/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo smoke failed; tail -20 $out/smoke.log; exit 1; }
grep smoke: $out/smoke.log
timeout -k 10 300 python bench.py > $out/bench.json 2> $out/bench.err || { echo bench failed; tail -20 $out/bench.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench.json'));print('fp16', d['value'], d['ms_per_step'], d['roofline']['frac'], d['conv_all']['step_frac'], d['cpu_baseline']['value'])"
timeout -k 10 300 python bench.py --mode train --no-cpu-baseline > $out/bench_train.json 2> $out/bench_train.err || { echo train failed; tail -20 $out/bench_train.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench_train.json'));print('train', d['value'], d['ms_per_step'])"
echo done
