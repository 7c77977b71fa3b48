#!/bin/bash
# wgrad change check: the training GPU tests, the wgrad microbenchmark, one PMC pass over the 32-channel wgrad
# (bank conflicts vs LDS-active cycles) and the training bench.   bash tools/gpu.sh 900 'bash tools/gpu_r06_wgrad.sh <tag>'
set -o pipefail
tag=${1:-r06w}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -x -v --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 \
    || { echo "tests failed rc=$?"; grep -E "FAIL|Error|assert" $out/pytest.log | head; tail -3 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 120 python3 tools/bench_wgrad.py --algos 1 > $out/bench_wgrad.log 2>&1 || { echo wgrad bench failed; tail $out/bench_wgrad.log; exit 1; }
grep algo $out/bench_wgrad.log
timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES --kernel-include-regex "conv_wgrad_dma" \
    -d $out/pmc -o run --output-format csv -- python3 tools/bench_wgrad.py --only dec.post --algos 1 --reps 3 > $out/pmc.log 2>&1 \
    || { echo pmc failed; tail -5 $out/pmc.log; exit 1; }
timeout -k 10 300 python bench.py --mode train --kernel-breakdown --no-cpu-baseline > $out/bench_train.json 2> $out/bench_train.err || { echo train failed; tail -20 $out/bench_train.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench_train.json'));print('train', d['value'], d['ms_per_step'])"
grep "^\[family\]" $out/bench_train.err | head -6
echo done
