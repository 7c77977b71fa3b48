#!/bin/bash
# Round-6 closing session: the whole -m gpu suite, smoke(), the fp16 bench with the per-op breakdown, the training
# bench, a rocprofv3 kernel trace of the bench and the FETCH / WRITE PMC passes (separate runs).
#   bash tools/gpu.sh 1150 'bash tools/gpu_r06_final.sh <tag>'
set -o pipefail
tag=${1:-r06z}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu --maxfail 5 -v -s --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 \
    || { echo "suite failed rc=$?"; grep -E "FAIL|Error|assert" $out/pytest.log | head -20; tail -3 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log; grep "precision vs oracle" $out/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo smoke failed; tail -20 $out/smoke.log; exit 1; }
tail -3 $out/smoke.log
timeout -k 10 300 python bench.py --kernel-breakdown > $out/bench.json 2> $out/bench.err || { echo bench failed; tail -20 $out/bench.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench.json'));print('fp16', d['value'], d['ms_per_step'], d['roofline']['frac'], d['conv_all']['step_frac'], d.get('cpu_baseline',{}) and d['cpu_baseline']['value'])"
timeout -k 10 300 python bench.py --mode train --kernel-breakdown --no-cpu-baseline > $out/bench_train.json 2> $out/bench_train.err || { echo train failed; tail -20 $out/bench_train.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench_train.json'));print('train', d['value'], d['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof/trace -o run --output-format csv -- python3 bench.py --steps 10 \
    --warmup 3 --no-cpu-baseline --no-op-timing > $out/prof.log 2>&1 || { echo "rocprof failed"; tail -5 $out/prof.log; exit 1; }
re="ks128|warp512|warp_kernel|fuse_softmax|fuse512|conv3x3|conv1x1|upsample_shuffle|upsample_blur|resblock|conv_fuse|conv2d_kernel|pwc_dense|pwc_extract"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$re" -d $out/prof/pmc_fetch -o run --output-format csv \
    -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-op-timing > $out/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; tail -5 $out/pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$re" -d $out/prof/pmc_write -o run --output-format csv \
    -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-op-timing > $out/pmc_write.log 2>&1 || { echo "pmc write failed"; tail -5 $out/pmc_write.log; exit 1; }
echo done
