#!/bin/bash
# Round-5 closing session: the training-step tests (train_ops changed), bench on the product build and on the
# build without DBSR_OWN_SIMDS (co-residency A/B), the training bench, and a rocprofv3
# kernel-trace --stats of the inference bench (csv, for profiles/).   bash tools/gpu.sh 1150 'bash tools/gpu_r05_final.sh <tag>'
set -o pipefail
tag=${1:-r05w}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_train.py -v --maxfail 3 --timeout 300 --timeout-method thread \
    > $out/pytest_train.log 2>&1 || { echo "train tests failed rc=$?"; grep -E "FAIL|Error|assert" $out/pytest_train.log | head; exit 1; }
tail -1 $out/pytest_train.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $out/bench.json 2> $out/bench.err || { echo bench failed; tail -5 $out/bench.err; exit 1; }
DBSR_HIP_LIB=deep-rawburst-sr_amd/libdbsr_hip_noown.so timeout -k 10 300 python bench.py --no-cpu-baseline \
    > $out/bench_noown.json 2> $out/bench_noown.err || { echo bench noown failed; tail -5 $out/bench_noown.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline > $out/bench2.json 2>> $out/bench.err || { echo bench failed; exit 1; }
python -c "
import json
for f in ('bench', 'bench_noown', 'bench2'):
    d = json.load(open('$out/%s.json' % f)); print(f, d['value'], d['ms_per_step'])"
timeout -k 10 400 python bench.py --mode train --no-cpu-baseline > $out/bench_train.json 2> $out/bench_train.err || { echo train bench failed; tail -5 $out/bench_train.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench_train.json'));print('train', d['value'], d['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o bench -- python3 bench.py --steps 20 --warmup 5 \
    --no-cpu-baseline > $out/prof.log 2>&1 || { echo "rocprof failed"; tail -5 $out/prof.log; exit 1; }
echo done
