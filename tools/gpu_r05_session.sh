#!/bin/bash
# Round-5 measurement session: the new fused-kernel tests, the whole -m gpu suite (precision lines kept), the
# two-lane race experiment (the bench-shape two-lane bitwise test ONCE on a build without
# DBSR_OWN_SIMDS; a test failure is recorded, anything else ends the session), the bench with the per-op
# breakdown, and a rocprofv3 kernel trace of the bench.   bash tools/gpu.sh 1150 'bash tools/gpu_r05_session.sh <tag>'
set -o pipefail
tag=${1:-r05s}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_resblock.py tests/test_gpu_upsample_blur.py -x -v --timeout 120 \
    --timeout-method thread > $out/pytest_new.log 2>&1 || { echo "new tests failed rc=$?"; grep -E "FAIL|Error|assert" $out/pytest_new.log | head; exit 1; }
tail -1 $out/pytest_new.log
timeout -k 10 700 python -u -m pytest tests -m gpu --maxfail 5 -v -s --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 \
    || { echo "suite failed rc=$?"; grep -E "FAIL|Error|assert" $out/pytest.log | head -20; tail -3 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log; grep "precision vs oracle" $out/pytest.log
DBSR_HIP_LIB=deep-rawburst-sr_amd/libdbsr_hip_noown.so timeout -k 10 300 python -u -m pytest \
    "tests/test_gpu_parity.py::test_bench_shape_two_lanes_bitwise" -x -v --timeout 240 --timeout-method thread \
    > $out/pytest_noown.log 2>&1
rc=$?
echo "two-lane bitwise without DBSR_OWN_SIMDS: rc=$rc"; tail -3 $out/pytest_noown.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 300 python bench.py --kernel-breakdown > $out/bench.json 2> $out/bench.err || { echo bench failed; tail -20 $out/bench.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench.json'));print('fp16', d['value'], d['ms_per_step'], d.get('cpu_baseline'))"
grep "^\[family\]" $out/bench.err | head -16
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o bench -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline \
    > $out/prof.log 2>&1 || { echo "rocprof failed"; tail -5 $out/prof.log; exit 1; }
echo done
