#!/bin/bash
# The fused upsample + blur: its tests, then the microbenchmark (two launches, fused, ablation variants), then a
# rocprofv3 kernel trace of the fused call.   bash tools/gpu.sh 900 'bash tools/gpu_ub.sh <tag> [variants]'
set -o pipefail
tag=${1:-ubA}; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_upsample_blur.py -x -v --timeout 120 --timeout-method thread \
    > $out/pytest.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" $out/pytest.log | head -20; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 120 python tools/bench_ub.py --two-kernel > $out/out.txt 2>&1 &&
timeout -k 10 120 python tools/bench_ub.py >> $out/out.txt 2>&1 || exit 1
for v in "$@"; do
    DBSR_HIP_LIB=deep-rawburst-sr_amd/libdbsr_hip_$v.so timeout -k 10 120 python tools/bench_ub.py 2>&1 | sed "s/^/$v /" >> $out/out.txt || exit 1
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/prof -o ub -- python tools/bench_ub.py > /dev/null 2>&1
grep -v amdgpu.ids $out/out.txt
