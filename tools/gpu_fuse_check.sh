#!/bin/bash
# conv_fuse change: its parity tests, then the microbench (two-kernel vs fused) and the bench-shape parity tests.
#   bash tools/gpu.sh 900 'bash tools/gpu_fuse_check.sh <tag>'
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/$1; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fuse.py -x -v --timeout 120 --timeout-method thread \
    > $out/pytest_fuse.log 2>&1 || { echo "fuse tests failed rc=$?"; grep -E "FAIL|Error|assert|Mismatch|Max" $out/pytest_fuse.log | head -30; exit 1; }
tail -1 $out/pytest_fuse.log
timeout -k 10 120 python tools/bench_fuse.py --two-kernel > $out/abl.txt 2>&1 || exit 1
timeout -k 10 120 python tools/bench_fuse.py >> $out/abl.txt 2>&1 || exit 1
grep -v amdgpu.ids $out/abl.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "bench_shape or two_lanes" \
    > $out/pytest_parity.log 2>&1 || { echo "parity failed rc=$?"; grep -E "FAIL|Error|assert" $out/pytest_parity.log | head -30; exit 1; }
tail -1 $out/pytest_parity.log
