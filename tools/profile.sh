#!/bin/bash
# Profiling recipe run on the GPU box (see DESIGN.md "Measurement"):
#   1. kernel trace + stats of the default bench workload (graph replays only: in-step kernel durations)
#   2. separate PMC passes (FETCH_SIZE, WRITE_SIZE) restricted to the HBM-bound kernels
#   3. kernel trace + stats of the training leg (bench.py --mode train)
# Usage: bash tools/profile.sh <tag>      (outputs under gpurun_out/prof_<tag>/)
set -o pipefail
tag=${1:-r01}
out=gpurun_out/prof_$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-op-timing > $out/bench_trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "warp512|warp_kernel|fuse_softmax|fuse512|conv3x3|conv1x1|upsample_shuffle|upsample_blur|resblock32|conv_fuse|conv2d_kernel|pwc_dense|pwc_extract" \
    -d $out/pmc_fetch -o run --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-op-timing > $out/bench_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "warp512|warp_kernel|fuse_softmax|fuse512|conv3x3|conv1x1|upsample_shuffle|upsample_blur|resblock32|conv_fuse|conv2d_kernel|pwc_dense|pwc_extract" \
    -d $out/pmc_write -o run --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-op-timing > $out/bench_write.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/train -o run --output-format csv -- \
    python3 bench.py --mode train --steps 4 --warmup 2 --no-op-timing > $out/bench_train_trace.log 2>&1 || exit $?
echo done
