#!/bin/bash
# HBM traffic (PMC) of the round-5 fused kernels under the bench: FETCH_SIZE and WRITE_SIZE in separate passes
# (TCC counter budget), kernel-filtered.   bash tools/gpu.sh 600 'bash tools/gpu_r05_pmc.sh <tag>'
set -o pipefail
tag=${1:-r05z}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "resblock32|upsample_blur|conv_fuse" -d $out/$c -o run \
        --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $out/$c.log 2>&1 || { echo "pmc $c failed"; tail -5 $out/$c.log; exit 1; }
done
echo done
