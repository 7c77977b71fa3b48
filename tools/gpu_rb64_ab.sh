#!/bin/bash
# Same-box A/B of the fused 64-channel ResBlock variants (tools/build_variant.sh libraries) against the two
# weight-stationary launches: an encoder ResBlock (112 frames of 48x48) uncapped and under the 128-CU cap, and a
# decoder pre-ResBlock (8 frames).   bash tools/gpu.sh 600 'bash tools/gpu_rb64_ab.sh <tag> lib1 lib2 ...'
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
for lib in "$@"; do
    for cfg in "--frames 112 --size 48" "--frames 112 --size 48 --cap 128" "--frames 8 --size 48"; do
        DBSR_HIP_LIB=deep-rawburst-sr_amd/$lib timeout -k 10 120 python tools/bench_rb.py --channels 64 $cfg $([ "$lib" = libdbsr_hip.so ] && echo --two-kernel) \
            >> $out/ab.log 2>&1 || { echo "$lib $cfg failed"; tail -5 $out/ab.log; exit 1; }
        echo "[$lib] $(tail -1 $out/ab.log)"
    done
done
grep -h "two convs" $out/ab.log
