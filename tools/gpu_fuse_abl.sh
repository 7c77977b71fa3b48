#!/bin/bash
# Same-box A/B of conv_fuse ablation builds (tools/build_variant.sh fa<bits> -DDBSR_FUSE_ABL=<bits> conv_fuse)
#   bash tools/gpu.sh 600 'bash tools/gpu_fuse_abl.sh <tag> <bits...>'
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/$1; shift; mkdir -p $out
timeout -k 10 120 python tools/bench_fuse.py --two-kernel > $out/abl.txt 2>&1 || exit 1
timeout -k 10 120 python tools/bench_fuse.py >> $out/abl.txt 2>&1 || exit 1
for v in "$@"; do DBSR_HIP_LIB=deep-rawburst-sr_amd/libdbsr_hip_fa$v.so timeout -k 10 120 python tools/bench_fuse.py >> $out/abl.txt 2>&1 || exit 1; done
timeout -k 10 120 python tools/bench_fuse.py >> $out/abl.txt 2>&1 || exit 1
grep -v amdgpu.ids $out/abl.txt
