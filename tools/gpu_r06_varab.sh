#!/bin/bash
# Same-box A/B of experiment libraries (tools/build_variant.sh) on the training step: one process per run,
# alternating product / variants.   bash tools/gpu.sh 900 'bash tools/gpu_r06_varab.sh <tag> <variant> ...'
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
for round in 1 2; do
  for v in product "$@"; do
    lib=deep-rawburst-sr_amd/libdbsr_hip.so
    [ "$v" != product ] && lib=deep-rawburst-sr_amd/libdbsr_hip_$v.so
    DBSR_HIP_LIB=$lib timeout -k 10 200 python tools/train_ab.py default default > $out/ab_${v}_$round.log 2>&1 || { echo "$v failed"; tail $out/ab_${v}_$round.log; exit 1; }
    echo "$v: $(grep ms/step $out/ab_${v}_$round.log | awk '{print $2}' | tr '\n' ' ')"
  done
done
echo done
