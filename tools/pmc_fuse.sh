#!/bin/bash
# PMC passes (stall breakdown, MFMA busy, LDS) over the fused weight-predictor microbenchmark, for the product
# library and ablation builds (libdbsr_hip_fa<bits>.so).  Usage: bash tools/pmc_fuse.sh <tag> <bits...>
set -o pipefail
tag=$1; shift
out=gpurun_out/pmcf_$tag
mkdir -p $out
export TMPDIR=/tmp
for v in 0 "$@"; do
  lib=deep-rawburst-sr_amd/libdbsr_hip.so; [ "$v" != 0 ] && lib=deep-rawburst-sr_amd/libdbsr_hip_fa$v.so
  DBSR_HIP_LIB=$lib timeout -k 10 120 python3 tools/bench_fuse.py --reps 10 >> $out/bench.txt 2>&1 || exit $?
  i=0
  for ctrs in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT" \
              "SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES SQ_INSTS_MFMA SQ_INSTS_SALU"; do
    i=$((i+1))
    DBSR_HIP_LIB=$lib timeout -k 10 120 rocprofv3 --pmc $ctrs --kernel-include-regex "conv_fuse" -d $out/v${v}_p$i -o run \
        --output-format csv -- python3 tools/bench_fuse.py --reps 3 > $out/v${v}_p$i.log 2>&1 || exit $?
  done
done
grep -v amdgpu.ids $out/bench.txt
echo done
