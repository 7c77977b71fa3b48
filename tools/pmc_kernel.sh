#!/bin/bash
# PMC passes (stall breakdown, MFMA busy, LDS, instruction mix) of one kernel under a microbenchmark, for the
# product library and variant builds (libdbsr_hip_<name>.so).
#   bash tools/pmc_kernel.sh <tag> <kernel regex> "<bench command>" [variant names...]
set -o pipefail
tag=$1; regex=$2; cmd=$3; shift 3
out=gpurun_out/pmc_$tag
mkdir -p $out
export TMPDIR=/tmp
for v in product "$@"; do
  lib=deep-rawburst-sr_amd/libdbsr_hip.so; [ "$v" != product ] && lib=deep-rawburst-sr_amd/libdbsr_hip_$v.so
  i=0
  for ctrs in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT" \
              "SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES SQ_INSTS_MFMA SQ_INSTS_SALU"; do
    i=$((i+1))
    DBSR_HIP_LIB=$lib timeout -k 10 120 rocprofv3 --pmc $ctrs --kernel-include-regex "$regex" -d $out/${v}_p$i -o run \
        --output-format csv -- $cmd > $out/${v}_p$i.log 2>&1 || exit $?
  done
done
echo done
