#!/bin/bash
# PMC passes over one conv shape of tools/bench_conv.py (tiled kernel), one counter group per pass.
# Usage: bash tools/profile_conv.sh <shape-substring> <tag>
set -o pipefail
shape=$1; tag=${2:-conv}
out=gpurun_out/pmc_$tag
mkdir -p $out
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS" \
           "SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $grp --kernel-include-regex "conv" -d $out/p$i -o run --output-format csv -- \
      python3 tools/bench_conv.py --only "$shape" --algos 1 --reps 3 > $out/p$i.log 2>&1 || exit $?
done
echo done
