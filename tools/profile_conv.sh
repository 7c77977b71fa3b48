#!/bin/bash
# PMC passes over one conv shape of tools/bench_conv.py, one counter group per pass.
# Usage: bash tools/profile_conv.sh <shape-substring> <tag> [algo (default 2)]
set -o pipefail
shape=$1; tag=${2:-conv}; algo=${3:-2}
out=gpurun_out/pmc_$tag
mkdir -p $out
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS" \
           "SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES" \
           "TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TCC_HIT_sum TCC_MISS_sum" \
           "TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TD_TD_BUSY_sum"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "conv" -d $out/p$i -o run --output-format csv -- \
      python3 tools/bench_conv.py --only "$shape" --algos $algo --reps 3 > $out/p$i.log 2>&1 || echo "pass $i failed: $grp"
done
echo done
