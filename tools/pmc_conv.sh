#!/bin/bash
# PMC passes over the isolated conv microbenchmark (tools/bench_conv.py) for one shape filter:
# stall breakdown (SQ), clock (GRBM) and L2 hit/miss (TCC), each pass its own rocprofv3 run.
# Usage: bash tools/pmc_conv.sh <tag> <shape-substring> [algo]
set -o pipefail
tag=$1; only=$2; algo=${3:-2}
out=gpurun_out/pmc_$tag
mkdir -p $out
export TMPDIR=/tmp
i=0
for ctrs in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT" \
            "SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $ctrs --kernel-include-regex "conv3x3" -d $out/p$i -o run --output-format csv -- \
      python3 tools/bench_conv.py --only "$only" --algos $algo --reps 5 > $out/p$i.log 2>&1 || exit $?
done
echo done
