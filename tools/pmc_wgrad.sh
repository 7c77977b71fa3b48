#!/bin/bash
# PMC passes over the wgrad microbenchmark (tools/bench_wgrad.py), ring kernel only, one shape filter.
# Usage: bash tools/pmc_wgrad.sh <tag> <shape-substring>
set -o pipefail
tag=$1; only=$2
out=gpurun_out/pmcw_$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/bench_wgrad.py > $out/bench.log 2>&1 || exit $?
cat $out/bench.log
i=0
for ctrs in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT" \
            "SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $ctrs --kernel-include-regex "conv_wgrad_dma" -d $out/p$i -o run --output-format csv -- \
      python3 tools/bench_wgrad.py --only "$only" --algos 1 --reps 3 > $out/p$i.log 2>&1 || exit $?
done
echo done
