#!/bin/bash
# A/B of the product library vs the experiment build (make exp EXP_FLAGS=...) on the bench workload:
# kernel trace (durations) + FETCH_SIZE pass per library, restricted to kernels matching $1.
# Usage: bash tools/profile_ab.sh <kernel-regex> <tag>
set -o pipefail
re=$1; tag=${2:-ab}
out=gpurun_out/ab_$tag
mkdir -p $out
export TMPDIR=/tmp
for v in prod exp; do
  lib=deep-rawburst-sr_amd/libdbsr_hip.so
  [ $v = exp ] && lib=deep-rawburst-sr_amd/libdbsr_hip_exp.so
  DBSR_HIP_LIB=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --kernel-include-regex "$re" \
      -d $out/$v/trace -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline \
      > $out/$v.trace.log 2>&1 || exit $?
  DBSR_HIP_LIB=$PWD/$lib timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$re" \
      -d $out/$v/fetch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline \
      > $out/$v.fetch.log 2>&1 || exit $?
done
echo done
