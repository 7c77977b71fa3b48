#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/trace_$1; mkdir -p $out
timeout -k 10 200 rocprofv3 --kernel-trace -d $out -o run --output-format csv -- python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline > $out/bench.log 2>&1 || exit $?
echo done
