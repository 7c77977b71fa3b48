#!/bin/bash
# PMC traffic of the generic conv launches (FETCH_SIZE and WRITE_SIZE in separate passes)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/pmc_generic
mkdir -p $out
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 240 rocprofv3 --pmc $c --kernel-include-regex "conv2d_kernel" -d $out/$c -o run --output-format csv -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-graph > $out/$c.log 2>&1 || { echo "[pmc] $c rc=$?"; exit 1; }
done
echo done
