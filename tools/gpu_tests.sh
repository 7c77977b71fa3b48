#!/bin/bash
# GPU test session without -x (every failure listed): bash tools/gpu.sh 1100 'bash tools/gpu_tests.sh <tag> [-k expr]'
set -o pipefail
tag=${1:-r04}
shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread "$@" \
    > $out/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" $out/pytest.log | grep -v PASSED | head -40
tail -3 $out/pytest.log
exit $rc
