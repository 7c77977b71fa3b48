#!/bin/bash
# Quick A/B session: selected GPU tests, then the bench under each dbsr_set_conv_algo value given.
#   bash tools/gpu.sh 900 'bash tools/gpu_ab.sh <tag> "<pytest -k expr>" <algo> [<algo> ...]'
set -o pipefail
tag=$1; kexpr=$2; shift 2
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
if [ -n "$kexpr" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$kexpr" \
      > $out/pytest.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "FAILED|Error" $out/pytest.log | head; tail -30 $out/pytest.log; exit 1; }
  tail -1 $out/pytest.log
fi
for a in "$@"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --kernel-breakdown --conv-algo $a > $out/bench_a$a.json 2> $out/bench_a$a.err || { echo "bench algo $a failed"; tail -20 $out/bench_a$a.err; exit 1; }
  python -c "import json;d=json.load(open('$out/bench_a$a.json'));print('algo $a', d['value'], d['ms_per_step'], d['roofline']['kernel'][:22], d['roofline']['frac'], 'chip', d['roofline_whole_chip']['kernel'][:22], d['roofline_whole_chip']['frac'])"
  grep "\[family\] conv3x3_ws" $out/bench_a$a.err
done
echo done
