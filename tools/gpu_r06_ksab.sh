#!/bin/bash
# K-split 128-channel kernel: timing-only ablations and variants (tools/build_variant.sh libraries) on the bench
# shape, then the product bench with the per-op breakdown.   bash tools/gpu.sh 900 'bash tools/gpu_r06_ksab.sh <tag>'
set -o pipefail
tag=${1:-r06ka}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ks128.py -x -q --timeout 120 --timeout-method thread > $out/pytest_ks.log 2>&1 \
    || { echo "ks tests failed"; grep -E "FAIL|Error|assert" $out/pytest_ks.log | head -10; tail -3 $out/pytest_ks.log; exit 1; }
tail -1 $out/pytest_ks.log
for v in "" ks_r4; do
  lib=deep-rawburst-sr_amd/libdbsr_hip${v:+_$v}.so
  [ -f $lib ] || continue
  echo "== ${v:-product}" >> $out/ab.txt
  DBSR_HIP_LIB=$PWD/$lib timeout -k 10 120 python -u tools/bench_conv.py --only "(104 frames)" --reps 40 --algos 2,5 >> $out/ab.txt 2>&1 || { echo "ab $v failed"; tail -5 $out/ab.txt; exit 1; }
done
cat $out/ab.txt
timeout -k 10 300 python bench.py --kernel-breakdown --no-cpu-baseline > $out/bench.json 2> $out/bench.err || { echo bench failed; tail -20 $out/bench.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench.json'));print('fp16', d['value'], d['ms_per_step'])"
grep -E "merge.wp|^\[family\]" $out/bench.err | head -30
