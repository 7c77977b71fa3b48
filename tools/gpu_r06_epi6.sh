#!/bin/bash
# EPI-6 (compile-time LeakyReLU epilogue) check: the PWC / e2e / two-lane tests on the variant library, then the
# forward and training benches alternating product / variant (per-op breakdown).
set -o pipefail
out=gpurun_out/epi6
mkdir -p $out
V=deep-rawburst-sr_amd/libdbsr_hip_epi6.so
DBSR_HIP_LIB=$V timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_e2e.py -x -q --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 \
    || { echo "tests failed rc=$?"; grep -E "FAIL|Error|assert" $out/pytest.log | head; tail -3 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for r in 1 2; do
  for v in product epi6; do
    lib=deep-rawburst-sr_amd/libdbsr_hip.so; [ $v = epi6 ] && lib=$V
    DBSR_HIP_LIB=$lib timeout -k 10 200 python bench.py --kernel-breakdown --no-cpu-baseline > $out/f_${v}_$r.json 2> $out/f_${v}_$r.err || { echo "$v fwd failed"; exit 1; }
    DBSR_HIP_LIB=$lib timeout -k 10 200 python bench.py --mode train --kernel-breakdown --no-cpu-baseline --steps 10 > $out/t_${v}_$r.json 2> $out/t_${v}_$r.err || { echo "$v train failed"; exit 1; }
    echo "$v fwd $(python -c "import json;print(json.load(open('$out/f_${v}_$r.json'))['value'])") train $(python -c "import json;print(json.load(open('$out/t_${v}_$r.json'))['ms_per_step'])") $(grep -E '^pwc.refiner0 ' $out/f_${v}_$r.err | awk '{print $3, $6}')"
  done
done
echo done
