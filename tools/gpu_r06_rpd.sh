set -o pipefail
mkdir -p gpurun_out/rpd
for v in product rpd4 rpd8 product rpd4 rpd8; do
  lib=deep-rawburst-sr_amd/libdbsr_hip.so; [ "$v" != product ] && lib=deep-rawburst-sr_amd/libdbsr_hip_$v.so
  DBSR_HIP_LIB=$lib timeout -k 10 200 python bench.py --mode train --kernel-breakdown --no-cpu-baseline --steps 10 > gpurun_out/rpd/$v.json 2> gpurun_out/rpd/$v.err || { echo "$v failed"; tail gpurun_out/rpd/$v.err; exit 1; }
  echo "$v $(python -c "import json;print(json.load(open('gpurun_out/rpd/$v.json'))['ms_per_step'])") $(grep -E '^bwd.proj.oth ' gpurun_out/rpd/$v.err)"
done
