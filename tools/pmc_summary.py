"""Average per-dispatch PMC values of the conv kernels in a tools/profile_conv.sh output dir.
Usage: python tools/pmc_summary.py gpurun_out/pmc_<tag> [kernel-substring]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else 'conv'
for f in sorted(glob.glob(d + '/p*/**/*counter_collection.csv', recursive=True)):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if sub in r['Kernel_Name']:
            agg[r['Counter_Name']].append(float(r['Counter_Value']))
    for k, v in agg.items():
        print(f'{k:32s} {sum(v) / len(v):16.0f}  (n={len(v)})')
