"""Summarise tools/pmc_kernel.sh output: per variant, the counters summed over the kernel's dispatches / dispatch
count (rocprofv3 csv: one row per dispatch and counter).  Usage: python tools/pmc_summary.py gpurun_out/pmc_<tag>"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(d):
    per = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for f in sorted(glob.glob(os.path.join(d, '*_p*', 'run_counter_collection.csv'))):
        v = os.path.basename(os.path.dirname(f)).rsplit('_p', 1)[0]
        for row in csv.DictReader(open(f)):
            per[v][row['Counter_Name']] += float(row['Counter_Value'])
            disp[(v, os.path.dirname(f))].add(row['Dispatch_Id'])
    for v, c in per.items():
        n = max(len(s) for (vv, _), s in disp.items() if vv == v)
        c = {k: x / n for k, x in c.items()}
        wc = c.get('SQ_WAVE_CYCLES', 1) or 1
        g = c.get('GRBM_GUI_ACTIVE', 0)
        print('%-10s dispatches %d  gui_active/XCD %.3g cyc' % (v, n, g / 8))
        print('   wait_any %.2f wait_inst %.2f active %.2f wait_lds %.2f | mfma_busy %.3g  lds_conflict %.3g lds_active %.3g' % (
            c.get('SQ_WAIT_ANY', 0) / wc, c.get('SQ_WAIT_INST_ANY', 0) / wc, c.get('SQ_ACTIVE_INST_ANY', 0) / wc,
            c.get('SQ_WAIT_INST_LDS', 0) / wc, c.get('SQ_VALU_MFMA_BUSY_CYCLES', 0), c.get('SQ_LDS_BANK_CONFLICT', 0),
            c.get('SQ_LDS_IDX_ACTIVE', 0)))
        print('   waves %.0f  insts valu %.3g lds %.3g vmem %.3g mfma %.3g salu %.3g  wave_cycles %.3g' % (
            c.get('SQ_WAVES', 0), c.get('SQ_INSTS_VALU', 0), c.get('SQ_INSTS_LDS', 0), c.get('SQ_INSTS_VMEM', 0),
            c.get('SQ_INSTS_MFMA', 0), c.get('SQ_INSTS_SALU', 0), wc))


if __name__ == '__main__':
    main(sys.argv[1])
