"""From a rocprofv3 kernel-trace CSV of bench.py, print per-queue busy time and cross-queue overlap for one
graph-replayed forward (between two consecutive pack_raw_kernel dispatches).
Usage: python tools/lane_timeline.py <run_kernel_trace.csv> [which-forward]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
marks = [i for i, r in enumerate(rows) if 'pack_raw_kernel' in r['Kernel_Name']]
k = int(sys.argv[2]) if len(sys.argv) > 2 else 5
fw = rows[marks[k]:marks[k + 1]]
t0 = int(fw[0]['Start_Timestamp'])
t1 = max(int(r['End_Timestamp']) for r in fw)
print('forward span %.1f us, %d kernels' % ((t1 - t0) / 1e3, len(fw)))
byq = {}
for r in fw:
    byq.setdefault(r['Queue_Id'], []).append((int(r['Start_Timestamp']) - t0, int(r['End_Timestamp']) - t0,
                                             r['Kernel_Name'].split('(')[0].replace('void (anonymous namespace)::', '')))
for q, iv in sorted(byq.items()):
    busy = sum(e - s for s, e, _ in iv)
    print('queue %s: %d kernels, first %.1f last-end %.1f us, busy %.1f us' % (q, len(iv), iv[0][0] / 1e3,
          max(e for _, e, _ in iv) / 1e3, busy / 1e3))
qs = sorted(byq)
if len(qs) >= 2:
    a, b = byq[qs[0]], byq[qs[1]]
    ov = 0
    for s1, e1, _ in a:
        for s2, e2, _ in b:
            ov += max(0, min(e1, e2) - max(s1, s2))
    print('cross-queue overlap %.1f us' % (ov / 1e3))
for s, e, n in sorted(sum(byq.values(), []))[:200]:
    print('%8.1f %8.1f %6.1f %s' % (s / 1e3, e / 1e3, (e - s) / 1e3, n[:50]))
