"""Timeline of one replayed forward from a rocprofv3 --kernel-trace CSV: per kernel its start offset, duration,
queue (lane) and the concurrency, plus per-queue busy time and the idle gaps of the critical path.
Usage: python tools/timeline.py gpurun_out/<dir>/trace/run_kernel_trace.csv [first_kernel_regex]"""
import csv
import re
import sys


def short(n):
    n = re.sub(r'\(anonymous namespace\)::', '', n)
    n = re.sub(r'\((ConvK|int|dbsr_tensor|DenseArgs).*$', '', n)
    return n[:70]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    first = re.compile(sys.argv[2] if len(sys.argv) > 2 else r'pack_raw|pack_burst|pack_rgb')
    rows = [r for r in rows if r['Kind'] == 'KERNEL_DISPATCH']
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    starts = [i for i, r in enumerate(rows) if first.search(r['Kernel_Name'])]
    # the last full forward before the per-op timing pass: the replay whose pack kernel is followed by
    # the most kernels before the next pack kernel (replays are back to back in the timed loop)
    segs = [(starts[i], starts[i + 1]) for i in range(len(starts) - 1)]
    big = max(s[1] - s[0] for s in segs)
    a, b = [s for s in segs if s[1] - s[0] >= 0.8 * big][-1]
    seg = rows[a:b]
    t0 = int(seg[0]['Start_Timestamp'])
    t1 = max(int(r['End_Timestamp']) for r in seg)
    print('forward: %d kernels, %.1f us' % (len(seg), (t1 - t0) / 1e3))
    qs = sorted({r['Queue_Id'] for r in seg})
    for r in seg:
        s, e = int(r['Start_Timestamp']) - t0, int(r['End_Timestamp']) - t0
        conc = sum(1 for o in seg if o is not r and int(o['Start_Timestamp']) - t0 < e and int(o['End_Timestamp']) - t0 > s)
        print('%8.1f %7.1f  q%s  c%d  grid %6s  %s' % (s / 1e3, (e - s) / 1e3, qs.index(r['Queue_Id']), conc,
                                                       int(r['Grid_Size_X']) // int(r['Workgroup_Size_X']),
                                                       short(r['Kernel_Name'])))
    for q in qs:
        ks = [r for r in seg if r['Queue_Id'] == q]
        busy = sum(int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in ks)
        span = (max(int(r['End_Timestamp']) for r in ks) - min(int(r['Start_Timestamp']) for r in ks))
        print('queue %d: %d kernels, busy %.1f us over a span of %.1f us' % (qs.index(q), len(ks), busy / 1e3, span / 1e3))
    # union of busy intervals (any lane) vs the forward span
    iv = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp'])) for r in seg)
    busy, cs, ce = 0, iv[0][0], iv[0][1]
    for s, e in iv[1:]:
        if s > ce:
            busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    print('GPU busy (any lane) %.1f us of %.1f us; idle %.1f us' % (busy / 1e3, (t1 - t0) / 1e3, (t1 - t0 - busy) / 1e3))


if __name__ == '__main__':
    main()
