"""Where a conv3x3_pipe_kernel launch spends its cycles, from the diagnostic stamp build.

Build:  make exp EXP_FLAGS=-DDBSR_PIPE_STAMPS EXP_NAME=stamps
Run:    DBSR_HIP_LIB=deep-rawburst-sr_amd/libdbsr_hip_stamps.so python tools/pipe_stamps.py --only enc.res
Per wave and stage: 'vm' = stage end -> its outstanding vector-memory ops drained (vmcnt(0)), 'bar' =
barrier skew, 'taps0-5' / 'taps6-8' = barrier exit -> tap 6 -> end of the 9 taps (the DMA of the next stage
is issued in taps 0-5; the epilogue of the previous tile sits in its first stage's taps0-5).  Cycles are s_memtime
ticks (shader clock)."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dbsr_amd import _lib as L                     # noqa: E402
from dbsr_amd.engine import NHWC, PackedConv, Plan, cpad  # noqa: E402
from tools.bench_conv import SHAPES                # noqa: E402

STAGES, EV = 24, 5
SLOTS = STAGES * EV + 2


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument('--only', default='enc.res')
    args = ap.parse_args()
    dev = torch.device('cuda')
    dt = torch.float16
    s = torch.cuda.current_stream().cuda_stream
    lib = L.lib()
    fn = lib.dbsr_diag_pipe_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_longlong]
    for name, F, H, W, cin, cout, k in SHAPES:
        if args.only not in name:
            continue
        conv = torch.nn.Conv2d(cin, cout, k, padding=k // 2).to(dev)
        pc = PackedConv(conv, dt, dev, s)
        x = NHWC(F, H, W, cpad(cin), dt, dev)
        x.t.normal_()
        y = NHWC(F, H, W, max(8, (cout + 7) // 8 * 8), dt, dev)
        plan = Plan()
        if 'res' in name or 'post' in name or 'pre' in name:
            r = NHWC(F, H, W, max(8, (cout + 7) // 8 * 8), dt, dev)
            r.t.normal_()
            plan.conv(name, pc, F, x, 0, (H, W), y, 0, L.ACT_NONE, res=r, post_act=L.ACT_RELU)
        else:
            plan.conv(name, pc, F, x, 0, (H, W), y, 0, L.ACT_RELU)
        plan.finalize_workspace(dev)
        for _ in range(20):
            plan.run(s)
        torch.cuda.synchronize()
        fn(None, 0)
        plan.run(s)
        torch.cuda.synchronize()
        buf = np.zeros(256 * 8 * SLOTS, dtype=np.uint64)
        fn(buf.ctypes.data, buf.size)
        st = buf.reshape(256, 8, SLOTS).astype(np.int64)
        live = st[:, :, 0] > 0
        t0 = st[:, :, 0][live].min()
        span = st[:, :, 1][live].max() - t0
        life = (st[:, :, 1] - st[:, :, 0])[live]
        print(f'{name}: kernel span {span} cyc; wave life median {np.median(life):.0f} min {life.min()} max {life.max()}')
        print(f'  start skew (first->last wave start) {st[:, :, 0][live].max() - t0}')
        nst = 0
        for si in range(STAGES):
            if not (st[:, :, 2 + EV * si] > 0).any():
                break
            nst = si + 1
        print('  stage  waves  pre-gap  vm(med/p90)   bar(med/p90)  taps0-5(med)  taps6-8(med)')
        for si in range(nst):
            a, a2, b, m, c = (st[:, :, 2 + EV * si + e] for e in range(EV))
            ok = (a > 0) & (a2 > 0) & (b > 0) & (m > 0) & (c > 0)
            if not ok.any():
                continue
            prevc = st[:, :, 0] if si == 0 else st[:, :, 2 + EV * (si - 1) + EV - 1]
            gap, vm, bar, t05, t68 = ((a - prevc)[ok], (a2 - a)[ok], (b - a2)[ok], (m - b)[ok], (c - m)[ok])
            print('  %5d %6d %8.0f %6.0f %6.0f  %6.0f %6.0f  %8.0f     %8.0f' % (
                si, ok.sum(), np.median(gap), np.median(vm), np.percentile(vm, 90), np.median(bar),
                np.percentile(bar, 90), np.median(t05), np.median(t68)))
        last = st[:, :, 1][live] - np.array([st[b_, w_, 2 + EV * (n - 1) + EV - 1] for (b_, w_), n in
                                            [((b_, w_), max(si + 1 for si in range(nst) if st[b_, w_, 2 + EV * si] > 0))
                                             for b_, w_ in zip(*np.nonzero(live))]])
        print(f'  final epilogue+stores median {np.median(last):.0f}')


if __name__ == '__main__':
    main()
