"""Where a conv3x3_ws_kernel launch spends its cycles (diagnostic stamp build, see tools/pipe_stamps.py).

Build:  make exp EXP_FLAGS=-DDBSR_PIPE_STAMPS EXP_NAME=stamps
Run:    DBSR_HIP_LIB=deep-rawburst-sr_amd/libdbsr_hip_stamps.so python tools/ws_stamps.py --only enc.res
Slots: 0 start, 2 weights loaded + first halo issued, per tile t: 3+5t before wait, 4+5t vmcnt(0) done,
5+5t barrier passed, 6+5t epilogue of the previous tile done, 7+5t steps done; 1 end."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dbsr_amd import _lib as L                     # noqa: E402
from dbsr_amd.engine import NHWC, PackedConv, Plan, cpad  # noqa: E402
from tools.bench_conv import SHAPES                # noqa: E402

SLOTS = 24 * 5 + 2
MAXT = 23


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument('--only', default='enc.res')
    args = ap.parse_args()
    dev = torch.device('cuda')
    dt = torch.float16
    s = torch.cuda.current_stream().cuda_stream
    L.lib().dbsr_set_conv_algo(2)                  # default selection: the weight-stationary kernel (the one with stamps)
    fn = L.lib().dbsr_diag_pipe_stamps
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
        life = (st[:, :, 1] - st[:, :, 0])[live]
        pro = (st[:, :, 2] - st[:, :, 0])[live]
        print(f'{name}: wave life median {np.median(life):.0f} (min {life.min()} max {life.max()}); '
              f'prologue (weights + first DMA issue) median {np.median(pro):.0f}')
        print('  tile  waves  pre-gap  vm      bar    epi    steps')
        for t in range(MAXT):
            a, a2, b, e, c = (st[:, :, 3 + 5 * t + i] for i in range(5))
            ok = (a > 0) & (c > 0)
            if not ok.any():
                break
            prevc = st[:, :, 2] if t == 0 else st[:, :, 3 + 5 * (t - 1) + 4]
            print('  %4d %6d %8.0f %6.0f %6.0f %6.0f %8.0f' % (
                t, ok.sum(), np.median((a - prevc)[ok]), np.median((a2 - a)[ok]), np.median((b - a2)[ok]),
                np.median((e - b)[ok]), np.median((c - e)[ok])))
        last_t = np.array([max(t for t in range(MAXT) if st[bb, ww, 3 + 5 * t] > 0) for bb, ww in zip(*np.nonzero(live))])
        ends = np.array([st[bb, ww, 3 + 5 * t + 4] for (bb, ww), t in zip(zip(*np.nonzero(live)), last_t)])
        print(f'  final epilogue+stores median {np.median(st[:, :, 1][live] - ends):.0f}')


if __name__ == '__main__':
    main()
