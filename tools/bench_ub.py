"""Microbenchmark of the decoder's PixelShuffle upsampler + blur at the configs[1] shape (B=8, 48x48 low-res,
64 -> 2048 channels, x8, fp16): dbsr_conv_shuffle_blur against dbsr_conv2d (OUT_SHUFFLE) + dbsr_gauss_blur3, each
re-launched back to back between HIP events (library: DBSR_HIP_LIB, for same-box A/B of variant builds).
Usage: python tools/bench_ub.py [--reps 50] [--two-kernel]"""
import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dbsr_amd import _lib as L                                 # noqa: E402
from dbsr_amd.engine import NHWC, PackedConv, Plan             # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=50)
    ap.add_argument('--two-kernel', action='store_true')
    ap.add_argument('--batch', type=int, default=8)
    ap.add_argument('--stamps', action='store_true', help='read the DBSR_PIPE_STAMPS build\'s per-wave stamps')
    args = ap.parse_args()
    B, H, W, cin, S, pc = args.batch, 48, 48, 64, 8, 32
    dt, dev = torch.float16, torch.device('cuda')
    s = torch.cuda.current_stream().cuda_stream
    conv = torch.nn.Conv2d(cin, pc * S * S, 1).to(dev)
    packed = PackedConv(conv, dt, dev, s, shuffle=S)
    X = NHWC(B, H, W, cin, dt, dev)
    X.t.normal_()
    Y = NHWC(B, H * S, W * S, pc, dt, dev)
    k9 = [1 / 16, 2 / 16, 1 / 16, 2 / 16, 4 / 16, 2 / 16, 1 / 16, 2 / 16, 1 / 16]
    plan = Plan()
    if args.two_kernel:
        T = NHWC(B, H * S, W * S, pc, dt, dev)
        plan.conv('up', packed, B, X, 0, (H, W), T, 0, L.ACT_RELU, out_mode=L.OUT_SHUFFLE, shuffle=S)
        kbuf = (ctypes.c_float * 9)(*k9)
        plan.keep.append(kbuf)
        plan.add('blur', L.lib().dbsr_gauss_blur3, B, H * S, W * S, pc, T.d(0), kbuf, Y.d(0))
    else:
        assert plan.conv_shuffle_blur('ub', packed, B, X, (H, W), Y, L.ACT_RELU, k9) is not None
    plan.finalize_workspace(dev)
    for _ in range(5):
        plan.run(s)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.reps):
        plan.run(s)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / args.reps
    if args.stamps:
        import numpy as np
        fn = L.lib().dbsr_diag_pipe_stamps
        fn.argtypes = [ctypes.c_void_p, ctypes.c_longlong]
        slots = 24 * 5 + 2
        fn(None, 0)
        plan.run(s)
        torch.cuda.synchronize()
        buf = np.zeros(256 * 8 * slots, dtype=np.uint64)
        fn(buf.ctypes.data, buf.size)
        st = buf.reshape(256, 8, slots).astype(np.int64)
        t0 = st[:, :, 0].min()
        # per tile: conv (2->3), barrier incl. next loads (3->4), blur (4->5), tile start gap (prev 5 -> 2)
        print('prologue (0->1) median %d' % np.median(st[:, :, 1] - st[:, :, 0]))
        for it in range(5):
            a, b, c, d = (st[:, :, 2 + 4 * it + i] for i in range(4))
            ok = (a > 0) & (d > 0)
            if not ok.any():
                break
            print('tile %d: start %6d  conv %6d  bar %6d  blur %6d  (medians over waves; max end %d)' % (
                it, np.median(a[ok] - t0), np.median((b - a)[ok]), np.median((c - b)[ok]), np.median((d - c)[ok]),
                (d[ok] - t0).max()))
    mb = B * H * S * W * S * pc * 2 / 1e6
    print('%s: %.1f us per call (%.0f MB written: %.2f TB/s)' % (
        'conv+blur' if args.two_kernel else 'shuffle_blur', us, mb, mb / us / 1e6 * 1e6 / 1e6))


if __name__ == '__main__':
    main()
