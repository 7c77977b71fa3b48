"""Microbenchmark of one decoder post-ResBlock at the configs[1] shape (8 frames of 384x384, 32 channels, fp16):
dbsr_resblock against the two dbsr_conv2d launches, re-launched back to back between HIP events
(library: DBSR_HIP_LIB, for same-box A/B of variant builds).  Usage: python tools/bench_rb.py [--two-kernel]"""
import argparse
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
    ap.add_argument('--frames', type=int, default=8)
    args = ap.parse_args()
    B, H, W = args.frames, 384, 384
    dt, dev = torch.float16, torch.device('cuda')
    s = torch.cuda.current_stream().cuda_stream
    pcs = [PackedConv(torch.nn.Conv2d(32, 32, 3, padding=1).to(dev), dt, dev, s) for _ in range(2)]
    X, M, Y = (NHWC(B, H, W, 32, dt, dev) for _ in range(3))
    X.t.normal_()
    plan = Plan()
    if args.two_kernel:
        plan.conv('c1', pcs[0], B, X, 0, (H, W), M, 0, L.ACT_RELU)
        plan.conv('c2', pcs[1], B, M, 0, (H, W), Y, 0, L.ACT_NONE, res=X, post_act=L.ACT_RELU)
    else:
        assert plan.resblock('rb', pcs[0], pcs[1], B, X, M, Y, (H, W))
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
    gf = 2 * 2.0 * B * H * W * 32 * 288 / 1e9
    print('%s: %.1f us per ResBlock (%.0f TF/s algorithmic, %.2f TB/s for x + y)' % (
        'two convs' if args.two_kernel else 'resblock', us, gf / us * 1e-3 * 1e6 / 1e6,
        2 * B * H * W * 64 / us / 1e6))


if __name__ == '__main__':
    main()
