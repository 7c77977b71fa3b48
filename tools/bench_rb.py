"""Microbenchmark of one fused ResBlock launch (dbsr_resblock) against the two dbsr_conv2d launches it replaces,
re-launched back to back between HIP events (library: DBSR_HIP_LIB, for same-box A/B of variant builds).
Defaults: a decoder post-ResBlock at the configs[1] shape (8 frames of 384x384, 32 channels, fp16); --channels 64
--frames 112 --size 48: an encoder ResBlock (--cap 128: under the encoder's CU cap while PWC-Net runs beside it).
Usage: python tools/bench_rb.py [--two-kernel] [--channels C] [--frames N] [--size S] [--cap CUS]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dbsr_amd import _lib as L                                 # noqa: E402
from dbsr_amd.engine import NHWC, PackedConv, Plan             # noqa: E402


def run(args, two_kernel):
    B, H, W, C = args.frames, args.size, args.size, args.channels
    dt, dev = torch.float16, torch.device('cuda')
    s = torch.cuda.current_stream().cuda_stream
    pcs = [PackedConv(torch.nn.Conv2d(C, C, 3, padding=1).to(dev), dt, dev, s) for _ in range(2)]
    X, M, Y = (NHWC(B, H, W, C, dt, dev) for _ in range(3))
    X.t.normal_()
    plan = Plan()
    plan.max_blocks = args.cap
    if two_kernel:
        plan.conv('c1', pcs[0], B, X, 0, (H, W), M, 0, L.ACT_RELU)
        plan.conv('c2', pcs[1], B, M, 0, (H, W), Y, 0, L.ACT_NONE, res=X, post_act=L.ACT_RELU)
    else:
        assert plan.resblock('rb', pcs[0], pcs[1], B, X, M, Y, (H, W))
    plan.finalize_workspace(dev)
    for _ in range(5):
        plan.run(s)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(20_000_000)           # the host stays ahead of the launches
    e0.record()
    for _ in range(args.reps):
        plan.run(s)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / args.reps
    gf = 2 * 2.0 * B * H * W * C * 9 * C / 1e9
    print('C %d %dx%dx%d cap %d  %-10s %7.1f us per ResBlock (%.0f TF/s algorithmic, %.2f TB/s for x + y)' % (
        C, B, H, W, args.cap, 'two convs' if two_kernel else 'resblock', us, gf / us * 1e-3 * 1e6 / 1e6,
        2 * B * H * W * 2 * C / us / 1e6), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=50)
    ap.add_argument('--two-kernel', action='store_true', help='also time the two-launch path')
    ap.add_argument('--frames', type=int, default=8)
    ap.add_argument('--size', type=int, default=384)
    ap.add_argument('--channels', type=int, default=32)
    ap.add_argument('--cap', type=int, default=0)
    args = ap.parse_args()
    run(args, False)
    if args.two_kernel:
        run(args, True)


if __name__ == '__main__':
    main()
