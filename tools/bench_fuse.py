"""Microbenchmark of the weight predictor's output conv + softmax + fusion at the cfg2 bench shape (B=8, N=14,
48x48, 128 -> 512, fp16): dbsr_conv_fuse_softmax against dbsr_conv2d (logits) + dbsr_fuse_softmax, each op
re-launched back to back between HIP events (library: DBSR_HIP_LIB, for same-box A/B of variant builds).
Usage: python tools/bench_fuse.py [--reps 20] [--two-kernel]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dbsr_amd import _lib as L                                 # noqa: E402
from dbsr_amd.engine import NHWC, PackedConv, Plan             # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=20)
    ap.add_argument('--two-kernel', action='store_true')
    ap.add_argument('--batch', type=int, default=8)
    args = ap.parse_args()
    B, N, H, W, cin, C = args.batch, 14, 48, 48, 128, 512
    dt, dev = torch.float16, torch.device('cuda')
    s = torch.cuda.current_stream().cuda_stream
    conv = torch.nn.Conv2d(cin, C, 3, padding=1).to(dev)
    pc = PackedConv(conv, dt, dev, s)
    X = NHWC(B * N, H, W, cin, dt, dev)
    X.t.normal_()
    E = NHWC(B * N, H, W, C, dt, dev)
    E.t.normal_()
    Wf = NHWC(B * (N - 1), H, W, C, dt, dev)
    Wf.t.normal_()
    FUS, FW = NHWC(B, H, W, C, dt, dev), NHWC(B * N, H, W, C, dt, dev)
    feats = [E.d(0, (1, N, 0, 1)), Wf.d(0), FUS.d(0), FW.d(0)]
    plan = Plan()
    flop = 2.0 * B * N * H * W * C * cin * 9
    if args.two_kernel:
        LG = NHWC(B * N, H, W, C, dt, dev)
        plan.conv('wp.out', pc, B * N, X, 0, (H, W), LG, 0, L.ACT_NONE)
        plan.add('fuse', L.lib().dbsr_fuse_softmax, B, N, H * W, C, LG.d(0), *feats)
    else:
        assert plan.conv_fuse('wp.out+fuse', pc, B, N, X, (H, W), *feats) is not None
    plan.finalize_workspace(dev)
    for _ in range(3):
        plan.run(s)
    torch.cuda.synchronize()
    tt = plan.time_ops(s, reps=args.reps)
    tot = sum(t for _, t in tt)
    print('%s: %s  total %.1f us  %.1f TF/s (%s)' % (os.path.basename(L.LIB_PATH),
          '  '.join('%s %.1f us' % (n, t * 1e3) for n, t in tt), tot * 1e3, flop / (tot * 1e-3) / 1e12,
          'two-kernel' if args.two_kernel else 'fused'))


if __name__ == '__main__':
    main()
