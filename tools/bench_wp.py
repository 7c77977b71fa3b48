"""Microbenchmark of dbsr_warp_project (warp + projection of the warped frames) against the two launches it replaces
(dbsr_warp_bilinear + the 1x1 projection conv) and the warp alone, at the configs[1] shape (8 bursts x 13 warped
frames of 48x48, 512 channels -> 64, fp16), each re-launched back to back between HIP events.  Library: DBSR_HIP_LIB
(same-box A/B of variant builds, tools/build_variant.sh).
Usage: python tools/bench_wp.py [--reps 50]"""
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
    ap.add_argument('--bursts', type=int, default=8)
    args = ap.parse_args()
    B, N, H, W, C, pd = args.bursts, 14, 48, 48, 512, 64
    P = B * (N - 1)
    dt, dev = torch.float16, torch.device('cuda')
    s = torch.cuda.current_stream().cuda_stream
    E = NHWC(B * N, H, W, C, dt, dev)
    E.t.normal_()
    flow = (torch.randn(P, 2, H, W, device=dev) * 2.0).contiguous()
    pc = PackedConv(torch.nn.Conv2d(C, pd, 1).to(dev), dt, dev, s)
    Wf = NHWC(P, H, W, C, dt, dev)
    WP = NHWC(B * N, H, W, 128, dt, dev)
    emap, ymap = (N - 1, N, 1, 1), (N - 1, N, 1, 1)
    lib = L.lib()
    plans = {}
    for name in ('warp', 'warp+conv', 'warp_project'):
        plan = Plan()
        if name == 'warp_project':
            plan.add(name, lib.dbsr_warp_project, P, H, W, C, E.d(0, emap), flow.data_ptr(), 2 * H * W, Wf.d(0),
                     pc.w.data_ptr(), pc.bias.data_ptr(), pd, WP.d(0, ymap))
        else:
            plan.add('warp', lib.dbsr_warp_bilinear, P, H, W, C, E.d(0, emap), flow.data_ptr(), 2 * H * W, Wf.d(0))
            if name == 'warp+conv':
                plan.conv('proj', pc, P, Wf, 0, (H, W), WP, 0, L.ACT_RELU, ymap=ymap)
        plan.finalize_workspace(dev)
        plans[name] = plan
    for name, plan in plans.items():
        for _ in range(5):
            plan.run(s)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(20_000_000)
        e0.record()
        for _ in range(args.reps):
            plan.run(s)
        e1.record()
        e1.synchronize()
        us = e0.elapsed_time(e1) / args.reps * 1e3
        by = 2.0 * P * H * W * C * 2 + 8.0 * P * H * W
        print('%-14s %8.1f us   (warp bytes %.1f MB -> %.0f GB/s)' % (name, us, by / 1e6, by / (us * 1e-6) / 1e9),
              flush=True)


if __name__ == '__main__':
    main()
