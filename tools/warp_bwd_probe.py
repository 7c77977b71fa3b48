"""Diagnostic (GPU box): the flow field the training bench's warp backward sees, its hit distribution over the
16x16 destination tiles, and the time of dbsr_warp_backward_gather on it (run under rocprofv3 --stats for the
per-kernel split).  python tools/warp_bwd_probe.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dbsr_amd  # noqa: E402
from dbsr_amd import ops  # noqa: E402
from dbsr_amd.burst import synthetic_bursts  # noqa: E402
from dbsr_amd.training import DBSRTrainer  # noqa: E402

dev = torch.device('cuda', 0)
B, N, S = 8, 14, 128
net = dbsr_amd.build_synthetic_net(seed=0).to(dev).set_compute_dtype(torch.bfloat16)
tr = DBSRTrainer(net)
burst, gt = synthetic_bursts(B, N, S, S, sr_factor=8, seed=2000)
loss, pred = tr.forward_backward(burst.to(dev), gt.to(dev))
torch.cuda.synchronize()
off = tr.plans[(B, N, S, S)].bufs['offsets']            # [P, 2, H, W]
P, _, H, W = off.shape
fx, fy = off[:, 0], off[:, 1]
print('flow |fx| max %.2f mean %.2f  |fy| max %.2f mean %.2f  finite %s' % (
    fx.abs().max(), fx.abs().mean(), fy.abs().max(), fy.abs().mean(), bool(torch.isfinite(off).all())))
ys, xs = torch.meshgrid(torch.arange(H, device=dev), torch.arange(W, device=dev), indexing='ij')
x0 = torch.floor(xs + fx).long()
y0 = torch.floor(ys + fy).long()
inb = (x0 >= 0) & (x0 < W) & (y0 >= 0) & (y0 < H)
tile = (y0.clamp(0, H - 1) // 16) * (W // 16) + x0.clamp(0, W - 1) // 16
cnt = torch.zeros(P, (H // 16) * (W // 16), device=dev)
cnt.scatter_add_(1, torch.where(inb, tile, 0).view(P, -1), inb.view(P, -1).float())
print('in-frame tap bases per pair: %.0f of %d; per-tile hits max %.0f mean %.1f, tiles with 0 hits %.3f' % (
    inb.view(P, -1).sum(1).float().mean(), H * W, cnt.max(), cnt.mean(), (cnt == 0).float().mean()))
dout = torch.randn(P, 512, H, W, device=dev, dtype=torch.bfloat16)
for _ in range(2):
    ops.warp_backward_gather(dout, off)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(5):
    ops.warp_backward_gather(dout, off)
torch.cuda.synchronize()
print('warp_backward_gather (incl. layout copies) %.2f ms' % ((time.perf_counter() - t0) / 5 * 1e3))
