"""Seeded synthetic bursts (the reference's cv2-based generator, data/synthetic_burst_generation.py,
cannot run here: no cv2, no datasets).

A smooth random RGB scene (sum of low-frequency sinusoids + mild texture) at the SR resolution is
translated per frame by a random sub-pixel shift (frame 0 unshifted), box-downsampled by
2*downsample, mosaicked to packed RGGB (camera_pipeline.py:139-162 layout: R, G, G, B planes) and
given shot/read noise (camera_pipeline.py:165-182 form), clamped to [0,1].  Deterministic in
(seed, shape) on CPU via torch.Generator; returns (burst[B,N,4,H,W], gt[B,3,sH,sW]).
"""
import math

import torch
import torch.nn.functional as F


def synthetic_bursts(B, N, H, W, sr_factor=8, seed=0, max_shift=2.0, noise=True):
    g = torch.Generator().manual_seed(int(seed))
    S = sr_factor
    Hr, Wr = H * S, W * S
    yy = torch.linspace(0, 1, Hr).view(1, 1, Hr, 1)
    xx = torch.linspace(0, 1, Wr).view(1, 1, 1, Wr)
    img = torch.zeros(B, 3, Hr, Wr)
    for _ in range(6):
        fx = torch.rand(B, 3, 1, 1, generator=g) * 6 + 0.5
        fy = torch.rand(B, 3, 1, 1, generator=g) * 6 + 0.5
        ph = torch.rand(B, 3, 1, 1, generator=g) * 2 * math.pi
        amp = torch.rand(B, 3, 1, 1, generator=g) * 0.15
        img = img + amp * torch.sin(2 * math.pi * (fx * xx + fy * yy) + ph)
    img = img + 0.02 * torch.rand(B, 3, Hr, Wr, generator=g)
    img = (img - img.amin(dim=(2, 3), keepdim=True))
    img = img / img.amax(dim=(2, 3), keepdim=True).clamp_min(1e-6) * 0.9 + 0.05
    gt = img.clone()

    # per-frame translation in LR-RAW pixels (frame 0 = reference, unshifted)
    shifts = (torch.rand(B, N, 2, generator=g) * 2 - 1) * max_shift
    shifts[:, 0] = 0
    ds = S // 2                           # SR image -> full-resolution RAW (RGB at 2H x 2W)
    frames = []
    for n in range(N):
        theta = torch.zeros(B, 2, 3)
        theta[:, 0, 0] = 1
        theta[:, 1, 1] = 1
        theta[:, 0, 2] = shifts[:, n, 0] * 2 * ds * 2 / Wr
        theta[:, 1, 2] = shifts[:, n, 1] * 2 * ds * 2 / Hr
        grid = F.affine_grid(theta, (B, 3, Hr, Wr), align_corners=False)
        sh = F.grid_sample(img, grid, mode='bilinear', padding_mode='border', align_corners=False)
        rgb = F.avg_pool2d(sh, ds)                                   # [B,3,2H,2W]
        raw = torch.stack((rgb[:, 0, 0::2, 0::2], rgb[:, 1, 0::2, 1::2],
                           rgb[:, 1, 1::2, 0::2], rgb[:, 2, 1::2, 1::2]), dim=1)   # [B,4,H,W]
        if noise:
            shot, read = 0.01, 0.0005
            var = raw * shot + read
            raw = raw + torch.randn(raw.shape, generator=g) * var.sqrt()
        frames.append(raw.clamp(0.0, 1.0))
    burst = torch.stack(frames, dim=1).contiguous()
    return burst, gt.contiguous()
