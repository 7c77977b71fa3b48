import os, sys, torch
sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), 'tests'))
import test_gpu_fuse as T
for case in [(2, 14, 48, 48, 128, 512, torch.bfloat16), (1, 14, 32, 16, 128, 128, torch.float16)]:
    B, N, H, W, cin, C, dt = case
    outs, (rf, rw) = T._case(B, N, H, W, cin, C, dt, seed=B * 100 + H + C)
    f1, w1 = outs[True]
    bad = ~torch.isfinite(w1) | ((w1 - rw).abs() > 1e-2)
    print(case, 'bad weights', int(bad.sum()), 'of', bad.numel(), 'fused bad', int((~torch.isfinite(f1) | ((f1 - rf).abs() > 5e-2)).sum()))
    if bad.any():
        idx = bad.nonzero()
        f = idx[:, 0]; y = idx[:, 1]; x = idx[:, 2]; c = idx[:, 3]
        print(' frames', torch.unique(f).tolist()[:20])
        print(' rows', torch.unique(y).tolist()[:50])
        print(' cols', torch.unique(x).tolist()[:50])
        print(' chans', torch.unique(c // 32).tolist()[:20], 'c%32', torch.unique(c % 32).tolist())
        print(' sample', idx[:10].tolist(), w1[tuple(idx[:5].T)].tolist(), rw[tuple(idx[:5].T)].tolist())
