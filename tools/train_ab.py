"""Same-box A/B of training-step schedule flags (diagnostic, GPU box): ms per DBSRTrainer.step at configs[3]'s shape
(B=8, 14 x 128^2, bf16) for each variant, alternating in one process, each on a fresh trainer.
python tools/train_ab.py <variant> ...   (variants: VARIANTS below)"""
import gc
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dbsr_amd  # noqa: E402
from dbsr_amd.burst import synthetic_bursts  # noqa: E402
from dbsr_amd.training import DBSRTrainer  # noqa: E402

VARIANTS = {'default': dict(), 'repack0': dict(BATCH_REPACK=False), 'fuse0': dict(FUSED_WP_OUT=False)}   # (r06l also had a wgrad side-lane flag)
dev = torch.device('cuda', 0)
burst, gt = synthetic_bursts(8, 14, 128, 128, sr_factor=8, seed=2000)
burst, gt = burst.to(dev), gt.to(dev)
base = {k: getattr(DBSRTrainer, k) for v in VARIANTS.values() for k in v}
for name in sys.argv[1:]:
    for k, v in base.items():
        setattr(DBSRTrainer, k, v)
    for k, v in VARIANTS[name].items():
        setattr(DBSRTrainer, k, v)
    net = dbsr_amd.build_synthetic_net(seed=0).to(dev).set_compute_dtype(torch.bfloat16)
    tr = DBSRTrainer(net)
    for _ in range(3):
        tr.step(burst, gt)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    steps = 10
    for _ in range(steps):
        loss = tr.step(burst, gt)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print('%-10s %.3f ms/step  loss %.6f' % (name, el / steps * 1e3, float(loss)), flush=True)
    del tr, net
    gc.collect()
    torch.cuda.empty_cache()
