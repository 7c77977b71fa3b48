"""A/B of the two-lane schedule on the bench workload (diagnostic, GPU box): bursts/s of the fp16 forward
with the default plan (one multi-branch HIP graph, PWC-Net on a normal-priority side lane) against other
side-lane priorities, CU shares, eager multi-stream launches (no graph) and one stream.  Each variant builds a
fresh engine in this process, in the order given (engines built one after another exposed the
high-priority side stream's bimodal slowdown).
python tools/lane_ab.py <variant> ...  (variants: VARIANTS below)"""
import gc
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dbsr_amd  # noqa: E402
from dbsr_amd import engine as E  # noqa: E402
from dbsr_amd.burst import synthetic_bursts  # noqa: E402

dev = torch.device('cuda', 0)
B, N, S = 8, 14, 48
burst, _ = synthetic_bursts(B, N, S, S, sr_factor=8, seed=1000)
burst = burst.to(dev)
orig_fork = E.Plan.fork


def run(tag, graph=True, prio=None, single=False, steps=40, share=0.5):
    E.Plan.MULTI_STREAM = not single
    E.DBSREngine.LANE0_CU_SHARE = share
    if prio is not None:
        E.Plan.fork = lambda self, lane, device, priority=0: orig_fork(self, lane, device, priority=prio)
    else:
        E.Plan.fork = orig_fork
    net = dbsr_amd.build_synthetic_net(seed=0).to(dev).eval().set_compute_dtype(torch.float16)
    net.use_graph = graph
    with torch.no_grad():
        for _ in range(5):
            net(burst)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            net(burst)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
    print('%-34s %8.1f bursts/s  %.3f ms/step' % (tag, B * steps / el, el / steps * 1e3), flush=True)
    del net
    if os.environ.get('LANE_AB_GC', '1') == '1':
        gc.collect()              # the engine <-> net reference cycle keeps the old HIP graphs alive otherwise
    torch.cuda.empty_cache()


VARIANTS = {
    'default': dict(),
    's625': dict(share=0.625), 's375': dict(share=0.375),
    'prio0': dict(prio=0), 'eager': dict(graph=False), 'single': dict(single=True),
    'prio_hi': dict(prio=-1),
}
# variants run in this order in one process (each builds a fresh engine; the side streams are shared)
for v in sys.argv[1:]:
    run(v, **VARIANTS[v])
