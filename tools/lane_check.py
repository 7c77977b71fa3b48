"""Eager vs graph vs single-stream consistency of the DBSR forward (debug aid for the lane plan)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import dbsr_amd
from dbsr_amd import engine
from dbsr_amd.burst import synthetic_bursts

DEV = 'cuda:0'


def run(multi, graph, burst, reps=3):
    engine.Plan.MULTI_STREAM = multi
    net = dbsr_amd.build_synthetic_net(seed=0).to(DEV).eval()
    net.set_compute_dtype(torch.bfloat16)
    net.use_graph = graph
    outs = []
    with torch.no_grad():
        for _ in range(reps):
            p, a = net(burst)
            torch.cuda.synchronize()
            outs.append((p.clone(), a['offsets'].clone()))
    return outs


B, N, S = int(sys.argv[1]) if len(sys.argv) > 1 else 1, 4, 48
burst = synthetic_bursts(B, N, S, S, sr_factor=8, seed=3)[0].to(DEV)
res = {}
for multi in (False, True):
    for graph in (False, True):
        res[(multi, graph)] = run(multi, graph, burst)
ref_p, ref_o = res[(False, False)][0]
for k, outs in res.items():
    for i, (p, o) in enumerate(outs):
        print(k, i, 'pred maxdiff %.3g' % (p - ref_p).abs().max().item(), 'offs maxdiff %.3g' % (o - ref_o).abs().max().item(),
              'offs absmax %.3g' % o.abs().max().item())
