"""Timeline of one bench-shape forward from HIP events, without a profiler (rocprofv3 delays the side lane's start in a
replayed graph): every op of the plan is bracketed by events on the stream it runs on, all queued
behind a spin kernel, and each op's start / end is reported relative to an event recorded on the main stream before
the fork.  Eager launches (not the graph), lanes on their own streams as Plan.run issues them.

Usage: python tools/lane_events.py [--batch 8 --frames 14 --size 48 --dtype fp16 --reps 3]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=8)
    ap.add_argument('--frames', type=int, default=14)
    ap.add_argument('--size', type=int, default=48)
    ap.add_argument('--dtype', default='fp16')
    ap.add_argument('--reps', type=int, default=3)
    ap.add_argument('--share', type=float, default=None, help='DBSREngine.LANE0_CU_SHARE override')
    args = ap.parse_args()
    import dbsr_amd
    from dbsr_amd import _lib as L
    from dbsr_amd.burst import synthetic_bursts
    from dbsr_amd.engine import DBSREngine, Plan
    if args.share is not None:
        DBSREngine.LANE0_CU_SHARE = args.share
    dev = torch.device('cuda', 0)
    net = dbsr_amd.build_synthetic_net(seed=0).to(dev).eval()
    net.set_compute_dtype({'fp16': torch.float16, 'bf16': torch.bfloat16}[args.dtype])
    net.use_graph = True
    B, N, S = args.batch, args.frames, args.size
    burst, _ = synthetic_bursts(B, N, S, S, sr_factor=8, seed=1000)
    burst = burst.to(dev)
    with torch.no_grad():
        for _ in range(3):
            net(burst)
        torch.cuda.synchronize()
        import time
        t0 = time.perf_counter()
        for _ in range(20):
            net(burst)
        torch.cuda.synchronize()
        print('graph step %.3f ms' % ((time.perf_counter() - t0) / 20 * 1e3))
        plan = net._engine.plans[(B, N, S, S)]
        main_s = torch.cuda.current_stream()
        acc = {}
        for rep in range(args.reps):
            torch.cuda._sleep(40_000_000)
            base = torch.cuda.Event(enable_timing=True)
            base.record(main_s)
            evs = []
            for fn, a, name, lane in plan.ops:
                if fn is Plan.FORK:
                    a[0].record(main_s)
                    plan.streams[lane].wait_event(a[0])
                    continue
                if fn is Plan.JOIN:
                    a[0].record(plan.streams[lane])
                    main_s.wait_event(a[0])
                    continue
                st = main_s if lane == 0 else plan.streams[lane]
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                rc = fn(*a, main_s.cuda_stream if lane == 0 else st.cuda_stream)
                if rc != 0:
                    L.check(rc, name)
                e1.record(st)
                evs.append((name, lane, e0, e1))
            end = torch.cuda.Event(enable_timing=True)
            end.record(main_s)
            torch.cuda.synchronize()
            for i, (name, lane, e0, e1) in enumerate(evs):
                s, e = base.elapsed_time(e0) * 1e3, base.elapsed_time(e1) * 1e3
                k = (i, name, lane)
                acc.setdefault(k, [0.0, 0.0])
                acc[k][0] += s / args.reps
                acc[k][1] += e / args.reps
            acc.setdefault('total', 0.0)
            acc['total'] += base.elapsed_time(end) * 1e3 / args.reps
    total = acc.pop('total')
    lanes = {}
    for (i, name, lane), (s, e) in sorted(acc.items()):
        print('%8.1f %8.1f %7.1f  L%d  %s' % (s, e, e - s, lane, name))
        lo, hi, busy = lanes.get(lane, (1e18, 0.0, 0.0))
        lanes[lane] = (min(lo, s), max(hi, e), busy + e - s)
    for lane, (lo, hi, busy) in sorted(lanes.items()):
        print('lane %d: %.1f .. %.1f us, busy %.1f us' % (lane, lo, hi, busy))
    print('eager forward with events: %.1f us' % total)


if __name__ == '__main__':
    main()
