"""Locate the two-lane nondeterminism: snapshot every plan buffer after a two-lane forward and diff it
against the single-stream forward on the same input.  The first buffer (in plan order) that differs
names the victim op; `touch` lists every op whose arguments point into that buffer.

Run modes (RB_MODES, comma separated):
  normal      Plan.run (fork/join events)
  side_only   only the side lane's ops (PWC-Net + offset features), nothing on lane 0
  sync_side   lane-0 ops enqueued first, then each side op followed by a host sync of the side stream
  sync_all    every op followed by a device sync (lane streams kept)

usage: python tools/race_bisect.py [B N H W] ; env RB_ALGO=<conv algo> RB_RUNS=<forwards>
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import dbsr_amd
from dbsr_amd import _lib, engine
from dbsr_amd.burst import synthetic_bursts

B, N, H, W = [int(v) for v in (sys.argv[1:5] if len(sys.argv) > 4 else (8, 14, 48, 48))]
RUNS = int(os.environ.get('RB_RUNS', '3'))
MODES = os.environ.get('RB_MODES', 'normal').split(',')
if os.environ.get('RB_ALGO'):
    _lib.lib().dbsr_set_conv_algo(int(os.environ['RB_ALGO']))


def tensors(obj, path, out, seen):
    if isinstance(obj, torch.Tensor):
        if obj.is_cuda and obj.data_ptr() not in seen:
            seen.add(obj.data_ptr())
            out.append((path, obj))
    elif isinstance(obj, engine.NHWC):
        tensors(obj.t, path, out, seen)
    elif isinstance(obj, (list, tuple)):
        for i, o in enumerate(obj):
            tensors(o, '%s[%d]' % (path, i), out, seen)
    elif isinstance(obj, dict):
        for k, o in obj.items():
            tensors(o, '%s.%s' % (path, k), out, seen)


def op_ptrs(args):
    ptrs = []
    for a in args:
        o = getattr(a, '_obj', a)
        if isinstance(o, _lib.ConvDesc):
            for f in ('x', 'y', 'res'):
                p = getattr(o, f).ptr
                if p:
                    ptrs.append((f, p))
            if o.workspace:
                ptrs.append(('ws', o.workspace))
        elif isinstance(o, _lib.Tensor):
            if o.ptr:
                ptrs.append(('t', o.ptr))
        elif isinstance(o, int) and o > 1 << 32:
            ptrs.append(('p', o))
    return ptrs


def buffers(plan):
    bl = []
    tensors(plan.keep, 'keep', bl, set())
    tensors(plan.bufs, 'bufs', bl, set())
    return bl


def run_mode(plan, mode):
    main = torch.cuda.current_stream()
    stream = main.cuda_stream
    if mode == 'normal':
        if os.environ.get('RB_POISON'):
            # poison the outputs of the named ops (their last tensor argument) before the run
            for fn, args, name, lane in plan.ops:
                if name in os.environ['RB_POISON'].split('+'):
                    out = [a for a in args if isinstance(a, _lib.Tensor)][-1]
                    for _, t in buffers(plan):
                        if t.data_ptr() == out.ptr:
                            t.fill_(float('nan'))
        plan.run(stream)
        return
    side_ops = [op for op in plan.ops if op[3] != 0 and op[0] not in (engine.Plan.FORK, engine.Plan.JOIN)]
    fork = [op for op in plan.ops if op[0] is engine.Plan.FORK]
    pre = []
    for op in plan.ops:
        if op[0] is engine.Plan.FORK:
            break
        pre.append(op)
    after_fork_main = []
    state = 0
    for op in plan.ops:
        if op[0] is engine.Plan.FORK:
            state = 1
            continue
        if op[0] is engine.Plan.JOIN:
            break
        if state == 1 and op[3] == 0:
            after_fork_main.append(op)
    side = plan.streams[1]
    plan.run_list(pre, stream)
    ev = fork[0][1][0]
    ev.record(main)
    side.wait_event(ev)
    if mode == 'side_only':
        plan.run_list(side_ops, side.cuda_stream)
    elif mode == 'side_dummy':
        # lane 0 busy with unrelated torch work (no DBSR kernel) while the side lane runs
        a = torch.randn(4096, 4096, device='cuda', dtype=torch.bfloat16)
        for _ in range(20):
            a = (a @ a).clamp_(-1, 1)
        plan.run_list(side_ops, side.cuda_stream)
    elif mode.startswith('bwloop:'):
        # lane 0: the encoder's pipelined convs; side lane: only the PWC backwarp ops (pure VALU
        # gather kernels, no LDS, no MFMA), repeated -- the victims of the co-residency corruption
        reps = int(mode.split(':')[1])
        plan.run_list(plan.ops, stream)          # serial pass: every buffer holds its correct value
        torch.cuda.synchronize()
        ev.record(main)
        side.wait_event(ev)
        sel = [op for op in after_fork_main if 'enc.res' in op[2] or 'enc.out' in op[2]]
        bw = [op for op in side_ops if op[2].endswith('.backwarp')]
        for _ in range(2):
            plan.run_list(sel, stream)
        for _ in range(reps):
            plan.run_list(bw, side.cuda_stream)
    elif mode.startswith('sub:'):
        # lane 0 runs only its ops whose name contains the filter, repeated, beside the side lane
        _, filt, reps = mode.split(':')
        sel = [op for op in after_fork_main if filt in op[2]]
        for _ in range(int(reps)):
            plan.run_list(sel, stream)
        plan.run_list(side_ops, side.cuda_stream)
    elif mode == 'sync_side':
        plan.run_list(after_fork_main, stream)
        for op in side_ops:
            plan.run_list([op], side.cuda_stream)
            side.synchronize()
    elif mode == 'sync_all':
        plan.run_list(after_fork_main, stream)
        for op in side_ops:
            plan.run_list([op], side.cuda_stream)
            torch.cuda.synchronize()
    torch.cuda.synchronize()


def run(multi, mode):
    engine.Plan.MULTI_STREAM = multi
    net = dbsr_amd.build_synthetic_net(seed=0).cuda().eval()
    net.set_compute_dtype(torch.bfloat16)
    snaps = []
    with torch.no_grad():
        net(burst)                         # builds the plan (normal run)
        torch.cuda.synchronize()
        plan = net._engine.plans[(B, N, H, W)]
        for _ in range(RUNS):
            run_mode(plan, mode) if multi else plan.run(torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            snaps.append([(p, t.clone()) for p, t in buffers(plan)])
    return plan, snaps


burst = synthetic_bursts(B, N, H, W, sr_factor=8, seed=9)[0].cuda()
plan_s, ref = run(False, None)
ref_last = ref[-1]
print('single-stream self-consistency:', all(torch.equal(a[1], b[1]) for a, b in zip(ref[0], ref[-1])))
for mode in MODES:
    plan_m, mul = run(True, mode)
    live = buffers(plan_m)
    side_names = {op[2] for op in plan_m.ops if op[3] != 0}
    for r, snap in enumerate(mul):
        nd = 0
        for (path, t), (rpath, rt), (lpath, lt) in zip(snap, ref_last, live):
            if t.shape != rt.shape:
                print('shape mismatch', path, rpath)
                continue
            if mode in ('side_only', 'side_dummy') or mode.startswith(('sub:', 'bwloop:')):
                # only buffers written by side-lane ops are comparable
                lo, hi = lt.data_ptr(), lt.data_ptr() + lt.numel() * lt.element_size()
                writers = [op[2] for op in plan_m.ops if op[0] not in (engine.Plan.FORK, engine.Plan.JOIN)
                           and any(lo <= p < hi for f, p in op_ptrs(op[1]) if f in ('y', 't', 'p'))]
                if not writers or not all(w in side_names for w in writers):
                    continue
            if not torch.equal(t, rt):
                nd += 1
                d = (t.float() - rt.float()).abs()
                if nd <= 4:
                    lo, hi = lt.data_ptr(), lt.data_ptr() + lt.numel() * lt.element_size()
                    touch = []
                    for fn, args, name, lane in plan_m.ops:
                        if fn in (engine.Plan.FORK, engine.Plan.JOIN):
                            continue
                        for f, p in op_ptrs(args):
                            if lo <= p < hi:
                                touch.append('%s:%s@L%d' % (name, f, lane))
                    nz = (d > 0).nonzero()
                    bad = nz[:, 0].unique().tolist()
                    print('%s run %d DIFF %-14s %-20s maxdiff %.4g ndiff %d imgs %s first %s touch %s' % (
                        mode, r, path, tuple(t.shape), d.max().item(), int((d > 0).sum()), bad[:8],
                        tuple(nz[0].tolist()), touch))
                    if nd == 1:
                        idx = [tuple(v) for v in nz[:12].tolist()]
                        print('   at  ', idx)
                        print('   mine', [round(t[i].float().item(), 5) for i in idx])
                        print('   ref ', [round(rt[i].float().item(), 5) for i in idx])
        print('%s run %d: %d of %d buffers differ' % (mode, r, nd, len(snap)))


def stray_check():
    """Serial run of a two-lane plan: after the side lane's ops, run every later op alone and report
    the first op that changes a buffer that only side-lane ops write (a stray write)."""
    engine.Plan.MULTI_STREAM = True
    net = dbsr_amd.build_synthetic_net(seed=0).cuda().eval()
    net.set_compute_dtype(torch.bfloat16)
    with torch.no_grad():
        net(burst)
        torch.cuda.synchronize()
    plan = net._engine.plans[(B, N, H, W)]
    st = torch.cuda.current_stream().cuda_stream
    ops = [op for op in plan.ops if op[0] not in (engine.Plan.FORK, engine.Plan.JOIN)]
    side_names = {op[2] for op in ops if op[3] != 0}
    live = buffers(plan)
    ws = [(f'ws{l}', t) for l, t in plan.ws.items()]
    watch = []
    for path, t in live + ws:
        lo, hi = t.data_ptr(), t.data_ptr() + t.numel() * t.element_size()
        writers = [op[2] for op in ops if any(lo <= p < hi for f, p in op_ptrs(op[1]) if f in ('y', 't', 'p', 'ws'))]
        if path.startswith('ws1') or (writers and all(w in side_names for w in writers)):
            watch.append((path, t, lo, hi))
    print('watching %d side-lane buffers' % len(watch))
    with torch.no_grad():
        for rep in range(2):
            snap = None
            for i, op in enumerate(ops):
                plan.run_list([op], st)
                torch.cuda.synchronize()
                if op[3] != 0:
                    snap = [t.clone() for _, t, _, _ in watch]     # state after the latest side op
                    continue
                if snap is None:
                    continue
                for (path, t, lo, hi), s in zip(watch, snap):
                    if not torch.equal(t, s):
                        d = (t.float() - s.float()).abs()
                        nz = (d > 0).nonzero()
                        print('rep %d STRAY by op %-24s into %-14s %s ndiff %d first %s' % (
                            rep, op[2], path, tuple(t.shape), int((d > 0).sum()), tuple(nz[0].tolist())))
                snap = [t.clone() for _, t, _, _ in watch]


if os.environ.get('RB_STRAY', '0') == '1':
    stray_check()
