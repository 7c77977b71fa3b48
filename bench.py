"""Throughput benchmark of the MI355X DBSR forward (BASELINE.json metric: bursts/s on
SyntheticBurstVal-shaped 14x48x48 RAW bursts -> 384x384 RGB, configs[1]: bf16, batch 8 per GPU).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch 8] [--frames 14] [--size 48]
                  [--dtype fp16|bf16|fp32] [--no-graph] [--no-cpu-baseline]

One process per GPU.  Under torchrun (WORLD_SIZE set) this process is one rank; with --gpus N > 1 and no
WORLD_SIZE, bench.py itself starts the N ranks (torch.distributed.run, before anything touches the GPU)
and exits with their status.  Every rank runs its own shard of the global batch (N x --batch independent
bursts; the path shards over bursts with no data-path collective: weak scaling).

Storage dtype: fp16 by default.  bf16 (configs[1]'s text) misses the metric's "PSNR within 0.01 dB" bar:
0.01 dB at the reference's published 39.17 dB is an RMS prediction error of 5.3e-4, and bf16 storage gives
~2.9e-3 against the fp32 oracle, fp16 ~4e-4 (tests/test_gpu_parity.py, DESIGN.md "Precision").  fp16 and
bf16 run at the same dense MFMA rate (2.5 PF) and move the same bytes.  A step = one full forward
(PWC-Net alignment, encoder, warp, merging/fusion incl. the fusion_weights aux output, decoder) over
one batch of synthetic bursts already resident in HBM, replayed as one HIP graph.  Timing: W untimed
steps, then K steps bracketed by barrier + synchronize, max over ranks.  Rank 0 prints one JSON line.
"""
import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

PEAK_HBM_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
PEAK_MFMA_TFLOPS = {'bf16': 2500.0, 'fp16': 2500.0, 'fp32': 157.3}   # dense peaks (MI355X_MICROARCH.md chip table)
DTYPES = {'bf16': 'bfloat16', 'fp16': 'float16', 'fp32': 'float32'}
# conv-like kernel families (MFMA-bound; bench reports each against the dense peak)
CONV_FAMILIES = ('conv3x3_ws', 'conv3x3_ks128', 'conv3x3_pipe', 'conv3x3_tiled', 'conv3x3_narrow', 'conv3x3_small', 'conv2d_generic', 'conv1x1',
                 'conv1x1_shuffle', 'conv1x1_shuffle_blur', 'resblock32', 'resblock64', 'conv_fuse', 'pwc_dense',
                 'pwc_extract')
KERNEL_DESC = {'conv3x3_ws': 'conv3x3_ws_kernel (persistent weight-stationary implicit-GEMM 3x3, Cin <= 64',
               'conv3x3_ks128': 'conv3x3_ks128_kernel (persistent K-split weight-stationary 128 -> 128 3x3: the '
                                'weight predictor',
               'conv3x3_pipe': 'conv3x3_pipe_kernel (persistent LDS-DMA-pipelined implicit-GEMM 3x3',
               'conv3x3_tiled': 'conv3x3_tiled_kernel (LDS-tiled implicit-GEMM 3x3',
               'conv3x3_narrow': 'conv3x3_narrow_kernel (cout <= 4 over a long K: the level-2 flow head',
               'conv3x3_small': 'conv3x3_small_kernel (3x3 of an 8-channel input, weights in registers: the encoder / '
                                'offset-feature first convs',
               'conv2d_generic': 'conv2d_kernel (generic implicit-GEMM',
               'conv1x1': 'conv1x1_kernel (pointwise projection, LDS-resident weights',
               'conv1x1_shuffle': 'upsample_shuffle_kernel (1x1 conv + PixelShuffle',
               'conv1x1_shuffle_blur': 'upsample_blur_kernel (1x1 conv + PixelShuffle + 3x3 Gaussian blur',
               'resblock32': 'resblock32_kernel (a whole 32-channel ResBlock, intermediate in the LDS',
               'resblock64': 'resblock64_kernel (a whole 64-channel ResBlock: conv1 / conv2 wave roles pipelined over '
                             'tiles, intermediate in the LDS',
               'conv_fuse': 'conv_fuse_kernel (weight-predictor output conv + softmax + fusion',
               'pwc_dense': 'pwc_dense_kernel (PWC-Net DenseNet decoder level in one launch',
               'pwc_extract': 'pwc_extract_kernel (PWC-Net feature pyramid in one launch'}
# PMC traffic per launch of each kernel family, from the committed rocprofv3 --pmc passes of this same
# command (tools/profile.sh -> tools/summarize_profile.py); bench.py cannot read its own counters
TRAFFIC_FILE = os.path.join(REPO, 'profiles', 'pmc_traffic.json')


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--batch', type=int, default=8)
    ap.add_argument('--frames', type=int, default=14)
    ap.add_argument('--size', type=int, default=48)
    ap.add_argument('--dtype', default=None, choices=['fp16', 'bf16', 'fp32'],
                    help='storage dtype (default fp16 for --mode infer, bf16 for --mode train)')
    ap.add_argument('--no-graph', action='store_true')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-seconds', type=float, default=15.0)
    ap.add_argument('--kernel-breakdown', action='store_true', help='print per-op device times to stderr')
    ap.add_argument('--wgrad-algo', type=int, default=None,
                    help='diagnostic A/B: dbsr_set_wgrad_algo value (1 LDS-DMA ring, 0 register-staged)')
    ap.add_argument('--conv-algo', type=int, default=None,
                    help='diagnostic A/B: dbsr_set_conv_algo value (include/dbsr_hip.h); default: the library default')
    ap.add_argument('--no-op-timing', action='store_true',
                    help='skip the per-op timing passes after the timed region (profiling runs: only graph replays)')
    ap.add_argument('--zero-flow', action='store_true', help='diagnostic: identity-flow stub instead of PWC-Net')
    ap.add_argument('--mode', default='infer', choices=['infer', 'train'],
                    help='train: configs[3] training step (defaults 128x128, batch 8 per GPU, RCCL grad all-reduce)')
    ap.add_argument('--dry-run', action='store_true',
                    help='CPU check of the rank launcher: gloo, no GPU; rank 0 prints every rank\'s batch shard')
    return ap.parse_args()


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n):
    """--gpus n > 1 outside torchrun: run this same command as n ranks of one node (torch.distributed.run,
    rendezvous on 127.0.0.1) as a CHILD process -- this process has not touched the GPU and never execs --
    and return the launcher's exit status (admin/multigpu.py:8-14 is the reference's single-process
    nn.DataParallel; here it is one process per GPU)."""
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={n}',
           '--master-addr=127.0.0.1', f'--master-port={_free_port()}', os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def cpu_model():
    try:
        for line in open('/proc/cpuinfo'):
            if line.startswith('model name'):
                return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return 'unknown'


def load_traffic():
    try:
        return json.load(open(TRAFFIC_FILE))
    except (OSError, ValueError):
        return {}


def dry_run(args, world, rank):
    """The launcher's rank layout without a GPU: every rank derives its shard of the global batch exactly as
    the GPU path does, and rank 0 all-gathers and prints them."""
    import torch.distributed as td
    from dbsr_amd.parallel import shard_range
    td.init_process_group('gloo')
    gb = args.batch * world
    lo, hi = shard_range(gb, rank, world)
    t = torch.tensor([rank, world, lo, hi], dtype=torch.int64)
    got = [torch.zeros_like(t) for _ in range(world)]
    td.all_gather(got, t)
    if rank == 0:
        print(json.dumps({'dry_run': True, 'n_gpus': world, 'global_batch': gb,
                          'ranks': [g.tolist() for g in got]}))
    td.destroy_process_group()


def train_main(args, world, rank, dev, dist):
    """configs[3]: SyntheticBurst 14-frame 128x128 -> 1024x1024 training step (forward, L1 loss, backward,
    bucketed RCCL gradient all-reduce over the ranks, Adam), bf16, batch 8 per GPU (global 8 * N)."""
    import dbsr_amd
    from dbsr_amd.burst import synthetic_bursts
    from dbsr_amd.training import DBSRTrainer
    B, N, S = args.batch, args.frames, (args.size if args.size != 48 else 128)
    dtype = getattr(torch, DTYPES[args.dtype])
    net = dbsr_amd.build_synthetic_net(seed=0).to(dev).set_compute_dtype(dtype)
    tr = DBSRTrainer(net)
    burst, gt = synthetic_bursts(B, N, S, S, sr_factor=8, seed=2000 + rank)
    burst, gt = burst.to(dev), gt.to(dev)
    for _ in range(max(1, args.warmup)):
        tr.step(burst, gt)
    torch.cuda.synchronize()
    if dist:
        import torch.distributed as td
        td.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = tr.step(burst, gt)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if dist:
        from dbsr_amd.parallel import max_over_ranks
        el = max_over_ranks(el, device=dev)
    # per-op device times of the step (HIP events, every op re-launched back to back, outside the timed region;
    # --no-op-timing: profiling runs, the step's own replays only)
    plan = tr.plans[(B, N, S, S)]
    times = None if args.no_op_timing else plan.time_ops(torch.cuda.current_stream(dev).cuda_stream, reps=3)
    fam = {}
    for i, (fn, _, name, _) in enumerate(plan.ops):
        if name.startswith('sync.'):
            continue
        kind = plan.kernel.get(i) or name.split('.')[0]
        f = fam.setdefault(kind, [0.0, 0.0, 0])
        f[0] += times[i][1] if times is not None else 0.0
        f[1] += plan.work[i][1] if (i in plan.work and plan.work[i][0] == 'flop') else 0.0
        f[2] += 1
    step_flop = sum(w for _, w, _ in fam.values())
    ms_step = el / args.steps * 1e3
    peak_t = PEAK_MFMA_TFLOPS[args.dtype]
    step_tf = step_flop / (ms_step * 1e-3) / 1e12
    if args.kernel_breakdown and rank == 0 and times is not None:
        for i, (name, ms) in enumerate(times):
            if name.startswith('sync.'):
                continue
            kind = plan.kernel.get(i) or '-'
            w = plan.work[i][1] if (i in plan.work and plan.work[i][0] == 'flop') else 0.0
            rate = '%8.1f TF/s' % (w / (ms * 1e-3) / 1e12) if (w and ms) else ''
            print(f'{name:40s} {ms * 1e3:9.1f} us  {kind:15s} {rate}', file=sys.stderr)
        for k, (ms, w, n) in sorted(fam.items(), key=lambda kv: -kv[1][0]):
            rate = (' %7.1f TF/s' % (w / (ms * 1e-3) / 1e12)) if w else ''
            print(f'[family] {k:16s} {ms * 1e3:10.1f} us  n={n}{rate}', file=sys.stderr)
        print(f'sum of op times {sum(t for _, t in times) * 1e3:.1f} us vs step {ms_step * 1e3:.1f} us',
              file=sys.stderr)
    conv_fams = {k: v for k, v in fam.items() if v[1] > 0}
    dom = max(conv_fams, key=lambda k: conv_fams[k][0]) if times is not None else None
    d_ms, d_flop, d_n = conv_fams[dom] if dom else (0.0, 0.0, 0)
    if rank == 0:
        print(json.dumps({
            'metric': 'training bursts/sec 14x%dx%d RAW->x8 (configs[3] step shape)' % (S, S),
            'value': round(world * B * args.steps / el, 3), 'unit': 'bursts/s', 'n_gpus': world,
            'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': round(el / args.steps * 1e3, 3),
            'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': args.dtype,
            'data': 'synthetic (seeded bursts, seeded random weights)', 'loss': float(loss),
            'config': {'workload': 'configs[3]: forward + L1 loss + backward + bucketed RCCL all-reduce + Adam',
                       'global_batch': B * world, 'frames': N, 'height': S, 'width': S,
                       'parallelism': 'dp%d (DDP-style gradient all-reduce)' % world,
                       'hip_graph': tr.use_graph},
            # whole step: the algorithmic conv FLOPs of the step (forward incl. PWC-Net, dgrad, wgrad) over the
            # timed step time, against the dense MFMA peak of the compute dtype
            'step_roofline': {'bound': 'mfma', 'achieved': round(step_tf, 2), 'peak': peak_t, 'unit': 'TFLOP/s',
                              'frac': round(step_tf / peak_t, 4), 'flop_per_step': step_flop},
            'roofline': ({'bound': 'mfma', 'kernel': '%s family, %d launches per step' % (dom, d_n),
                          'achieved': round(d_flop / (d_ms * 1e-3) / 1e12, 2), 'peak': peak_t, 'unit': 'TFLOP/s',
                          'frac': round(d_flop / (d_ms * 1e-3) / 1e12 / peak_t, 4), 'traffic': None} if dom else None),
            'roofline_families': ({k: {'ms': round(ms, 3), 'launches': n,
                                       'frac': round(w / (ms * 1e-3) / 1e12 / peak_t, 4)}
                                   for k, (ms, w, n) in conv_fams.items()} if dom else None)}))


def cpu_baseline(N, H, W, seconds):
    """Oracle (torch-CPU restatement of the reference forward, oracle/dbsr_oracle.py) timed on this
    node's host cores on a bounded sample: batch-1 bursts of the same workload, fp32, until
    `seconds` of CPU work have elapsed."""
    from oracle import dbsr_oracle as orc
    import dbsr_amd
    from dbsr_amd import arch
    from dbsr_amd.weights import generate_state_dict
    from dbsr_amd.burst import synthetic_bursts
    net = dbsr_amd.dbsrnet_cvpr2021(**dbsr_amd.DBSR_SYNTHETIC_KWARGS)
    sd = orc.state_dict_to_torch(generate_state_dict(arch.state_dict_shapes(net), seed=0))
    burst, _ = synthetic_bursts(1, N, H, W, sr_factor=8, seed=1)
    with torch.no_grad():
        orc.dbsr_forward(burst, sd)              # warm-up
        n, t0 = 0, time.perf_counter()
        while True:
            orc.dbsr_forward(burst, sd)
            n += 1
            el = time.perf_counter() - t0
            if el >= seconds or n >= 50:
                break
    return {'value': n / el, 'unit': 'bursts/s', 'cores': torch.get_num_threads(), 'kind': 'port',
            'cpu_model': cpu_model(), 'host_cpus': os.cpu_count(),
            'cores_note': 'torch intra-op threads = OMP_NUM_THREADS (%s): the GPU box allots 16 CPUs per GPU of its '
                          '%d host CPUs, so the baseline runs on that share, not on all of them'
                          % (os.environ.get('OMP_NUM_THREADS', 'unset'), os.cpu_count()),
            'sample': f'{n} batch-1 bursts of {N}x{H}x{W} (fp32 oracle/dbsr_oracle.py, {el:.1f} s)'}


def main():
    args = parse()
    if args.dtype is None:
        args.dtype = 'bf16' if args.mode == 'train' else 'fp16'
    if args.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world != args.gpus:
        raise SystemExit(f'bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: one rank per GPU')
    if args.dry_run:
        return dry_run(args, world, rank)
    dist = world > 1
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)
    if dist:
        import torch.distributed as td
        td.init_process_group('nccl', device_id=dev)

    if args.wgrad_algo is not None:
        from dbsr_amd import _lib
        _lib.check(_lib.lib().dbsr_set_wgrad_algo(args.wgrad_algo), 'dbsr_set_wgrad_algo')
    if args.mode == 'train':
        train_main(args, world, rank, dev, dist)
        if dist:
            td.destroy_process_group()
        return
    import dbsr_amd
    from dbsr_amd.burst import synthetic_bursts
    from dbsr_amd.parallel import shard_range
    dtype = getattr(torch, DTYPES[args.dtype])
    if args.conv_algo is not None:
        from dbsr_amd import _lib
        _lib.check(_lib.lib().dbsr_set_conv_algo(args.conv_algo), 'dbsr_set_conv_algo')
    net = dbsr_amd.build_synthetic_net(seed=0).to(dev).eval()
    net.set_compute_dtype(dtype)
    net.use_graph = not args.no_graph
    net.zero_flow = args.zero_flow
    B, N, S = args.batch, args.frames, args.size
    lo, hi = shard_range(B * world, rank, world)     # this rank's bursts [lo, hi) of the global batch
    assert hi - lo == B
    burst, _ = synthetic_bursts(B, N, S, S, sr_factor=8, seed=1000 + lo)
    burst = burst.to(dev)

    with torch.no_grad():
        for _ in range(max(1, args.warmup)):
            net(burst)
        torch.cuda.synchronize()
        if dist:
            td.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            net(burst)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        if dist:
            from dbsr_amd.parallel import max_over_ranks
            el = max_over_ranks(el, device=dev)
            td.barrier()

        # ---- per-kernel device times (HIP events), outside the timed region: inside the step as the step runs
        # them (lanes concurrent, lane-0 convs capped while PWC-Net runs), and each op alone on the whole chip ----
        eng = net._engine
        plan = eng.plans[(B, N, S, S)]
        times, times_chip = None, None
        if not args.no_op_timing:
            cur = torch.cuda.current_stream(dev).cuda_stream
            times = plan.time_ops_in_step(cur, reps=5)
            times_chip = plan.time_ops(cur, reps=10)

    ms_step = el / args.steps * 1e3
    value = world * B * args.steps / el
    is_conv = lambda k: k in CONV_FAMILIES                  # noqa: E731
    peak_t = PEAK_MFMA_TFLOPS[args.dtype]
    traffic = load_traffic() if args.dtype != 'fp32' else {}
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count

    def families(tt):
        fam = {}
        for i, (name, ms) in enumerate(tt):
            if name.startswith('sync.'):
                continue
            kind = plan.kernel.get(i) or name.split('.')[-1]
            f = fam.setdefault(kind, [0.0, 0.0, 0])
            f[0] += ms
            f[1] += plan.work[i][1] if i in plan.work else 0.0
            f[2] += 1
        return fam

    def conv_roofline(fam, dom, timing):
        t_ms, t_flop, t_n = fam[dom]
        t_tf = t_flop / (t_ms * 1e-3) / 1e12
        return {'bound': 'mfma', 'kernel': KERNEL_DESC[dom] + ', %d launches per forward; achieved = their '
                'algorithmic FLOPs / their summed event-timed durations)' % t_n,
                'achieved': round(t_tf, 2), 'peak': peak_t, 'unit': 'TFLOP/s', 'frac': round(t_tf / peak_t, 4),
                'traffic': traffic.get(dom, {}).get('bytes_per_launch'),
                'traffic_source': traffic.get(dom, {}).get('source'), 'timing': timing}

    def fam_rooflines(fam):
        return {k: {'achieved_tflops': round(w / (ms * 1e-3) / 1e12, 2), 'frac': round(w / (ms * 1e-3) / 1e12 / peak_t, 4),
                    'ms': round(ms, 4), 'launches': n, 'traffic': traffic.get(k, {}).get('bytes_per_launch')}
                for k, (ms, w, n) in fam.items() if is_conv(k) and ms > 0}

    roof = roof_chip = fam_roof = fam_roof_chip = hbm = conv_all = None
    conv_flop = None
    if times is not None:
        fam, fam_chip = families(times), families(times_chip)
        conv_flop = sum(w for kind, (ms, w, n) in fam.items() if is_conv(kind))
        # the dominant kernel family: the most device time per forward INSIDE the step
        dom = max((k for k in fam if is_conv(k)), key=lambda k: fam[k][0])
        roof = conv_roofline(fam, dom, 'in-step: each op of 5 eagerly issued forwards bracketed by HIP events on '
                             'the stream it runs on, lanes concurrent as in the step (lane-0 convs capped to %d of %d '
                             'CUs while PWC-Net runs on the side lane), the forward queued behind a spin kernel so no '
                             'host gap falls inside an op' % (plan.max_blocks_cap, ncu))
        dom_chip = max((k for k in fam_chip if is_conv(k)), key=lambda k: fam_chip[k][0])
        roof_chip = conv_roofline(fam_chip, dom_chip, 'whole chip: each op re-launched 10x alone between HIP events '
                                  'on the plan stream, uncapped')
        fam_roof, fam_roof_chip = fam_rooflines(fam), fam_rooflines(fam_chip)
        conv_ms = sum(ms for kind, (ms, w, n) in fam_chip.items() if is_conv(kind))
        conv_n = sum(n for kind, (ms, w, n) in fam_chip.items() if is_conv(kind))
        conv_all = {'achieved_tflops_whole_chip': round(conv_flop / (conv_ms * 1e-3) / 1e12, 2), 'launches': conv_n,
                    'step_frac': round(conv_flop / (ms_step * 1e-3) / 1e12 / peak_t, 4),
                    'ms_by_kernel_in_step': {k: round(v[0], 3) for k, v in fam.items() if is_conv(k)},
                    'ms_by_kernel_whole_chip': {k: round(v[0], 3) for k, v in fam_chip.items() if is_conv(k)}}
        hbm = {}
        # the fused conv kernels' algorithmic HBM bytes against 8 TB/s too (north_star: "achieved HBM GB/s on the
        # warp/fusion kernels"; the softmax fusion runs inside conv_fuse since round 5).  These are MFMA- or
        # issue-bound (their 'roofline_families' entry is the binding roof); this is their HBM side.
        hb = {}
        for i, by in plan.hbm.items():
            kind = plan.kernel.get(i)
            e = hb.setdefault(kind, [0.0, 0.0, 0.0, 0])
            e[0] += times_chip[i][1]
            e[1] += times[i][1]
            e[2] += by
            e[3] += 1
        for k, (ms, ms_in, by, n) in hb.items():
            gbs = by / (ms * 1e-3) / 1e9
            hbm[k] = {'bound': 'mfma' if k == 'conv_fuse' else 'issue', 'achieved': round(gbs, 1),
                      'peak': PEAK_HBM_GBS, 'unit': 'GB/s', 'frac': round(gbs / PEAK_HBM_GBS, 4),
                      'traffic': traffic.get(k, {}).get('bytes_per_launch'), 'us': round(ms * 1e3, 2),
                      'launches': n, 'alg_bytes': by / n,
                      'frac_in_step': round(by / (ms_in * 1e-3) / 1e9 / PEAK_HBM_GBS, 4), 'us_in_step': round(ms_in * 1e3, 2),
                      'note': 'algorithmic bytes per launch = ' + {
                          'conv_fuse': 'hidden input + the N frames\' features + fusion weights + fused output',
                          'resblock32': 'x in + y (or the fused head\'s fp32 RGB) out',
                          'resblock64': 'x in + y out',
                          'conv1x1_shuffle_blur': 'low-res input + blurred high-res output'}.get(k, '')}
        for k in ('warp', 'fuse'):
            if k in fam_chip:
                ms, by, n = fam_chip[k]
                gbs = by / (ms * 1e-3) / 1e9
                ms_in = fam[k][0]
                hbm[k] = {'bound': 'hbm', 'achieved': round(gbs, 1), 'peak': PEAK_HBM_GBS, 'unit': 'GB/s',
                          'frac': round(gbs / PEAK_HBM_GBS, 4), 'traffic': traffic.get(k, {}).get('bytes_per_launch'),
                          'us': round(ms * 1e3, 2), 'alg_bytes': by / n,
                          'frac_in_step': round(by / (ms_in * 1e-3) / 1e9 / PEAK_HBM_GBS, 4), 'us_in_step': round(ms_in * 1e3, 2)}
        if args.kernel_breakdown and rank == 0:
            for i, ((name, ms), (_, msc)) in enumerate(zip(times, times_chip)):
                if name.startswith('sync.'):
                    continue
                kind = plan.kernel.get(i) or '-'
                w = plan.work[i][1] if i in plan.work else 0.0
                rate = '%8.1f %s' % ((w / (msc * 1e-3) / 1e12, 'TF/s') if is_conv(kind) else
                                     (w / (msc * 1e-3) / 1e9, 'GB/s')) if (w and msc) else ''
                print(f'{name:32s} in-step {ms * 1e3:8.1f} us  chip {msc * 1e3:8.1f} us  {kind:15s} {rate}',
                      file=sys.stderr)
            for k, (ms, w, n) in sorted(fam.items(), key=lambda kv: -kv[1][0]):
                print(f'[family] {k:12s} in-step {ms * 1e3:9.1f} us  chip {fam_chip[k][0] * 1e3:9.1f} us  n={n}',
                      file=sys.stderr)
            print(f'sum of op times in-step {sum(t for _, t in times) * 1e3:.1f} us (lanes overlap), whole chip '
                  f'{sum(t for _, t in times_chip) * 1e3:.1f} us vs step {ms_step * 1e3:.1f} us', file=sys.stderr)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(N, S, S, args.cpu_seconds)

    if rank == 0:
        out = {
            'metric': 'bursts/sec 14x48x48 RAW->4x (SyntheticBurstVal shape), DBSR forward',
            'value': round(value, 2), 'unit': 'bursts/s', 'n_gpus': world, 'steps': args.steps,
            'warmup': args.warmup, 'ms_per_step': round(ms_step, 4), 'higher_is_better': True, 'scaling': 'weak',
            'vs_baseline': None, 'dtype': args.dtype, 'data': 'synthetic (seeded bursts, seeded random weights)',
            'config': {'workload': 'configs[1]: SyntheticBurstVal 14-frame 48x48 -> 384x384 (sr x8 of RAW, x4 of '
                                   'full-res), batch %d per GPU, full PWC-Net + warp + fusion + decoder' % B,
                       'global_batch': B * world, 'frames': N, 'height': S, 'width': S, 'out_size': S * 8,
                       'parallelism': 'dp%d (independent bursts per rank)' % world,
                       'hip_graph': not args.no_graph, 'fusion_weights_written': True},
            'roofline': roof, 'roofline_whole_chip': roof_chip, 'roofline_hbm': hbm,
            'roofline_families': fam_roof, 'roofline_families_whole_chip': fam_roof_chip,
            'conv_all': conv_all,
            'cpu_baseline': cpu,
            'conv_flop_per_step': conv_flop,
        }
        print(json.dumps(out))
    if dist:
        td.destroy_process_group()


if __name__ == '__main__':
    main()
