"""World-size-2 gloo tests (CPU) of the multi-GPU path's host logic: burst sharding, the
max-over-ranks timing reduction and the prediction gather used by bench.py / parallel.run_sharded."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from dbsr_amd.parallel import shard_range


def test_shard_range_covers_batch():
    for gb in [1, 7, 8, 13, 64]:
        for world in [1, 2, 3, 8]:
            ranges = [shard_range(gb, r, world) for r in range(world)]
            assert ranges[0][0] == 0 and ranges[-1][1] == gb
            assert all(ranges[i][1] == ranges[i + 1][0] for i in range(world - 1))
            sizes = [b - a for a, b in ranges]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    from dbsr_amd import parallel
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        gb = 5
        bursts = torch.arange(gb * 2 * 4 * 3 * 3, dtype=torch.float32).view(gb, 2, 4, 3, 3)
        local = parallel.shard(bursts)

        class FakeNet:                       # stands in for the HIP forward (needs a GPU)
            def __call__(self, b):
                return b.sum(dim=(1, 2)) * 2.0, {}
        full = parallel.run_sharded(FakeNet(), bursts)
        t = parallel.max_over_ranks(0.5 + rank)
        q.put((rank, local.shape[0], torch.equal(full, bursts.sum(dim=(1, 2)) * 2.0), t))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_shard_gather_and_timing():
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert [r[1] for r in res] == [3, 2]          # 5 bursts over 2 ranks
    assert all(r[2] for r in res)                  # gathered predictions == single-process result
    assert all(abs(r[3] - 1.5) < 1e-12 for r in res)   # max over ranks


def test_frame_shard_assignment():
    from dbsr_amd.parallel import frame_shard
    for N in [2, 4, 14]:
        for world in range(1, N):
            seen = []
            for r in range(world):
                frames, first = frame_shard(N, r, world)
                assert frames[0] == 0 and len(frames) >= 2
                assert first == (0 if r == 0 else 1)
                seen += frames[first:]
            assert sorted(seen) == list(range(N))      # every frame enters the softmax exactly once
    with pytest.raises(ValueError):
        frame_shard(4, 0, 4)


def _frame_worker(rank, world, port, q):
    """Frame-sharded forward over gloo with the oracle standing in for the HIP kernels (the product's
    kernels are checked against the same restatement on the GPU, tests/test_gpu_e2e.py)."""
    import torch.distributed as dist
    from dbsr_amd import parallel
    from dbsr_amd.burst import synthetic_bursts
    from dbsr_amd.weights import generate_state_dict
    import dbsr_amd
    from dbsr_amd import arch
    from oracle import dbsr_oracle as orc
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        torch.set_num_threads(2)
        net = dbsr_amd.dbsrnet_cvpr2021(**dbsr_amd.DBSR_SYNTHETIC_KWARGS)
        sd = orc.state_dict_to_torch(generate_state_dict(arch.state_dict_shapes(net), seed=0))
        kw = orc.DBSR_SYNTHETIC_KWARGS
        burst, _ = synthetic_bursts(1, 4, 48, 24, sr_factor=8, seed=4)
        halo = parallel.decoder_halo_rows(kw['dec_num_pre_res_blocks'], kw['dec_num_post_res_blocks'],
                                          kw['upsample_factor'], kw.get('gauss_blur_sd') is not None)
        assert halo == 13

        def partial_fn(local, first):
            all_feat, logits = orc.merging(orc.encoder(local, sd, kw), sd, kw, return_logits=True)
            return orc.fuse_partial_stats(all_feat, logits, first)

        def combine_fn(gathered, rows=None):
            fused = orc.fuse_combine(gathered)
            if rows is None:
                return orc.decoder({'fused_enc': fused}, sd, kw)
            # the decoder on this rank's LR rows + halo (zero padding at the slab edges), valid rows kept
            lo, hi = rows
            y0, y1 = max(0, lo - halo), min(fused.shape[2], hi + halo)
            s = kw['upsample_factor']
            return orc.decoder({'fused_enc': fused[:, :, y0:y1].contiguous()}, sd, kw)[:, :, (lo - y0) * s:(hi - y0) * s]
        pred = parallel.frame_sharded_forward(None, burst, partial_fn, combine_fn)
        if rank == 0:
            ref, _ = orc.dbsr_forward(burst, sd)
            q.put((rank, float((pred - ref).abs().max())))
        else:
            q.put((rank, 0.0))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_frame_sharded_fusion():
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_frame_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res[0][1] <= 1e-4, res            # sharded == unsharded forward (fp32, rounding order only)


def _ddp_worker(rank, world, port, q):
    """Data-parallel training gradient (configs[3]): each rank differentiates the oracle forward on its
    shard of the global batch (stand-in for the HIP step, which needs a GPU), flattens the gradients in
    the trainer's layout and averages them with the trainer's bucketed all-reduce."""
    import torch.distributed as dist
    import torch.nn.functional as F
    import dbsr_amd
    from dbsr_amd import parallel, training
    from dbsr_amd.burst import synthetic_bursts
    from oracle import dbsr_oracle as orc
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        torch.set_num_threads(2)
        net = dbsr_amd.build_synthetic_net(seed=0)
        layout, buckets = training.flat_layout(net)
        sd0 = {k: v.detach().clone() for k, v in net.state_dict().items()}
        burst, gt = synthetic_bursts(4, 3, 16, 16, sr_factor=8, seed=5)

        def grads(b, g):
            sd = {k: v.clone().requires_grad_(not k.startswith('encoder.alignment_net')) for k, v in sd0.items()}
            pred, _ = orc.dbsr_forward(b, sd)
            F.l1_loss(pred[..., 40:-40, 40:-40], g[..., 40:-40, 40:-40]).backward()
            return torch.cat([sd[n].grad.reshape(-1) for n, _ in layout])

        a, b = parallel.shard_range(burst.shape[0], rank, world)
        flat = grads(burst[a:b], gt[a:b])
        works = [training.allreduce_bucket(flat, lo, hi) for lo, hi in buckets]
        for w in works:
            w.wait()
        flat /= world
        full = grads(burst, gt)
        q.put((rank, float((flat - full).abs().max() / full.abs().max()), buckets[-1][1] == flat.numel()))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_ddp_gradients_equal_single_process():
    """the all-reduced sharded gradients equal a single-process step on the
    concatenated batch (L1 mean over equal shards; fp32 summation-order tolerance)."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ddp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for rank, err, covers in res:
        assert covers                      # the three buckets cover every trainable parameter
        assert err <= 1e-5, (rank, err)


def test_bench_launcher_spawns_ranks_gloo():
    """bench.py --gpus N outside torchrun starts N rank processes itself (before any GPU call) and every rank
    derives the same tiling of the global batch (admin/multigpu.py:8-14 is the reference's
    single-process DataParallel).  --dry-run swaps the GPU work for a gloo all-gather of the shards."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK')}
    for n in (2, 3):
        out = subprocess.run([sys.executable, os.path.join(repo, 'bench.py'), '--gpus', str(n), '--batch', '8',
                              '--dry-run'], capture_output=True, text=True, timeout=240, env=env, cwd=repo)
        assert out.returncode == 0, out.stderr[-2000:]
        line = [ln for ln in out.stdout.splitlines() if ln.startswith('{')][-1]
        res = json.loads(line)
        assert res['n_gpus'] == n and res['global_batch'] == 8 * n
        ranks = sorted(res['ranks'])
        assert [r[0] for r in ranks] == list(range(n)) and all(r[1] == n for r in ranks)
        assert ranks[0][2] == 0 and ranks[-1][3] == 8 * n
        assert all(a[3] == b[2] for a, b in zip(ranks, ranks[1:]))       # contiguous, no overlap
        assert all(r[3] - r[2] == 8 for r in ranks)                      # weak scaling: --batch per rank


def test_bench_rejects_gpus_world_mismatch():
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE='1', RANK='0', LOCAL_RANK='0')
    out = subprocess.run([sys.executable, os.path.join(repo, 'bench.py'), '--gpus', '2', '--dry-run'],
                         capture_output=True, text=True, timeout=120, env=env, cwd=repo)
    assert out.returncode != 0 and 'one rank per GPU' in out.stderr


def test_dbsrnet_training_mode_dispatch():
    """net.train() with autograd routes DBSRNet.forward to the HIP training path (saved activations + HIP
    backward); eval / no_grad / frozen DBSR parameters route it to the inference engine (CPU check of the
    dispatch only)."""
    import dbsr_amd
    net = dbsr_amd.dbsrnet_cvpr2021(**dbsr_amd.DBSR_SYNTHETIC_KWARGS)
    assert net.train()._trains()
    with torch.no_grad():
        assert not net._trains()
    assert not net.eval()._trains()
    net.train()
    for n, p in net.named_parameters():
        if not n.startswith('encoder.alignment_net'):
            p.requires_grad_(False)
    assert not net._trains()
