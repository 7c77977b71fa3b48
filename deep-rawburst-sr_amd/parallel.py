"""Multi-GPU execution of the DBSR forward: one process per GPU, bursts sharded over ranks.

Bursts are independent, so inference partitions as an embarrassingly parallel batch split with no
data-path collective.  The reference's only multi-GPU mechanism is single-process
nn.DataParallel (admin/multigpu.py:8-14: scatter on dim 0, replicate, gather to GPU 0); here each rank
holds a full weight replica and runs its own shard; the optional gather of predictions is one
all_gather (RCCL over xGMI on GPUs, gloo in the CPU tests).
"""
import torch
import torch.distributed as dist


def shard_range(global_batch, rank, world):
    """[start, stop) of the bursts rank `rank` owns; shards differ by at most one burst."""
    base, rem = divmod(global_batch, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def shard(bursts, rank=None, world=None):
    rank = dist.get_rank() if rank is None else rank
    world = dist.get_world_size() if world is None else world
    a, b = shard_range(bursts.shape[0], rank, world)
    return bursts[a:b]


def max_over_ranks(seconds, device=None):
    """Slowest rank's elapsed time (the whole job is done when the slowest rank is)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(seconds)
    t = torch.tensor([float(seconds)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_predictions(pred_local, global_batch):
    """All-gather per-rank predictions [b_r, ...] into [global_batch, ...] in rank order."""
    world = dist.get_world_size()
    sizes = [shard_range(global_batch, r, world) for r in range(world)]
    maxb = max(b - a for a, b in sizes)
    padded = pred_local.new_zeros((maxb,) + tuple(pred_local.shape[1:]))
    padded[:pred_local.shape[0]] = pred_local
    bufs = [torch.empty_like(padded) for _ in range(world)]
    dist.all_gather(bufs, padded)
    return torch.cat([buf[:b - a] for buf, (a, b) in zip(bufs, sizes)], dim=0)


def run_sharded(net, bursts):
    """Forward of this rank's shard of `bursts` (a global batch) and the gathered predictions."""
    local = shard(bursts)
    pred, _ = net(local)
    return gather_predictions(pred, bursts.shape[0])
