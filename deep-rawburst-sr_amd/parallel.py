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
    """Forward of this rank's shard of `bursts` (a global batch) and the gathered predictions.
    Every rank validates the batch before any collective, so a too-small batch fails on all ranks
    instead of leaving some of them blocked in the all-gather."""
    world = dist.get_world_size()
    if bursts.shape[0] < world:
        raise ValueError(f'global batch {bursts.shape[0]} < world size {world}: every rank needs >= 1 burst')
    local = shard(bursts)
    pred, _ = net(local)
    return gather_predictions(pred, bursts.shape[0])


# ---------------------------------------------------------------------------------------------------
# Frame sharding (BASELINE configs[4]): the frames of each burst split over ranks.
# Encoder, PWC-Net alignment and warp are per frame; every rank also holds the reference frame (the
# warp target and base_feat_proj, merging.py:80, need it).  The one coupling point is the softmax over
# the burst (merging.py:116-124): each rank reduces its own frames to (max, sum exp, sum exp*feat)
# statistics, one all-gather moves them (3*C*H*W fp32 per burst per rank -- instead of gathering the
# warped 512-channel features of every frame), and a log-sum-exp combine rebuilds the fused embedding.
# The decoder is split by rows: rank r decodes LR rows shard_range(H, r, R) plus the decoder's receptive-field
# halo (DBSREngine.decoder_halo: one LR row per LR 3x3 conv, the HR 3x3 convs in LR rows), which makes its rows of
# the prediction exactly the unsplit ones; one all-gather assembles the prediction.
# ---------------------------------------------------------------------------------------------------
def frame_shard(num_frames, rank, world):
    """Frame indices rank `rank` processes: [0] + its contiguous share of frames 1..N-1, and the first
    local index whose statistics it contributes (0 on rank 0, which owns the reference frame; 1 elsewhere,
    so frame 0 enters the softmax exactly once)."""
    if not 1 <= world <= num_frames - 1:
        raise ValueError(f'frame sharding needs 1 <= world ({world}) <= N-1 ({num_frames - 1})')
    a, b = shard_range(num_frames - 1, rank, world)
    return [0] + list(range(1 + a, 1 + b)), (0 if rank == 0 else 1)


def decoder_halo_rows(n_pre, n_post, s, blur=True):
    """LR rows of context a row slab of the decoder (decoders.py:54-62) needs for an exact prediction: one per
    LR 3x3 conv (init + 2 per pre-ResBlock), plus the HR 3x3 convs (blur + 2 per post-ResBlock) in LR rows."""
    n_lr = 1 + 2 * n_pre
    n_hr = 2 * n_post + (1 if blur else 0)
    return n_lr + (n_hr + s - 1) // s


def decoder_slab(lo, hi, total_rows, halo, align=16):
    """LR rows [y0, y1) a rank decodes for its rows [lo, hi): widened by `halo` on each side, then to a multiple
    of `align` rows where the image allows (the conv tiles' height; extra context leaves [lo, hi) exact).  Its
    convs dispatch as on the whole image (dbsr_conv_desc.plan_h), which every multiple of 16 rows can tile."""
    y0, y1 = max(0, lo - halo), min(total_rows, hi + halo)
    while (y1 - y0) % align and (y0 > 0 or y1 < total_rows):
        if y0 > 0:
            y0 -= 1
        else:
            y1 += 1
    return y0, y1


def gather_rows(slab, total_rows, rows_per_lr=1):
    """All-gather per-rank row slabs [B, C, r_i, W] (rank r holds LR rows shard_range(total_rows, r, R), i.e.
    rows_per_lr times as many prediction rows) into [B, C, rows_per_lr * total_rows, W] in rank order."""
    world = dist.get_world_size()
    sizes = [(b - a) * rows_per_lr for a, b in (shard_range(total_rows, r, world) for r in range(world))]
    mx = max(sizes)
    pad = slab.new_zeros(slab.shape[:2] + (mx,) + slab.shape[3:])
    pad[:, :, :slab.shape[2]] = slab
    bufs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(bufs, pad.contiguous())
    return torch.cat([bf[:, :, :n] for bf, n in zip(bufs, sizes)], dim=2)


def frame_sharded_forward(net, burst, partial_fn=None, combine_fn=None, gathered_fn=None, split_decoder=True):
    """pred [B,3,sH,sW] of `burst` [B,N,4,H,W] (same on every rank) with its frames sharded over the
    process group.  partial_fn(local_burst, first) -> stats and combine_fn(gathered [R,...], rows) -> pred rows
    default to the HIP engine (DBSREngine.forward_partial / combine_decode); gathered_fn(R, stats, rows) gives
    the all-gather destination (the engine's combine input buffer, so the collective writes in place).
    split_decoder: each rank decodes its LR rows shard_range(H, rank, R) (+ halo) and one all-gather assembles
    the prediction; False: every rank decodes the whole image."""
    rank, world = dist.get_rank(), dist.get_world_size()
    frames, first = frame_shard(burst.shape[1], rank, world)
    local = burst[:, frames]
    if partial_fn is None:
        eng = net._get_engine()
        partial_fn = lambda x, f: eng.forward_partial(x, f)[0]                          # noqa: E731
        combine_fn = eng.combine_decode
        gathered_fn = lambda R, st, rows: eng.gathered_buffer(R, *st.shape[:3], rows)  # noqa: E731
    H = burst.shape[-2]
    rows = shard_range(H, rank, world) if split_decoder else None
    stats = partial_fn(local, first)
    gathered = gathered_fn(world, stats, rows) if gathered_fn is not None else \
        stats.new_empty((world,) + tuple(stats.shape))
    # concatenated along dim 0 ([R*B,...] view of the [R,B,...] buffer): the layout gloo and RCCL both take
    dist.all_gather_into_tensor(gathered.view((-1,) + tuple(stats.shape[1:])), stats.contiguous())
    if not split_decoder:
        return combine_fn(gathered)
    slab = combine_fn(gathered, rows)
    return gather_rows(slab, H, slab.shape[3] // burst.shape[-1])
