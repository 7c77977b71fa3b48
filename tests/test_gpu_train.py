"""Training step (BASELINE configs[3]) on the HIP kernels: op-level backward parity against torch autograd
of the same ops, and whole-step gradients / Adam update against torch autograd of the oracle forward
(the reference's training step: L1(pred, gt, boundary_ignore=40).backward(), Adam(lr=1e-4);
trainers/simple_trainer.py:78-81, actors/dbsr_actors.py:27-47, default_synthetic.py:85-96).

Tolerances: fp32 kernels vs torch fp32 -- 1e-4 relative to the gradient's max magnitude (different
summation orders over up to 10^5 pixels); bf16 kernels vs torch on the same bf16-rounded operands --
2e-2 relative.  Whole network: the gradients of the early weight-predictor / offset-feature layers
sit behind ReLU gates that flip on rounding-level forward differences (the oracle's own fp32 vs fp64
gradients differ by 6.5e-4 of the max at weight_predictor.1.conv2), so fp32 is held to the loss within
1e-5, per-tensor cosine similarity >= 1 - 1e-4 and max-rel <= 2e-2; bf16 to the loss within 1 % and
cosine similarity >= 0.97 per tensor."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = 'cuda'


@pytest.fixture(scope='module')
def ops():
    from dbsr_amd import ops as O
    return O


def _rel(a, b):
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-12))


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('case', [(2, 64, 20, 36, 64, 3), (1, 4, 9, 17, 64, 3), (2, 512, 8, 16, 64, 1),
                                  (1, 32, 24, 40, 3, 1), (1, 128, 12, 12, 512, 3), (2, 192, 16, 16, 128, 3),
                                  (3, 32, 20, 36, 32, 3), (1, 32, 33, 47, 3, 3), (2, 24, 16, 40, 32, 1)])
def test_conv_wgrad(ops, dtype, case):
    # (the last three run the 32-channel-block variant with two tiles prefetched)
    N, Cin, H, W, Cout, k = case
    gen = torch.Generator().manual_seed(Cin + Cout * 3 + H)
    x = torch.randn(N, Cin, H, W, generator=gen)
    dy = torch.randn(N, Cout, H, W, generator=gen)
    xr, dyr = x.to(dtype).float(), dy.to(dtype).float()
    w = torch.zeros(Cout, Cin, k, k, requires_grad=True)
    F.conv2d(xr, w, padding=k // 2).backward(dyr)
    out = ops.conv2d_wgrad(x.to(DEV), dy.to(DEV), k, compute_dtype=dtype).cpu()
    assert _rel(out, w.grad) <= 1e-4
    # the bias gradient from the same pass (dbsr_conv_wgrad_bias): the weight gradient is bitwise the same
    ow, ob = ops.conv2d_wgrad(x.to(DEV), dy.to(DEV), k, compute_dtype=dtype, with_bias=True)
    assert torch.equal(ow.cpu(), out)
    if dtype != torch.float32:
        # the register-staged kernel (dbsr_set_wgrad_algo(0)) sums in the same order as the LDS-DMA ring kernel
        from dbsr_amd import _lib as L
        L.lib().dbsr_set_wgrad_algo(0)
        try:
            ow0, ob0 = ops.conv2d_wgrad(x.to(DEV), dy.to(DEV), k, compute_dtype=dtype, with_bias=True)
        finally:
            L.lib().dbsr_set_wgrad_algo(1)
        assert torch.equal(ow0.cpu(), out)
        assert float((ob0.cpu() - ob.cpu()).abs().max()) <= 1e-5 * float(dyr.abs().sum((0, 2, 3)).max())
    db = dyr.sum((0, 2, 3))
    # fp32 sums of the same (rounded) values in another order: 1e-5 of the channel's absolute sum
    assert float((ob.cpu() - db).abs().max()) <= 1e-5 * float(dyr.abs().sum((0, 2, 3)).max())


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('case', [(2, 64, 20, 36, 64, 3), (1, 64, 12, 16, 4, 3), (2, 64, 8, 16, 512, 1),
                                  (1, 3, 24, 40, 32, 1), (1, 512, 12, 12, 64, 3)])
def test_conv_dgrad_gate_residual(ops, dtype, case):
    """dX of a conv (dgrad-packed weights on the forward kernel) + residual, gated by a ReLU output."""
    N, Cout, H, W, Cin, k = case
    gen = torch.Generator().manual_seed(Cin * 5 + Cout + W)
    dy = torch.randn(N, Cout, H, W, generator=gen)
    w = torch.randn(Cout, Cin, k, k, generator=gen) / (Cin * k * k) ** 0.5
    res = torch.randn(N, Cin, H, W, generator=gen)
    gate = F.relu(torch.randn(N, Cin, H, W, generator=gen))
    dyr, wr, rr = (t.to(dtype).float() for t in (dy, w, res))
    x = torch.zeros(N, Cin, H, W, requires_grad=True)
    F.conv2d(x, wr, padding=k // 2).backward(dyr)
    ref = (x.grad + rr) * (gate > 0)
    out = ops.conv2d_dgrad(dy.to(DEV), w.to(DEV), residual=res.to(DEV), gate=gate.to(DEV),
                           compute_dtype=dtype).float().cpu()
    tol = 1e-4 if dtype == torch.float32 else 2e-2
    assert _rel(out, ref) <= tol


# (N, Cout, H, W, Cin, expected kernel): the gated (training dgrad) epilogues of the fast kernels -- weight-
# stationary EPI 5 on 16x8 tiles (12 frames of 48x48) and 16x16 tiles (40 frames of 32x16, 96 dgrad couts: a
# partial cout tile), the pipelined kernel's run-time epilogue (48 frames of 48x48, 128 -> 64 channels) and its
# epilogue 5 at the 32x16 tile (64 frames of 32x32, 96 dgrad couts: a partial cout tile), and the K-split 128-channel
# kernel's epilogue 5 (64 frames of 32x32, 128 -> 128: the training step's weight-predictor ResBlock dgrads)
GATED = [(12, 64, 48, 48, 64, 4), (40, 64, 32, 16, 96, 4), (48, 128, 48, 48, 64, 2), (64, 128, 32, 32, 128, 7),
         (64, 128, 32, 32, 96, 2)]


@pytest.mark.parametrize('case', GATED)
def test_conv_dgrad_gated_fast_kernels(ops, case):
    """the gated epilogues the training step runs at 48x48 / 128x128 against autograd, with the
    kernel asserted (dbsr_conv_kernel_for), with and without the ResBlock residual."""
    N, Cout, H, W, Cin, kern = case
    dtype = torch.bfloat16
    gen = torch.Generator().manual_seed(Cin * 7 + Cout + W)
    dy = torch.randn(N, Cout, H, W, generator=gen)
    w = torch.randn(Cout, Cin, 3, 3, generator=gen) / (Cin * 9) ** 0.5
    res = torch.randn(N, Cin, H, W, generator=gen)
    gate = F.relu(torch.randn(N, Cin, H, W, generator=gen))
    dyr, wr, rr = (t.to(dtype).float() for t in (dy, w, res))
    x = torch.zeros(N, Cin, H, W, requires_grad=True)
    F.conv2d(x, wr, padding=1).backward(dyr)
    for use_res in (True, False):
        ref = ((x.grad + rr) if use_res else x.grad) * (gate > 0)
        out = ops.conv2d_dgrad(dy.to(DEV), w.to(DEV), residual=res.to(DEV) if use_res else None, gate=gate.to(DEV),
                               compute_dtype=dtype).float().cpu()
        assert ops.conv2d_dgrad.last_kernel == kern, (case, ops.conv2d_dgrad.last_kernel)
        assert _rel(out, ref) <= 2e-2
        assert bool(((out != 0) <= (gate > 0)).all())           # gated-off outputs are exactly zero


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_fuse_backward(ops, dtype):
    gen = torch.Generator().manual_seed(3)
    B, N, C, H, W = 2, 5, 64, 6, 7
    lg = torch.randn(B, N, C, H, W, generator=gen)
    f = torch.randn(B, N, C, H, W, generator=gen)
    df = torch.randn(B, C, H, W, generator=gen)
    lgr, fr = lg.to(dtype).float().requires_grad_(), f.to(dtype).float().requires_grad_()
    w = F.softmax(lgr, dim=1)
    fused = (fr * w).sum(dim=1)
    fused.backward(df.to(dtype).float())
    dl, dfe = ops.fuse_backward(w.detach().to(DEV).to(dtype), f.to(DEV).to(dtype), fused.detach().to(DEV).to(dtype),
                                df.to(DEV).to(dtype))
    tol = 1e-5 if dtype == torch.float32 else 3e-2
    assert _rel(dl.float().cpu(), lgr.grad) <= tol
    assert _rel(dfe.float().cpu(), fr.grad) <= tol


def test_warp_backward(ops):
    from oracle import dbsr_oracle as orc
    gen = torch.Generator().manual_seed(4)
    x = torch.randn(3, 16, 12, 20, generator=gen, requires_grad=True)
    fl = torch.randn(3, 2, 12, 20, generator=gen) * 3.0
    dy = torch.randn(3, 16, 12, 20, generator=gen)
    orc.warp(x, fl).backward(dy)
    out = ops.warp_backward(dy.to(DEV), fl.to(DEV)).cpu()
    assert _rel(out, x.grad) <= 1e-5


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('case', [(2, 3, 40, 56), (3, 32, 64, 64), (2, 64, 17, 23), (1, 512, 12, 20), (1, 72, 9, 9)])
def test_chan_sum(ops, dtype, case):
    """Bias gradient (per-channel sum): the 16-B kernel (16-bit, any c) and the element kernel (fp32)."""
    N, C, H, W = case
    t = torch.randn(N, C, H, W, generator=torch.Generator().manual_seed(C + H)).to(dtype)
    out = ops.chan_sum(t.to(DEV)).cpu()
    ref = t.double().sum(dim=(0, 2, 3))
    assert float((out.double() - ref).abs().max()) <= 1e-4 * float(t.double().abs().sum(dim=(0, 2, 3)).max())


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('case', [(2, 40, 56, 3), (1, 33, 47, 3), (3, 16, 16, 1), (1, 64, 64, 4)])
def test_head_forward_backward(dtype, case):
    """The training step's predictor (dbsr_head_forward / dbsr_head_backward; decoders.py:61, 1x1 conv 32 -> hc +
    ReLU) against torch on the same rounded operands: pred, the gated dgrad, dW and db."""
    from dbsr_amd import _lib as L
    from dbsr_amd.ops import _nhwc
    N, H, W, hc = case
    gen = torch.Generator().manual_seed(H * 7 + hc)
    h = torch.randn(N, 32, H, W, generator=gen).to(dtype).float()        # negative entries: the ReLU gate
    w = torch.randn(hc, 32, 1, 1, generator=gen) * 0.2
    b = torch.randn(hc, generator=gen) * 0.1
    dp = torch.randn(N, hc, H, W, generator=gen).to(dtype).float()
    lib, s = L.lib(), L.stream_ptr(torch.device(DEV))
    hs, ldh = _nhwc(h.to(DEV), dtype)
    wd, bd = w.to(DEV).contiguous(), b.to(DEV).contiguous()
    out = torch.zeros(N, hc, H, W, device=DEV)
    L.check(lib.dbsr_head_forward(N, H * W, L.tensor_desc(hs, ldh), 32, wd.data_ptr(), bd.data_ptr(), hc,
                                  out.data_ptr(), s), 'head_forward')
    ref = F.relu(F.conv2d(h, w, b))
    assert float((out.cpu() - ref).abs().max()) <= 1e-4 * float(ref.abs().max())
    dps = torch.zeros(N, H, W, 8, dtype=dtype, device=DEV)
    dps[..., :hc] = dp.permute(0, 2, 3, 1).to(DEV).to(dtype)
    dh = torch.zeros(N, H, W, 32, dtype=dtype, device=DEV)
    dw = torch.zeros(hc, 32, device=DEV)
    db = torch.zeros(hc, device=DEV)
    need = lib.dbsr_head_backward_workspace_bytes(N, H * W, 32, hc)
    wsb = torch.empty(need // 4 + 1, device=DEV)
    L.check(lib.dbsr_head_backward(N, H * W, L.tensor_desc(hs, ldh), 32, L.tensor_desc(dps, 8), wd.data_ptr(), hc,
                                   L.tensor_desc(dh, 32), dw.data_ptr(), db.data_ptr(), 0, wsb.data_ptr(), need, s),
            'head_backward')
    hh = h.clone().requires_grad_(True)
    ww = w.clone().requires_grad_(True)
    bb = b.clone().requires_grad_(True)
    F.conv2d(hh, ww, bb).backward(dp)
    gh = hh.grad * (h > 0)
    got = dh.float().cpu().permute(0, 3, 1, 2)
    tol = 1e-4 if dtype == torch.float32 else 1e-2                  # dh is stored in the compute dtype
    assert float((got - gh).abs().max()) <= tol * float(gh.abs().max())
    assert _rel(dw.cpu(), ww.grad.reshape(hc, 32)) <= 1e-4
    assert float((db.cpu() - bb.grad).abs().max()) <= 1e-5 * float(dp.abs().sum((0, 2, 3)).max())


@pytest.mark.parametrize('case', [(3, 16, 12, 20, 3.0, torch.float32, False),     # random flow: list flushes
                                  (2, 64, 40, 56, 20.0, torch.float32, True),     # far taps, window = frame
                                  (2, 72, 33, 47, 0.7, torch.float32, True),      # ragged tiles, C % 64 != 0
                                  (2, 64, 32, 48, 2.0, torch.bfloat16, True)])
def test_warp_backward_gather(ops, case):
    """The owner-computes gather (no atomics) against autograd through the oracle's grid_sample warp,
    with the encoder-ReLU gate of the training step."""
    from oracle import dbsr_oracle as orc
    N, C, H, W, scale, dtype, gated = case
    gen = torch.Generator().manual_seed(C + H)
    x = torch.randn(N, C, H, W, generator=gen, requires_grad=True)
    fl = torch.randn(N, 2, H, W, generator=gen) * scale
    dy = torch.randn(N, C, H, W, generator=gen).to(dtype).float()
    gate = F.relu(torch.randn(N, C, H, W, generator=gen)).to(dtype) if gated else None
    orc.warp(x, fl).backward(dy)
    ref = x.grad * (gate.float() > 0) if gated else x.grad
    out = ops.warp_backward_gather(dy.to(DEV).to(dtype), fl.to(DEV), gate.to(DEV) if gated else None).float().cpu()
    tol = 1e-5 if dtype == torch.float32 else 8e-3
    assert _rel(out, ref) <= tol


@pytest.mark.parametrize('converge', [False, True])
def test_warp_backward_gather_deterministic(ops, converge):
    """the gather sums each pixel's contributions in source-pixel order, so repeated runs are bitwise
    equal -- also when flows converge (hundreds of contributions per pixel: the > 64 wave-minimum path)."""
    from oracle import dbsr_oracle as orc
    N, C, H, W = 2, 64, 32, 48
    gen = torch.Generator().manual_seed(11)
    if converge:
        yy, xx = torch.meshgrid(torch.arange(H, dtype=torch.float32), torch.arange(W, dtype=torch.float32),
                                indexing='ij')
        fl = torch.stack([(W / 2 - xx) * 0.97, (H / 2 - yy) * 0.97])[None].repeat(N, 1, 1, 1)
        fl = fl + 0.3 * torch.randn(N, 2, H, W, generator=gen)
    else:
        fl = torch.randn(N, 2, H, W, generator=gen) * 3.0
    x = torch.randn(N, C, H, W, generator=gen, requires_grad=True)
    dy = torch.randn(N, C, H, W, generator=gen)
    orc.warp(x, fl).backward(dy)
    outs = [ops.warp_backward_gather(dy.to(DEV), fl.to(DEV), None).cpu() for _ in range(3)]
    assert all(torch.equal(outs[0], o) for o in outs[1:])
    assert _rel(outs[0], x.grad) <= 1e-5


# ----------------------------------------------------------------------------------------------------
# whole training step
# ----------------------------------------------------------------------------------------------------
def _oracle_grads(sd_t, burst, gt, bi):
    from oracle import dbsr_oracle as orc
    sd = {k: v.clone().requires_grad_(not k.startswith('encoder.alignment_net')) for k, v in sd_t.items()}
    pred, _ = orc.dbsr_forward(burst, sd)
    loss = F.l1_loss(pred[..., bi:-bi, bi:-bi], gt[..., bi:-bi, bi:-bi])
    loss.backward()
    return float(loss), {k: v.grad for k, v in sd.items() if v.grad is not None}


def _trainer(synth_sd, dtype):
    import dbsr_amd
    from dbsr_amd.training import DBSRTrainer
    net = dbsr_amd.dbsrnet_cvpr2021(**dbsr_amd.DBSR_SYNTHETIC_KWARGS)
    net.load_state_dict(synth_sd)
    net = net.to(DEV).set_compute_dtype(dtype)
    return net, DBSRTrainer(net, boundary_ignore=40)


@pytest.mark.parametrize('shape', [(2, 3, 24, 32), (1, 3, 48, 48), (1, 14, 128, 128)])
@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_train_step_grads_vs_oracle(synth_sd, dtype, shape):
    """Whole-step gradients against autograd through the oracle: a small ragged shape, 48x48 (the gated
    weight-stationary dgrads on 16-row tiles) and configs[3]'s 14 x 128x128 frames at batch 1 (VERDICT r3 #4:
    the 128-wide pipelined tile, the gated ws dgrads and the 128^2 warp-gather backward)."""
    from dbsr_amd import _lib as L
    from dbsr_amd.burst import synthetic_bursts
    B, N, H, W = shape
    burst, gt = synthetic_bursts(B, N, H, W, sr_factor=8, seed=17)
    ref_loss, ref_g = _oracle_grads(synth_sd, burst, gt, 40)
    net, tr = _trainer(synth_sd, dtype)
    loss, _ = tr.forward_backward(burst.to(DEV), gt.to(DEV))
    torch.cuda.synchronize()
    if dtype == torch.bfloat16 and H >= 48:
        gated = {L.lib().dbsr_conv_kernel_for(d) for d, _ in tr.plans[(B, N, H, W)].convs if d.gate.ptr}
        assert 4 in gated, gated                              # the gated weight-stationary dgrad ran
    mine = {k: v.cpu() for k, v in tr.grads().items()}
    assert set(mine) == set(ref_g), set(mine) ^ set(ref_g)
    print('loss', float(loss), ref_loss)
    gmax = max(float(g.abs().max()) for g in ref_g.values())
    rel, cos = [], []
    for k, g in ref_g.items():
        if k == 'merging.weight_predictor.4.0.bias':
            # the last logit conv's bias is shared by all N frames of the softmax: its exact gradient is 0
            # (softmax shift invariance, merging.py:117); both sides are rounding noise
            assert float(mine[k].abs().max()) <= 1e-4 * gmax
            continue
        rel.append((_rel(mine[k], g), k))
        cos.append((1 - float(F.cosine_similarity(mine[k].double().flatten(), g.double().flatten(), dim=0)), k))
    rel.sort(reverse=True)
    cos.sort(reverse=True)
    print('max-rel worst', rel[:4])
    print('1-cos worst', cos[:4])
    if dtype == torch.float32:
        assert abs(float(loss) - ref_loss) <= 1e-5 * max(1.0, abs(ref_loss))
        assert rel[0][0] <= 2e-2, rel[:3]
        assert cos[0][0] <= 1e-4, cos[:3]
    else:
        assert abs(float(loss) - ref_loss) <= 1e-2 * abs(ref_loss)
        assert cos[0][0] <= 3e-2, cos[:3]


def test_train_step_adam_update_fp32(synth_sd):
    """One step updates the parameters exactly as torch.optim.Adam(lr=1e-4) does with that step's
    gradients (the gradients themselves are checked against the oracle above)."""
    from dbsr_amd.burst import synthetic_bursts
    burst, gt = synthetic_bursts(1, 3, 24, 32, sr_factor=8, seed=18)
    net, tr = _trainer(synth_sd, torch.float32)
    before = {k: v.detach().clone() for k, v in net.named_parameters() if not k.startswith('encoder.alignment_net')}
    tr.step(burst.to(DEV), gt.to(DEV))
    torch.cuda.synchronize()
    grads = tr.grads()
    params = {k: before[k].clone().requires_grad_() for k in before}
    opt = torch.optim.Adam(list(params.values()), lr=1e-4)
    for k, p in params.items():
        p.grad = grads[k].clone()
    opt.step()
    cur = dict(net.named_parameters())
    for k, p in params.items():
        np.testing.assert_allclose(cur[k].detach().cpu().numpy(), p.detach().cpu().numpy(), rtol=1e-6, atol=1e-7)


def test_train_step_graph_replay_equals_eager(synth_sd):
    """DBSRTrainer.step replays HIP graphs of its segments from the second step on; three steps with
    graphs equal three eager steps (losses and parameters, fp32) from the same initialisation."""
    from dbsr_amd.burst import synthetic_bursts
    burst, gt = synthetic_bursts(1, 3, 24, 32, sr_factor=8, seed=23)
    b, g = burst.to(DEV), gt.to(DEV)
    res = {}
    for use_graph in (True, False):
        net, tr = _trainer(synth_sd, torch.float32)
        tr.use_graph = use_graph
        losses = [float(tr.step(b, g)) for _ in range(3)]
        torch.cuda.synchronize()
        assert (tr.plans[(1, 3, 24, 32)].graphs is not None) == use_graph
        res[use_graph] = (losses, tr.flat.detach().clone())
    assert res[True][0] == pytest.approx(res[False][0], rel=1e-6, abs=1e-7)
    torch.testing.assert_close(res[True][1], res[False][1], rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float32])
def test_batched_repack_bitwise(synth_sd, dtype, monkeypatch):
    """dbsr_conv_pack_weights_batch (one launch for every conv's forward and dgrad weights, ABI 22) packs bitwise
    what the per-conv dbsr_conv_pack_weights / dbsr_dgrad_weights / dbsr_conv_pack_weights launches pack: every
    packed buffer (incl. the pipe copies, the shuffled upsampler and the weight predictor's sliced dgrad copies)
    after two steps, and the steps' losses and parameters."""
    from dbsr_amd.burst import synthetic_bursts
    from dbsr_amd.training import DBSRTrainer
    burst, gt = synthetic_bursts(1, 3, 24, 32, sr_factor=8, seed=29)
    b, g = burst.to(DEV), gt.to(DEV)
    res = {}
    for batched in (False, True):
        monkeypatch.setattr(DBSRTrainer, 'BATCH_REPACK', batched)
        net, tr = _trainer(synth_sd, dtype)
        for tc in tr.tconvs:        # (fp32 packs leave the pipe-copy half of the buffer unwritten)
            for p in [tc.fwd, tc.bwd] + getattr(tc, 'extra', []):
                p.w.zero_()
        losses = [float(tr.step(b, g)) for _ in range(2)]
        torch.cuda.synchronize()
        names = [o[2] for o in tr.plans[(1, 3, 24, 32)].ops]
        assert ('repack.all' in names) == batched and (any(n.startswith('packT.') for n in names) != batched)
        bufs = []
        for tc in tr.tconvs:
            for p in [tc.fwd, tc.bwd] + getattr(tc, 'extra', []):
                bufs.append(p.w.detach().clone())
                if p.bias is not None:
                    bufs.append(p.bias.detach().clone())
        res[batched] = (losses, tr.flat.detach().clone(), bufs)
    assert res[True][0] == res[False][0]
    assert torch.equal(res[True][1], res[False][1])
    assert len(res[True][2]) == len(res[False][2])
    for a, c in zip(res[True][2], res[False][2]):
        assert torch.equal(a.view(torch.int16) if a.element_size() == 2 else a,
                           c.view(torch.int16) if c.element_size() == 2 else c)


def _ddp_worker(rank, world, port, sd_path, data_path, out_path):
    """One rank of a 2-process DBSRTrainer run over gloo, both ranks on cuda:0 (RCCL refuses two ranks on
    one device): two steps on this rank's burst of the global batch, then its parameters and last gradients."""
    import os
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        sd = torch.load(sd_path, weights_only=True)
        data = torch.load(data_path, weights_only=True)
        net, tr = _trainer(sd, torch.float32)
        assert tr.world == world
        b, g = data['burst'][rank:rank + 1].to(DEV), data['gt'][rank:rank + 1].to(DEV)
        losses = [float(tr.step(b, g)) for _ in range(2)]
        torch.cuda.synchronize()
        torch.save({'flat': tr.flat.cpu(), 'grad': tr.flat_grad.cpu(), 'losses': losses}, out_path % rank)
    finally:
        dist.destroy_process_group()


def test_trainer_two_ranks_equals_one_process(synth_sd, tmp_path):
    """DBSRTrainer.step with world = 2 (the bucketed all-reduce between graph segments, then
    Adam with 1/world) -- two steps, the second a graph replay -- leaves the parameters a single-process trainer
    reaches on the concatenated batch; the summed gradients / 2 equal its gradients (admin/multigpu.py:8-14's
    DataParallel semantics: mean loss over the global batch)."""
    import socket
    import torch.multiprocessing as mp
    from dbsr_amd.burst import synthetic_bursts
    burst, gt = synthetic_bursts(2, 3, 24, 32, sr_factor=8, seed=29)
    sd_path, data_path = str(tmp_path / 'sd.pt'), str(tmp_path / 'data.pt')
    torch.save(dict(synth_sd), sd_path)
    torch.save({'burst': burst, 'gt': gt}, data_path)
    with socket.socket() as sk:
        sk.bind(('127.0.0.1', 0))
        port = sk.getsockname()[1]
    out = str(tmp_path / 'rank%d.pt')
    mp.start_processes(_ddp_worker, args=(2, port, sd_path, data_path, out), nprocs=2, join=True,
                       start_method='spawn')
    ranks = [torch.load(out % r, weights_only=True) for r in range(2)]
    torch.testing.assert_close(ranks[0]['flat'], ranks[1]['flat'], rtol=0, atol=0)      # replicas stay in sync
    net, tr = _trainer(synth_sd, torch.float32)
    b, g = burst.to(DEV), gt.to(DEV)
    losses = [float(tr.step(b, g)) for _ in range(2)]
    torch.cuda.synchronize()
    for i in range(2):
        assert (ranks[0]['losses'][i] + ranks[1]['losses'][i]) / 2 == pytest.approx(losses[i], rel=1e-5)
    gsum = (ranks[0]['grad'] / 2)
    ref = tr.flat_grad.cpu()
    assert float((gsum - ref).abs().max()) <= 1e-4 * float(ref.abs().max())
    # Adam's first steps move each weight by ~lr * grad / |grad|: within 2 % of a step wherever the gradient is
    # resolved; where it is rounding-level (|g| ~ its fp32 summation error) the normalised step may flip, which
    # bounds the difference by the two steps' 2 * lr
    diff = (ranks[0]['flat'] - tr.flat.cpu()).abs()
    assert float(diff.max()) <= 2 * tr.lr * 1.01
    assert float((diff > 2e-2 * tr.lr).float().mean()) <= 1e-3, float((diff > 2e-2 * tr.lr).float().mean())


def test_trainer_refuses_alignmentnet_training(synth_sd):
    """train_alignmentnet=True (the reference then trains PWC-Net, encoders.py:56-57) raises instead of
    silently freezing PWC-Net; with the default (False) the trainer leaves the PWC parameters' flags alone."""
    import dbsr_amd
    from dbsr_amd.training import DBSRTrainer
    net = dbsr_amd.dbsrnet_cvpr2021(**dict(dbsr_amd.DBSR_SYNTHETIC_KWARGS, train_alignmentnet=True))
    net.load_state_dict(synth_sd)
    net = net.to(DEV)
    with pytest.raises(NotImplementedError, match='train_alignmentnet'):
        DBSRTrainer(net)
    net2, _ = _trainer(synth_sd, torch.float32)
    assert all(p.requires_grad for p in net2.encoder.alignment_net.parameters())


def test_train_forward_follows_replaced_parameters(synth_sd):
    """after the parameters' storage is replaced (load_state_dict(assign=True)), the next train-mode
    forward packs the new weights, not the trainer's stale flat copy."""
    import dbsr_amd
    from dbsr_amd.burst import synthetic_bursts
    burst, _ = synthetic_bursts(1, 3, 24, 32, sr_factor=8, seed=5)
    net = dbsr_amd.dbsrnet_cvpr2021(**dbsr_amd.DBSR_SYNTHETIC_KWARGS)
    net.load_state_dict(synth_sd)
    net = net.to(DEV).train()
    b = burst.to(DEV)
    p1, _ = net(b)
    sd2 = {k: (v * 0.5 if k.startswith('decoder.predictor') else v).to(DEV) for k, v in synth_sd.items()}
    net.load_state_dict(sd2, assign=True)
    p2, _ = net(b)
    net.eval()
    with torch.no_grad():
        pe, _ = net(b)
    assert not torch.equal(p1.detach(), p2.detach())
    assert float((p2.detach() - pe).abs().max()) <= 1e-3


def test_engine_repacks_in_place_after_trainer_step(synth_sd):
    """after DBSRTrainer.step the inference engine keeps its plans and graphs and re-packs the
    updated weights into its own buffers; its forward equals a freshly built engine's, bitwise."""
    from dbsr_amd.burst import synthetic_bursts
    burst, gt = synthetic_bursts(1, 3, 24, 32, sr_factor=8, seed=31)
    b, g = burst.to(DEV), gt.to(DEV)
    net, tr = _trainer(synth_sd, torch.bfloat16)
    net.eval()
    with torch.no_grad():
        p0, _ = net(b)
    eng = net._engine
    tr.step(b, g)
    tr.step(b, g)
    with torch.no_grad():
        p1, _ = net(b)
        assert net._engine is eng and not eng.weights_stale
        net._engine = None
        p2, _ = net(b)
    assert not torch.equal(p0, p1)
    assert torch.equal(p1, p2)


def test_cfg4_training_steps_bf16(synth_sd):
    """configs[3]'s step shape (SyntheticBurst 14 frames, 128x128 -> 1024x1024, bf16; batch 2 here to
    keep the test short): three Adam steps on one batch run, stay finite and lower the loss."""
    from dbsr_amd.burst import synthetic_bursts
    burst, gt = synthetic_bursts(2, 14, 128, 128, sr_factor=8, seed=19)
    net, tr = _trainer(synth_sd, torch.bfloat16)
    b, g = burst.to(DEV), gt.to(DEV)
    losses = [float(tr.step(b, g)) for _ in range(3)]
    print('losses', losses)
    assert all(np.isfinite(losses))
    assert losses[-1] < losses[0]


# ----------------------------------------------------------------------------------------------------
# autograd through DBSRNet.forward: the reference's own loop, unchanged
# ----------------------------------------------------------------------------------------------------
def _objective(name, pred, gt, bi=40):
    p, g = pred[..., bi:-bi, bi:-bi], gt[..., bi:-bi, bi:-bi]
    return F.l1_loss(p, g) if name == 'l1' else F.mse_loss(p, g)


@pytest.mark.parametrize('dtype,objective', [(torch.float32, 'l1'), (torch.float32, 'mse'), (torch.bfloat16, 'l1')])
def test_autograd_reference_loop(synth_sd, dtype, objective):
    """actors/dbsr_actors.py:27-47 + trainers/simple_trainer.py:78-81 as written: pred, _ = net(burst);
    loss = objective(pred, gt); optimizer.zero_grad(); loss.backward(); optimizer.step() -- with
    torch.optim.Adam over the DBSR parameters.  The .grad the HIP backward leaves behind matches autograd
    through the oracle (the tolerances of test_train_step_grads_vs_oracle), the step moves the weights, a
    second iteration runs, and eval mode then serves the updated weights through the inference engine."""
    import dbsr_amd
    from dbsr_amd.burst import synthetic_bursts
    from oracle import dbsr_oracle as orc
    burst, gt = synthetic_bursts(2, 3, 24, 32, sr_factor=8, seed=17)
    sd = {k: v.clone().requires_grad_(not k.startswith('encoder.alignment_net')) for k, v in synth_sd.items()}
    rpred, _ = orc.dbsr_forward(burst, sd)
    rloss = _objective(objective, rpred, gt)
    rloss.backward()
    ref_g = {k: v.grad for k, v in sd.items() if v.grad is not None}
    net = dbsr_amd.dbsrnet_cvpr2021(**dbsr_amd.DBSR_SYNTHETIC_KWARGS)
    net.load_state_dict(synth_sd)
    net = net.to(DEV).set_compute_dtype(dtype).train()
    for p in net.encoder.alignment_net.parameters():
        p.requires_grad_(False)                          # train_alignmentnet=False (encoders.py:56-61)
    params = [p for p in net.parameters() if p.requires_grad]
    opt = torch.optim.Adam(params, lr=1e-4)
    b, g = burst.to(DEV), gt.to(DEV)
    pred, aux = net(b)
    assert pred.grad_fn is not None and aux['offsets'].shape == (2, 2, 2, 24, 32)
    loss = _objective(objective, pred, g)
    opt.zero_grad()
    loss.backward()
    mine = {k: p.grad.cpu() for k, p in net.named_parameters() if p.grad is not None}
    assert set(mine) == set(ref_g), set(mine) ^ set(ref_g)
    gmax = max(float(x.abs().max()) for x in ref_g.values())
    rel, cos = [], []
    for k, gr in ref_g.items():
        if k == 'merging.weight_predictor.4.0.bias':     # exact gradient 0 (softmax shift invariance)
            assert float(mine[k].abs().max()) <= 1e-4 * gmax
            continue
        rel.append((_rel(mine[k], gr), k))
        cos.append((1 - float(F.cosine_similarity(mine[k].double().flatten(), gr.double().flatten(), dim=0)), k))
    rel.sort(reverse=True)
    cos.sort(reverse=True)
    print(objective, dtype, 'loss', float(loss), float(rloss), 'max-rel worst', rel[:2], '1-cos worst', cos[:2])
    if dtype == torch.float32:
        assert abs(float(loss) - float(rloss)) <= 1e-5 * max(1.0, abs(float(rloss)))
        assert rel[0][0] <= 2e-2 and cos[0][0] <= 1e-4, (rel[:3], cos[:3])
    else:
        assert abs(float(loss) - float(rloss)) <= 1e-2 * abs(float(rloss))
        assert cos[0][0] <= 3e-2, cos[:3]
    before = [p.detach().clone() for p in params]
    opt.step()
    assert all(not torch.equal(a, p.detach()) for a, p in zip(before, params))
    pred2, _ = net(b)                                    # second iteration on the updated weights
    loss2 = _objective(objective, pred2, g)
    opt.zero_grad()
    loss2.backward()
    opt.step()
    assert torch.isfinite(loss2) and all(torch.isfinite(p.grad).all() for p in params)
    net.eval()
    with torch.no_grad():
        pe, _ = net(b)                                   # inference engine, repacked from the updated weights
    pt, _ = net.train()(b)
    assert float((pe.float() - pt.detach().float()).abs().max()) <= (1e-3 if dtype == torch.float32 else 0.1)


def test_autograd_backward_after_second_forward_raises(synth_sd):
    import dbsr_amd
    from dbsr_amd.burst import synthetic_bursts
    burst, _ = synthetic_bursts(1, 3, 24, 32, sr_factor=8, seed=3)
    net = dbsr_amd.dbsrnet_cvpr2021(**dbsr_amd.DBSR_SYNTHETIC_KWARGS)
    net.load_state_dict(synth_sd)
    net = net.to(DEV).train()
    b = burst.to(DEV)
    p1, _ = net(b)
    p2, _ = net(b)
    p2.sum().backward()
    with pytest.raises(RuntimeError, match='saved activations'):
        p1.sum().backward()
