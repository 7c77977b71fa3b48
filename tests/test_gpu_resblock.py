"""dbsr_resblock: a whole ResBlock (models/layers/blocks.py:81-96) in one kernel -- 32 channels (the decoder's post
blocks, decoders.py:46-49) and 64 channels (the encoder's, the offset-feature extractor's and the decoder's pre blocks:
encoders.py:36-46, merging.py:85-87, decoders.py:41-44) -- against the two dbsr_conv2d launches it replaces -- bitwise: both convs sum their
taps in the weight-stationary kernel's order, add the bias after the taps and the residual after the bias, and the
intermediate is rounded to the activation dtype exactly as the first launch stores it -- and against torch on the
same 16-bit operands (fp32 convs, the intermediate rounded to the dtype: atol 2e-2 + rtol 2 quanta)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

DEV = 'cuda'
pytestmark = pytest.mark.gpu


class _Slice:
    def __init__(self, t, c0):
        self.nhwc, self.c0 = t, c0

    def d(self, c0=0, fmap=None):
        return self.nhwc.d(self.c0 + c0) if fmap is None else self.nhwc.d(self.c0 + c0, fmap)


def _run(B, H, W, dt, seed, y_ld=32, y_c0=0, x_ld=32, x_c0=0, C=32, cap=0):
    from dbsr_amd import _lib as L
    from dbsr_amd.engine import NHWC, PackedConv, Plan
    gen = torch.Generator().manual_seed(seed)
    x = torch.randn(B, C, H, W, generator=gen)
    convs = []
    for _ in range(2):
        c = torch.nn.Conv2d(C, C, 3, padding=1)
        with torch.no_grad():
            c.weight.copy_(torch.randn(C, C, 3, 3, generator=gen) * (2.0 / (9 * C)) ** 0.5)
            c.bias.copy_(torch.randn(C, generator=gen) * 0.1)
        convs.append(c)
    dev = torch.device(DEV)
    s = torch.cuda.current_stream().cuda_stream
    pcs = [PackedConv(c.to(dev), dt, dev, s) for c in convs]
    X = NHWC(B, H, W, x_ld, dt, dev)
    X.t[..., x_c0:x_c0 + C].copy_(x.permute(0, 2, 3, 1).to(dt))
    Xs = _Slice(X, x_c0)
    outs = {}
    for fused in (True, False):
        Y = NHWC(B, H, W, y_ld, dt, dev)
        Y.t.fill_(7.0)                                  # channels outside the slice stay untouched
        M = NHWC(B, H, W, C, dt, dev)
        plan = Plan()
        plan.max_blocks = cap                           # a CU cap (the encoder's while PWC-Net runs beside it)
        if fused:
            assert plan.resblock('rb', pcs[0], pcs[1], B, Xs, M, _Slice(Y, y_c0), (H, W)), 'dbsr_resblock_ok rejected'
        else:
            plan.conv('c1', pcs[0], B, Xs, 0, (H, W), M, 0, L.ACT_RELU)
            plan.conv('c2', pcs[1], B, M, 0, (H, W), _Slice(Y, y_c0), 0, L.ACT_NONE, res=Xs, post_act=L.ACT_RELU)
        plan.finalize_workspace(dev)
        plan.run(s)
        torch.cuda.synchronize()
        outs[fused] = Y.t.cpu()
        if not fused:
            outs['kernels'] = set(plan.kernel.values())
    xb = x.to(dt).float()
    w = [c.weight.detach().cpu().to(dt).float() for c in convs]
    b = [c.bias.detach().cpu() for c in convs]
    mid = F.relu(F.conv2d(xb, w[0], b[0], padding=1)).to(dt).float()
    ref = F.relu(F.conv2d(mid, w[1], b[1], padding=1) + xb)
    return outs, ref.permute(0, 2, 3, 1)


@pytest.mark.parametrize('case', [(8, 384, 384, torch.float16, 32, 0, 32, 0),   # the bench decoder's post blocks
                                  (4, 128, 128, torch.bfloat16, 32, 0, 32, 0),
                                  (1, 384, 384, torch.float16, 32, 0, 32, 0),  # 288 tiles: a partial last round
                                  (3, 256, 256, torch.bfloat16, 32, 0, 32, 0), # 384 tiles
                                  (8, 64, 128, torch.float16, 48, 8, 40, 8),   # channel slices of x and y
                                  (1, 16, 32, torch.float16, 48, 8, 40, 8),    # one tile per frame
                                  (3, 48, 64, torch.bfloat16, 40, 0, 48, 16),
                                  # 64 channels (16 x 8 tiles, at most 2 per CU): 28 frames of 48x48 (504 tiles: full
                                  # XCD rounds + a partial one), 12 under a 128-CU cap, the decoder pre blocks (8
                                  # frames: 144 tiles), 96x96 frames, channel slices, one tile per frame
                                  (28, 48, 48, torch.float16, 64, 0, 64, 0, 64),
                                  (12, 48, 48, torch.float16, 64, 0, 64, 0, 64, 128),
                                  (8, 48, 48, torch.float16, 64, 0, 64, 0, 64),
                                  (4, 96, 96, torch.bfloat16, 64, 0, 64, 0, 64),
                                  (3, 32, 64, torch.float16, 80, 8, 72, 8, 64),
                                  (2, 8, 16, torch.bfloat16, 72, 0, 80, 16, 64)])
def test_resblock_vs_two_convs_and_torch(case):
    B, H, W, dt, y_ld, y_c0, x_ld, x_c0 = case[:8]
    C = case[8] if len(case) > 8 else 32
    cap = case[9] if len(case) > 9 else 0
    outs, ref = _run(B, H, W, dt, seed=B * 100 + H + W + C, y_ld=y_ld, y_c0=y_c0, x_ld=x_ld, x_c0=x_c0, C=C, cap=cap)
    f, t = outs[True], outs[False]
    nd = int((f.view(torch.int16) != t.view(torch.int16)).sum())
    if outs['kernels'] == {'conv3x3_ws'}:
        # the two launches ran the weight-stationary kernel, whose summation order the fused kernel keeps
        assert nd == 0, 'fused ResBlock differs from the two dbsr_conv2d launches at %d elements' % nd
    else:
        # (small frames dispatch the two launches to another kernel: same sums in another order)
        np.testing.assert_allclose(f.float().numpy(), t.float().numpy(), atol=1e-2, rtol=1e-2)
    if y_ld > C:
        mask = torch.ones(y_ld, dtype=torch.bool)
        mask[y_c0:y_c0 + C] = False
        assert torch.all(f[..., mask].float() == 7.0)
    eps = 2.0 ** -8 if dt == torch.bfloat16 else 2.0 ** -11
    np.testing.assert_allclose(f[..., y_c0:y_c0 + C].float().numpy(), ref.numpy(), atol=2e-2, rtol=2 * eps)


def test_resblock64_rejects_large_grids():
    """The 64-channel kernel serves at most 2 tiles (16 x 8) per CU (the decoder's pre-ResBlocks); the encoder's
    ResBlocks (112 frames of 48x48: 2016 tiles) keep the two weight-stationary launches (host-only check)."""
    import ctypes
    from dbsr_amd import _lib as L
    from dbsr_amd.engine import NHWC, PackedConv, Plan
    dev = torch.device(DEV)
    s = torch.cuda.current_stream().cuda_stream
    pcs = [PackedConv(torch.nn.Conv2d(64, 64, 3, padding=1).to(dev), torch.float16, dev, s) for _ in range(2)]
    for n, ok in ((112, False), (8, True)):
        X, M, Y = (NHWC(n, 48, 48, 64, torch.float16, dev) for _ in range(3))
        assert Plan().resblock('rb', pcs[0], pcs[1], n, X, M, Y, (48, 48)) == ok, n


def test_resblock64_in_engine_bitwise(synth_sd):
    """configs[1]'s forward (B=8, N=14, 48x48, fp16, HIP graph) with the 64-channel fused ResBlocks on and off
    (DBSREngine.FUSED_RESBLOCK64): the decoder-pre blocks are bitwise the two weight-stationary launches, so the
    prediction, the offsets and the fusion weights are bitwise equal."""
    import dbsr_amd
    from dbsr_amd.burst import synthetic_bursts
    from dbsr_amd.engine import DBSREngine
    burst, _ = synthetic_bursts(8, 14, 48, 48, sr_factor=8, seed=101)
    outs = {}
    old = DBSREngine.FUSED_RESBLOCK64
    try:
        for flag in (True, False):
            DBSREngine.FUSED_RESBLOCK64 = flag
            net = dbsr_amd.dbsrnet_cvpr2021(**dbsr_amd.DBSR_SYNTHETIC_KWARGS)
            net.load_state_dict(synth_sd)
            net = net.to(DEV).eval().set_compute_dtype(torch.float16)
            net.use_graph = True
            with torch.no_grad():
                net(burst.to(DEV))
                pred, aux = net(burst.to(DEV))
            plan = net._engine.plans[(8, 14, 48, 48)]
            kinds = list(plan.kernel.values())
            assert (kinds.count('resblock64') == 5) == flag, kinds
            outs[flag] = (pred.cpu(), aux['offsets'].cpu(), aux['fusion_weights'].cpu())
    finally:
        DBSREngine.FUSED_RESBLOCK64 = old
    for a, b, name in zip(outs[True], outs[False], ('pred', 'offsets', 'fusion_weights')):
        assert torch.equal(a, b), name


def test_resblock_in_engine_matches_unfused():
    """The DBSR forward (configs[1]'s architecture, seeded random weights, 24x24 bursts: 192x192 decoder frames)
    with DBSREngine.FUSED_RESBLOCK on and off.  The first post-blocks are bitwise the two ws launches; the last
    one carries the RGB head, which the unfused path computes on the pipelined kernel's conv2 (its own tap
    order), so the predictions agree to fp32 rounding (atol 1e-4; 24x24 bursts, every value printed)."""
    import dbsr_amd
    from dbsr_amd.engine import DBSREngine
    torch.manual_seed(0)
    sd = dbsr_amd.dbsrnet_cvpr2021(**dbsr_amd.DBSR_SYNTHETIC_KWARGS).state_dict()
    burst = torch.rand(2, 14, 4, 24, 24)
    outs = []
    old = DBSREngine.FUSED_RESBLOCK
    try:
        for flag in (True, False):
            DBSREngine.FUSED_RESBLOCK = flag
            net = dbsr_amd.dbsrnet_cvpr2021(**dbsr_amd.DBSR_SYNTHETIC_KWARGS)
            net.load_state_dict(sd)
            net = net.to(DEV).eval().set_compute_dtype(torch.float16)
            with torch.no_grad():
                pred, _ = net(burst.to(DEV))
            outs.append(pred.float().cpu())
    finally:
        DBSREngine.FUSED_RESBLOCK = old
    d = (outs[0] - outs[1]).abs()
    print('engine fused vs unfused ResBlocks: %.1f %% bitwise, max |diff| %.3g' % (
        100.0 * float((d == 0).float().mean()), float(d.max())))
    np.testing.assert_allclose(outs[0].numpy(), outs[1].numpy(), atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize('dt', [torch.float16, torch.bfloat16])
def test_resblock_head_vs_conv_head_and_torch(dt):
    """dbsr_resblock_head (the last decoder post-ResBlock + the RGB predictor, decoders.py:59-61) against conv1 +
    dbsr_conv2d_head (the pipelined kernel's fused head) and torch: the head is computed from the block's fp32
    output in both kernels with the same products and lane reduction; conv2's taps may be summed in another
    order by the pipelined kernel, so the comparison is at fp32 rounding (atol 1e-4), against torch at 2e-2."""
    from dbsr_amd import _lib as L
    from dbsr_amd.engine import NHWC, PackedConv, Plan
    B, H, W, hc = 2, 384, 384, 3
    gen = torch.Generator().manual_seed(77)
    x = torch.randn(B, 32, H, W, generator=gen)
    convs = []
    for _ in range(2):
        c = torch.nn.Conv2d(32, 32, 3, padding=1)
        with torch.no_grad():
            c.weight.copy_(torch.randn(32, 32, 3, 3, generator=gen) * (2.0 / 288) ** 0.5)
            c.bias.copy_(torch.randn(32, generator=gen) * 0.1)
        convs.append(c)
    hw = torch.randn(hc, 32, generator=gen) * 0.2
    hb = torch.randn(hc, generator=gen) * 0.1
    dev = torch.device(DEV)
    s = torch.cuda.current_stream().cuda_stream
    pcs = [PackedConv(c.to(dev), dt, dev, s) for c in convs]
    X = NHWC(B, H, W, 32, dt, dev)
    X.t.copy_(x.permute(0, 2, 3, 1).to(dt))
    preds = {}
    for fused in (True, False):
        M, Y = NHWC(B, H, W, 32, dt, dev), NHWC(B, H, W, 32, dt, dev)
        pred = torch.zeros(B, hc, H, W, dtype=torch.float32, device=dev)
        pdesc = L.tensor_desc(pred, 1, 0, img_stride=hc * H * W, dtype=torch.float32)
        head = ('predictor', hw.to(dev), hb.to(dev), pdesc)
        plan = Plan()
        if fused:
            assert plan.resblock('rb', pcs[0], pcs[1], B, X, M, Y, (H, W), head=head)
        else:
            plan.conv('c1', pcs[0], B, X, 0, (H, W), M, 0, L.ACT_RELU)
            d = plan.conv('c2', pcs[1], B, M, 0, (H, W), Y, 0, L.ACT_NONE, res=X, post_act=L.ACT_RELU, head=head)
            assert d.fused_head
        plan.finalize_workspace(dev)
        plan.run(s)
        torch.cuda.synchronize()
        preds[fused] = pred.cpu()
    f, t = preds[True], preds[False]
    print('resblock head vs conv head: %.1f %% bitwise, max |diff| %.3g' % (
        100.0 * float((f == t).float().mean()), float((f - t).abs().max())))
    np.testing.assert_allclose(f.numpy(), t.numpy(), atol=1e-4, rtol=1e-4)
    xb = x.to(dt).float()
    w = [c.weight.detach().cpu().to(dt).float() for c in convs]
    b = [c.bias.detach().cpu() for c in convs]
    mid = F.relu(F.conv2d(xb, w[0], b[0], padding=1)).to(dt).float()
    tt = F.relu(F.conv2d(mid, w[1], b[1], padding=1) + xb)
    ref = F.relu(F.conv2d(tt, hw.view(hc, 32, 1, 1), hb))
    np.testing.assert_allclose(f.numpy(), ref.numpy(), atol=2e-2, rtol=2e-2)
