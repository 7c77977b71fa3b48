"""dbsr_conv_fuse_softmax (the weight predictor's last conv + softmax over the
burst + fusion in one kernel, models/dbsr/merging.py:55-57,113-124; the product default,
DBSREngine.FUSED_WP_OUT) against torch on the same 16-bit operands, and against the two-kernel path
(dbsr_conv2d to a 16-bit logits buffer + dbsr_fuse_softmax).

Tolerances.  Against torch (fp32 conv of the rounded operands + bias, fp32 softmax, fp32 weighted sum --
the kernel's own arithmetic, the logits never rounded): the outputs differ by the K summation order and the
final rounding to the 16-bit output dtype: weights atol 1e-3 + rtol 1e-2 of the dtype, fused atol 1e-2.
Against the two-kernel path, which rounds every logit to 16 bits before the softmax: a weight moves by up
to |l| * 2^-8 (bf16) / 2^-11 (fp16) relative, so rtol 5e-2 (bf16) / 1e-2 (fp16) at the |l| <~ 6 here."""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as F

DEV = 'cuda'
pytestmark = pytest.mark.gpu


def _case(B, N, H, W, cin, C, dt, seed, want_fw=True, strided=False, relu=False):
    """relu: WeightedSum(softmax=False) -- dbsr_conv_fuse_relu_norm / dbsr_fuse_relu_norm, torch relu(l) / (sum + 1e-12).
    strided: every tensor addressed through a non-identity frame map -- the hidden input as every
    second stored image (f -> 2f + 1), the reference embeddings behind one leading burst (b -> (b + 1) N), the
    warped frames behind 3 images, the fused output behind one image; the kernel derives all of its addressing
    from these maps (affine_frames)."""
    from dbsr_amd import _lib as L
    from dbsr_amd.engine import NHWC, PackedConv, Plan
    gen = torch.Generator().manual_seed(seed)
    h = torch.randn(B * N, cin, H, W, generator=gen)
    conv = torch.nn.Conv2d(cin, C, 3, padding=1)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(C, cin, 3, 3, generator=gen) * (3.0 / (cin * 9) ** 0.5))
        conv.bias.copy_(torch.randn(C, generator=gen))
    feat = torch.randn(B, N, C, H, W, generator=gen)
    w_cpu, b_cpu = conv.weight.detach().clone(), conv.bias.detach().clone()
    dev = torch.device(DEV)
    s = torch.cuda.current_stream().cuda_stream
    pc = PackedConv(conv.to(dev), dt, dev, s)
    P = B * (N - 1)
    xo, eo, wo, fo = (1, N, 3, 1) if strided else (0, 0, 0, 0)
    X = NHWC(2 * B * N if strided else B * N, H, W, cin, dt, dev)
    (X.t[1::2] if strided else X.t).copy_(h.permute(0, 2, 3, 1).to(dt))
    xmap = (1, 2, 1, 1) if strided else (1, 1, 0, 1)
    E = NHWC(B * N + eo, H, W, C, dt, dev)      # frame embeddings, ref = frame b*N (+ eo)
    E.t[eo:].copy_(feat.reshape(B * N, C, H, W).permute(0, 2, 3, 1).to(dt))
    Wf = NHWC(P + wo, H, W, C, dt, dev)         # "warped" frames 1..N-1 of each burst (+ wo)
    Wf.t[wo:].copy_(feat[:, 1:].reshape(P, C, H, W).permute(0, 2, 3, 1).to(dt))
    outs = {}
    for fused_path in (True, False):
        FUS = NHWC(B + fo, H, W, C, dt, dev)
        FW = NHWC(B * N, H, W, C, dt, dev)
        plan = Plan()
        feats = [E.d(0, (1, N, eo, 1)), Wf.d(0, (1, 1, wo, 1)), FUS.d(0, (1, 1, fo, 1)),
                 FW.d(0) if want_fw else L.NULL_TENSOR]
        if fused_path:
            idx = plan.conv_fuse('fz', pc, B, N, X, (H, W), *feats, xmap=xmap, softmax=not relu)
            assert idx is not None, 'dbsr_conv_fuse_ok rejected the case'
        else:
            LG = NHWC(B * N, H, W, C, dt, dev)
            plan.conv('lg', pc, B * N, X, 0, (H, W), LG, 0, L.ACT_NONE, xmap=xmap)
            fn = L.lib().dbsr_fuse_relu_norm if relu else L.lib().dbsr_fuse_softmax
            plan.add('fuse', fn, B, N, H * W, C, LG.d(0), *feats)
        plan.finalize_workspace(dev)
        plan.run(s)
        torch.cuda.synchronize()
        if strided:
            assert FUS.t[:fo].abs().max() == 0 and X.t[0::2].abs().max() == 0     # nothing outside the maps
        outs[fused_path] = (FUS.t[fo:].float().cpu(), FW.t.float().cpu())
    # torch reference on the rounded operands, fp32 logits (as the fused kernel keeps them)
    hb = h.to(dt).float()
    wb = w_cpu.to(dt).float()
    lg = F.conv2d(hb, wb, b_cpu, padding=1).reshape(B, N, C, H, W)
    if relu:
        wts = F.relu(lg)
        wts = wts / (wts.sum(dim=1, keepdim=True) + 1e-12)
    else:
        wts = torch.softmax(lg, dim=1)
    fz = (feat.to(dt).float() * wts).sum(dim=1)
    ref = (fz.permute(0, 2, 3, 1), wts.reshape(B * N, C, H, W).permute(0, 2, 3, 1))
    return outs, ref


@pytest.mark.parametrize('case', [(2, 14, 48, 48, 128, 512, torch.bfloat16),    # the bench shape's layer
                                  (2, 14, 48, 48, 128, 512, torch.float16),     # ... at the bench dtype
                                  (1, 14, 32, 16, 128, 128, torch.float16),     # non-square, one channel slice
                                  (3, 14, 8, 48, 96, 256, torch.bfloat16),      # 3 input chunks, 2 slices
                                  (2, 14, 16, 48, 128, 512, torch.float16, True),  # strided / offset frame maps
                                  (3, 14, 8, 32, 128, 256, torch.bfloat16, True)])
def test_conv_fuse_vs_torch_and_two_kernel(case):
    B, N, H, W, cin, C, dt = case[:7]
    strided = len(case) > 7
    outs, (rf, rw) = _case(B, N, H, W, cin, C, dt, seed=B * 100 + H + C, strided=strided)
    (f1, w1), (f0, w0) = outs[True], outs[False]
    eps = 2.0 ** -8 if dt == torch.bfloat16 else 2.0 ** -11
    # against torch: summation order + one rounding of each output to the dtype
    np.testing.assert_allclose(w1.numpy(), rw.numpy(), atol=1e-3, rtol=2 * eps)
    np.testing.assert_allclose(f1.numpy(), rf.numpy(), atol=1e-2, rtol=4 * eps)
    # against the two-kernel path: its logits are rounded to the dtype first (bf16: a weight moves by up to
    # |l| * 2^-8 relative, a fused value by the sum of those over the burst -- measured up to 0.047 here)
    rt = 5e-2 if dt == torch.bfloat16 else 1e-2
    np.testing.assert_allclose(w1.numpy(), w0.numpy(), atol=2e-3, rtol=rt)
    np.testing.assert_allclose(f1.numpy(), f0.numpy(), atol=8e-2 if dt == torch.bfloat16 else 2e-2, rtol=rt)
    # the fused kernel is closer to torch than the two-kernel path (the logits are not rounded)
    assert (w1 - rw).abs().mean() <= (w0 - rw).abs().mean()
    # the weights of a pixel sum to 1 over the burst
    s = w1.reshape(B, N, H, W, C).sum(dim=1)
    assert (s - 1).abs().max() < 0.05


def test_conv_fuse_without_aux_weights():
    outs, (rf, _) = _case(1, 14, 16, 48, 128, 128, torch.bfloat16, seed=7, want_fw=False)
    f1, w1 = outs[True]
    assert w1.abs().max() == 0                   # aux output skipped
    np.testing.assert_allclose(f1.numpy(), rf.numpy(), atol=1e-2, rtol=2 ** -6)


def test_conv_fuse_rejects_unsupported():
    from dbsr_amd import _lib as L
    d = L.ConvDesc()
    d.n_frames = 13 * 2
    d.x = L.Tensor(1, L.DBSR_BF16, 48 * 48 * 128, 128, 0, L.FrameMap(1, 1, 0, 1))
    d.in_h = d.in_w = d.out_h = d.out_w = 48
    d.cin, d.cout, d.kh, d.kw, d.stride, d.pad, d.dil = 128, 512, 3, 3, 1, 1, 1
    d.w = 1
    assert L.lib().dbsr_conv_fuse_ok(ctypes.byref(d), 2, 13) == 0          # burst size 13
    d.n_frames = 28
    assert L.lib().dbsr_conv_fuse_ok(ctypes.byref(d), 2, 14) == 1
    d.cout = 192
    assert L.lib().dbsr_conv_fuse_ok(ctypes.byref(d), 2, 14) == 0          # cout % 128
    d.cout = 512
    d.in_h = d.out_h = 47
    assert L.lib().dbsr_conv_fuse_ok(ctypes.byref(d), 2, 14) == 0          # odd height
    d.in_h = d.out_h = 48
    d.x.dtype = L.DBSR_F32
    assert L.lib().dbsr_conv_fuse_ok(ctypes.byref(d), 2, 14) == 0          # fp32: two-kernel path


@pytest.mark.parametrize('dt', [torch.float16, torch.bfloat16])
def test_engine_fused_wp_out_matches_default(synth_sd, dt):
    """The whole 16-bit forward (fp16 = the product dtype, and bf16) with DBSREngine.FUSED_WP_OUT on (weight-
    predictor output conv + softmax + fusion in one launch) against the two-kernel plan, B=2 N=14 48x48: pred
    within the bench-shape parity bounds and the fusion weights within the torch tolerance above."""
    import dbsr_amd
    from dbsr_amd.burst import synthetic_bursts
    from dbsr_amd.engine import DBSREngine
    burst, _ = synthetic_bursts(2, 14, 48, 48, sr_factor=8, seed=77)
    burst = burst.to(DEV)
    outs = {}
    old = DBSREngine.FUSED_WP_OUT
    try:
        for flag in (True, False):
            DBSREngine.FUSED_WP_OUT = flag
            net = dbsr_amd.dbsrnet_cvpr2021(**dbsr_amd.DBSR_SYNTHETIC_KWARGS)
            net.load_state_dict(synth_sd)
            net = net.to(DEV).eval().set_compute_dtype(dt)
            with torch.no_grad():
                pred, aux = net(burst)
            names = [name for _, _, name, _ in net._engine.plans[(2, 14, 48, 48)].ops]
            assert ('merge.wp.out+fuse' in names) == flag, names
            outs[flag] = (pred.float().cpu(), aux['fusion_weights'].float().cpu())
    finally:
        DBSREngine.FUSED_WP_OUT = old
    (p1, w1), (p0, w0) = outs[True], outs[False]
    # bf16 differences from the logits' K order and the online softmax grow through the decoder (~30
    # bf16 convs): the bench-shape parity bounds of tests/test_gpu_parity.py (2^14 quanta)
    dq = ((p1 - p0).abs() * 2 ** 14).flatten()
    assert torch.quantile(dq[:2 ** 24].float(), 0.999) <= 320 and dq.max() <= 800, (dq.max().item(),)
    np.testing.assert_allclose(w1.numpy(), w0.numpy(), atol=2e-3, rtol=5e-2 if dt == torch.bfloat16 else 1e-2)


def _frac_outside(a, b, atol, rtol):
    return float(((a - b).abs() > atol + rtol * b.abs()).float().mean())


@pytest.mark.parametrize('dt', [torch.float16, torch.bfloat16])
def test_conv_fuse_relu_norm(dt):
    """softmax=False (merging.py:119-121) at the bench shape's layer: the fused kernel (fp32 logits) against torch on
    the same operands and against the two-kernel path (16-bit logits + dbsr_fuse_relu_norm).  relu(l) / sum relu(l)
    has no floor under its denominator: where a pixel's positive logits sum to ~1e-4 a 1e-6 change of a logit (K
    order) moves its weights by ~1e-2, so the bounds are the softmax test's tolerances met by all but 1e-4 of the
    elements against torch (1e-3 against the rounded-logit path)."""
    B, N, H, W, cin, C = 2, 14, 48, 48, 128, 512
    outs, (rf, rw) = _case(B, N, H, W, cin, C, dt, seed=901, relu=True)
    (f1, w1), (f0, w0) = outs[True], outs[False]
    eps = 2.0 ** -8 if dt == torch.bfloat16 else 2.0 ** -11
    assert _frac_outside(w1, rw, 1e-3, 2 * eps) <= 1e-4
    assert _frac_outside(f1, rf, 1e-2, 4 * eps) <= 1e-4
    rt = 5e-2 if dt == torch.bfloat16 else 1e-2
    assert _frac_outside(w1, w0, 2e-3, rt) <= 1e-3
    assert _frac_outside(f1, f0, 8e-2 if dt == torch.bfloat16 else 2e-2, rt) <= 1e-3
    assert (w1 - rw).abs().mean() <= (w0 - rw).abs().mean()
    s = w1.reshape(B, N, H, W, C).sum(dim=1)
    assert float(torch.minimum((s - 1).abs(), s.abs()).max()) < 0.05     # 1, or 0 where every logit is <= 0
    assert float((s == 0).float().mean()) > 0                               # (both cases occur here)
