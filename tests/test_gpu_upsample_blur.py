"""dbsr_conv_shuffle_blur: the decoder's PixelShuffle upsampler (1x1 conv Cin -> 64 x 32 + ReLU, PixelShuffle(8))
and its 3x3 Gaussian blur in one kernel (models/layers/upsampling.py:51-66, decoders.py:43,57), against the
two launches it replaces (dbsr_conv2d with DBSR_OUT_SHUFFLE + dbsr_gauss_blur3) -- bitwise: the fused kernel
rounds the conv output to the activation dtype in its LDS image exactly as the conv kernel stores it and sums
the blur taps in the blur kernel's order -- and against torch on the same 16-bit operands (fp32 conv, one
rounding of the conv output and of the result to the dtype: atol 2e-2 + rtol 2 quanta)."""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as F

DEV = 'cuda'
pytestmark = pytest.mark.gpu


def _gauss3(sd=1.0):
    ax = torch.arange(3, dtype=torch.float64) - 1
    g = torch.exp(-ax ** 2 / (2 * sd ** 2))
    k = torch.outer(g, g)
    return (k / k.sum()).float()


def _run(B, H, W, cin, dt, seed, y_ld=32, y_c0=0):
    from dbsr_amd import _lib as L
    from dbsr_amd.engine import NHWC, PackedConv, Plan
    S, pc = 8, 32
    gen = torch.Generator().manual_seed(seed)
    x = torch.randn(B, cin, H, W, generator=gen)
    conv = torch.nn.Conv2d(cin, pc * S * S, 1)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(pc * S * S, cin, 1, 1, generator=gen) * (2.0 / cin ** 0.5))
        conv.bias.copy_(torch.randn(pc * S * S, generator=gen) * 0.5)
    k9 = _gauss3(1.0)
    dev = torch.device(DEV)
    s = torch.cuda.current_stream().cuda_stream
    packed = PackedConv(conv.to(dev), dt, dev, s, shuffle=S)
    X = NHWC(B, H, W, 32 if cin <= 32 else 64, dt, dev)     # the packed K: cin padded to 32 / 64 channels
    X.t.zero_()
    X.t[..., :cin].copy_(x.permute(0, 2, 3, 1).to(dt))
    outs = {}
    for fused in (True, False):
        Y = NHWC(B, H * S, W * S, y_ld, dt, dev)
        Y.t.fill_(7.0)                                   # channels outside the slice must stay untouched
        plan = Plan()
        if fused:
            d = plan.conv_shuffle_blur('ub', packed, B, X, (H, W), _Slice(Y, y_c0), L.ACT_RELU, k9.flatten().tolist())
            assert d is not None, 'dbsr_conv_shuffle_blur_ok rejected the case'
        else:
            T = NHWC(B, H * S, W * S, pc, dt, dev)
            plan.conv('up', packed, B, X, 0, (H, W), T, 0, L.ACT_RELU, out_mode=L.OUT_SHUFFLE, shuffle=S)
            kbuf = (ctypes.c_float * 9)(*k9.flatten().tolist())
            plan.keep.append(kbuf)
            plan.add('blur', L.lib().dbsr_gauss_blur3, B, H * S, W * S, pc, T.d(0), kbuf, Y.d(y_c0))
        plan.finalize_workspace(dev)
        plan.run(s)
        torch.cuda.synchronize()
        outs[fused] = Y.t.cpu()
    # torch: the conv on the rounded operands, its output rounded to the dtype, blurred, rounded again
    xb = x.to(dt).float()
    wb = conv.weight.detach().cpu().to(dt).float()
    up = F.pixel_shuffle(F.relu(F.conv2d(xb, wb, conv.bias.detach().cpu())), S).to(dt).float()
    bl = F.conv2d(up.reshape(-1, 1, H * S, W * S), k9.view(1, 1, 3, 3), padding=1).reshape(B, pc, H * S, W * S)
    return outs, bl.permute(0, 2, 3, 1)


class _Slice:
    """An NHWC buffer viewed from channel c0 (Plan.conv_shuffle_blur writes y.d(0))."""
    def __init__(self, t, c0):
        self.nhwc, self.c0 = t, c0

    def d(self, c0=0, fmap=None):
        return self.nhwc.d(self.c0 + c0) if fmap is None else self.nhwc.d(self.c0 + c0, fmap)


@pytest.mark.parametrize('case', [(2, 48, 48, 64, torch.bfloat16, 32, 0),     # the bench decoder's shape
                                  (2, 48, 48, 64, torch.float16, 32, 0),      # ... at the bench dtype
                                  (1, 8, 12, 32, torch.float16, 48, 8),       # Cin 32, a channel slice of y
                                  (3, 4, 4, 64, torch.bfloat16, 32, 0),       # one tile per frame: all-zero ring
                                  (1, 12, 20, 48, torch.bfloat16, 40, 8)])    # Cin 48 (padded to 64)
def test_shuffle_blur_vs_two_launches_and_torch(case):
    B, H, W, cin, dt, y_ld, y_c0 = case
    outs, ref = _run(B, H, W, cin, dt, seed=B * 1000 + H * 10 + cin, y_ld=y_ld, y_c0=y_c0)
    f, t = outs[True], outs[False]
    assert torch.equal(f.view(torch.int16), t.view(torch.int16)), \
        'fused upsample+blur differs from dbsr_conv2d + dbsr_gauss_blur3 at %d elements' % \
        int((f.view(torch.int16) != t.view(torch.int16)).sum())
    # the channels outside [c0, c0 + 32) are untouched
    if y_ld > 32:
        mask = torch.ones(y_ld, dtype=torch.bool)
        mask[y_c0:y_c0 + 32] = False
        assert torch.all(f[..., mask].float() == 7.0)
    eps = 2.0 ** -8 if dt == torch.bfloat16 else 2.0 ** -11
    np.testing.assert_allclose(f[..., y_c0:y_c0 + 32].float().numpy(), ref.numpy(), atol=2e-2, rtol=2 * eps)


def test_shuffle_blur_in_engine_matches_unfused():
    """The DBSR forward (configs[1]'s architecture, seeded random weights) with DBSREngine.FUSED_UPSAMPLE_BLUR on
    and off: bitwise equal predictions."""
    import dbsr_amd
    from dbsr_amd.engine import DBSREngine
    torch.manual_seed(0)
    sd = dbsr_amd.dbsrnet_cvpr2021(**dbsr_amd.DBSR_SYNTHETIC_KWARGS).state_dict()
    burst = torch.rand(2, 14, 4, 24, 24)
    outs = []
    old = DBSREngine.FUSED_UPSAMPLE_BLUR
    try:
        for flag in (True, False):
            DBSREngine.FUSED_UPSAMPLE_BLUR = flag
            net = dbsr_amd.dbsrnet_cvpr2021(**dbsr_amd.DBSR_SYNTHETIC_KWARGS)
            net.load_state_dict(sd)
            net = net.to(DEV).eval().set_compute_dtype(torch.float16)
            with torch.no_grad():
                pred, _ = net(burst.to(DEV))
            outs.append(pred.float().cpu())
    finally:
        DBSREngine.FUSED_UPSAMPLE_BLUR = old
    assert torch.equal(outs[0], outs[1])
