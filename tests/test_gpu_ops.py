"""Op-level parity of the HIP kernels (through the C ABI) against the oracle and the reference
fixtures.  fp32 tolerances are written per test; bf16 tests use relative tolerances sized for
8-bit mantissas with fp32 accumulation."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import dbsr_oracle as orc

pytestmark = pytest.mark.gpu
DEV = 'cuda'


@pytest.fixture(scope='module')
def ops():
    from dbsr_amd import ops as O
    return O


def test_correlation_fixture(golden, ops):
    g = golden('ops')
    out = ops.FunctionCorrelation(torch.from_numpy(g['corr_f1']).to(DEV), torch.from_numpy(g['corr_f2']).to(DEV))
    np.testing.assert_allclose(out.cpu().numpy(), g['corr_out'], atol=1e-5, rtol=0)


@pytest.mark.parametrize('shape', [(3, 196, 1, 1), (2, 128, 2, 2), (2, 96, 4, 4), (2, 64, 8, 8), (3, 32, 16, 16),
                                   (1, 20, 5, 7)])
def test_correlation_levels(ops, shape):
    gen = torch.Generator().manual_seed(shape[1])
    a, b = torch.randn(*shape, generator=gen), torch.randn(*shape, generator=gen)
    out = ops.FunctionCorrelation(a.to(DEV), b.to(DEV), leaky=True)
    ref = F.leaky_relu(orc.correlation(a, b), 0.1)
    np.testing.assert_allclose(out.cpu().numpy(), ref.numpy(), atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize('tag', ['bw8', 'bw2'])
def test_backwarp_fixture(golden, ops, tag):
    g = golden('ops')
    x = torch.from_numpy(g[f'{tag}_x']).to(DEV)
    fl = torch.from_numpy(g[f'{tag}_flow']).to(DEV) * float(g[f'{tag}_scale'])
    out = ops.backwarp(x, fl)
    np.testing.assert_allclose(out.cpu().numpy(), g[f'{tag}_out'], atol=1e-5, rtol=0)


def test_warp_fixture(golden, ops):
    g = golden('ops')
    out = ops.warp(torch.from_numpy(g['warp_x']).to(DEV), torch.from_numpy(g['warp_flow']).to(DEV))
    np.testing.assert_allclose(out.cpu().numpy(), g['warp_out'], atol=1e-5, rtol=0)


def test_warp_large_flow_and_zero(ops):
    gen = torch.Generator().manual_seed(7)
    x = torch.randn(4, 512, 48, 48, generator=gen)
    fl = torch.randn(4, 2, 48, 48, generator=gen) * 4.0
    fl[0] = 0.0
    fl[3] *= 20.0             # mostly outside the frame -> zeros
    out = ops.warp(x.to(DEV), fl.to(DEV)).cpu()
    np.testing.assert_allclose(out.numpy(), orc.warp(x, fl).numpy(), atol=1e-5, rtol=0)


CONV_CASES = [
    # (N, Cin, H, W, Cout, k, stride, pad, dil)
    (3, 4, 12, 12, 64, 3, 1, 1, 1),
    (2, 64, 16, 16, 64, 3, 1, 1, 1),
    (2, 64, 9, 11, 512, 3, 1, 1, 1),
    (2, 512, 7, 7, 64, 1, 1, 0, 1),
    (2, 3, 64, 64, 16, 3, 2, 1, 1),
    (3, 196, 1, 1, 128, 3, 1, 1, 1),
    (2, 117, 16, 16, 128, 3, 1, 1, 1),
    (2, 565, 16, 16, 128, 3, 1, 1, 1),
    (2, 128, 16, 16, 96, 3, 1, 8, 8),
    (2, 64, 16, 16, 32, 3, 1, 16, 16),
    (2, 32, 16, 16, 2, 3, 1, 1, 1),
    (2, 2, 10, 10, 64, 3, 1, 1, 1),
    (1, 32, 40, 24, 3, 1, 1, 0, 1),
    (2, 32, 40, 24, 32, 3, 1, 1, 1),       # tiled kernel, 32-cout variant, partial tiles
    (2, 192, 20, 17, 128, 3, 1, 1, 1),     # tiled kernel, 6 chunks, 2 cout tiles
    (3, 128, 48, 48, 512, 3, 1, 1, 1),     # tiled kernel at the weight-predictor shape
    (2, 565, 16, 16, 2, 3, 1, 1, 1),       # split-K (2-channel flow head)
    (104, 529, 1, 1, 32, 3, 1, 1, 1),      # split-K (PWC level 6)
    (7, 469, 4, 4, 64, 3, 1, 1, 1),        # split-K (PWC level 4)
    (2, 128, 16, 16, 128, 3, 1, 2, 2),     # tiled kernel, dilation 2 (PWC refiner)
    (2, 128, 19, 16, 128, 3, 1, 4, 4),     # tiled kernel, dilation 4, partial tile
    (1, 64, 48, 48, 64, 3, 1, 1, 1),       # tiled kernel, small grid -> 16x4-pixel tiles
]
DILATED_BF16 = [
    (2, 128, 16, 16, 128, 3, 1, 2, 2),
    (2, 128, 16, 16, 128, 3, 1, 4, 4),
    (2, 128, 16, 16, 96, 3, 1, 8, 8),
    (3, 96, 20, 16, 64, 3, 1, 8, 8),
]


@pytest.mark.parametrize('case', CONV_CASES)
def test_conv2d_fp32(ops, case):
    N, Cin, H, W, Cout, k, s, p, d = case
    gen = torch.Generator().manual_seed(Cin * 1000 + Cout)
    x = torch.randn(N, Cin, H, W, generator=gen)
    w = torch.randn(Cout, Cin, k, k, generator=gen) / (Cin * k * k) ** 0.5
    b = torch.randn(Cout, generator=gen) * 0.1
    ref = F.leaky_relu(F.conv2d(x, w, b, stride=s, padding=p, dilation=d), 0.1)
    out = ops.conv2d(x.to(DEV), w.to(DEV), b.to(DEV), stride=s, padding=p, dilation=d, act=2).cpu()
    np.testing.assert_allclose(out.numpy(), ref.numpy(), atol=2e-5, rtol=1e-4)


@pytest.mark.parametrize('case', CONV_CASES[:4] + DILATED_BF16 + CONV_CASES[-1:])
def test_conv2d_bf16(ops, case):
    N, Cin, H, W, Cout, k, s, p, d = case
    gen = torch.Generator().manual_seed(Cin * 1000 + Cout + 1)
    x = torch.randn(N, Cin, H, W, generator=gen)
    w = torch.randn(Cout, Cin, k, k, generator=gen) / (Cin * k * k) ** 0.5
    xb = x.to(torch.bfloat16).float()
    wb = w.to(torch.bfloat16).float()
    ref = F.conv2d(xb, wb, None, stride=s, padding=p, dilation=d)    # same rounded inputs, fp32 math
    out = ops.conv2d(x.to(DEV), w.to(DEV), None, stride=s, padding=p, dilation=d,
                     compute_dtype=torch.bfloat16, out_f32=True).cpu()
    np.testing.assert_allclose(out.numpy(), ref.numpy(), atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('case', [(2, 64, 48, 48, 64), (2, 32, 70, 36, 32), (1, 128, 17, 33, 96)])
def test_conv2d_tiled_vs_generic(ops, dtype, case):
    from dbsr_amd import _lib
    N, Cin, H, W, Cout = case
    gen = torch.Generator().manual_seed(H * W)
    x = torch.randn(N, Cin, H, W, generator=gen).to(DEV)
    w = (torch.randn(Cout, Cin, 3, 3, generator=gen) / (Cin * 9) ** 0.5).to(DEV)
    b = (torch.randn(Cout, generator=gen) * 0.1).to(DEV)
    res = torch.randn(N, Cout, H, W, generator=gen).to(DEV)
    outs = []
    for algo in (1, 0):
        _lib.lib().dbsr_set_conv_algo(algo)
        outs.append(ops.conv2d(x, w, b, padding=1, act=1, residual=res, post_act=1, compute_dtype=dtype).float().cpu())
    _lib.lib().dbsr_set_conv_algo(2)
    # same products, fp32 accumulation, different summation order; outputs rounded to dtype
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    np.testing.assert_allclose(outs[0].numpy(), outs[1].numpy(), atol=tol, rtol=tol)


def test_conv2d_residual_relu(ops):
    gen = torch.Generator().manual_seed(5)
    x = torch.randn(2, 64, 12, 12, generator=gen)
    w = torch.randn(64, 64, 3, 3, generator=gen) / 24.0
    b = torch.randn(64, generator=gen) * 0.1
    res = torch.randn(2, 64, 12, 12, generator=gen)
    ref = F.relu(F.conv2d(x, w, b, padding=1) + res)
    out = ops.conv2d(x.to(DEV), w.to(DEV), b.to(DEV), padding=1, residual=res.to(DEV), post_act=1).cpu()
    np.testing.assert_allclose(out.numpy(), ref.numpy(), atol=2e-5, rtol=1e-4)


def test_pwcnet_fixture(golden, synth_sd):
    import dbsr_amd
    g = golden('ops')
    net = dbsr_amd.dbsrnet_cvpr2021(**dbsr_amd.DBSR_SYNTHETIC_KWARGS)
    net.load_state_dict(synth_sd)
    pwc = net.encoder.alignment_net.to(DEV)
    with torch.no_grad():
        fl = pwc(torch.from_numpy(g['pwc_src']).to(DEV), torch.from_numpy(g['pwc_tgt']).to(DEV))
    np.testing.assert_allclose(fl.cpu().numpy(), g['pwc_flow'], atol=1e-3, rtol=0)


PIPE_CASES = [   # N, Cin, H, W, Cout  (pipelined kernel configs: 64 x 48x8 and 32 x 64x8 tiles)
    (2, 64, 48, 48, 64),        # encoder ResBlock shape, 2 chunks
    (1, 192, 16, 48, 128),      # weight-predictor init: 6 chunks, 2 cout tiles
    (1, 128, 8, 96, 80),        # partial cout tile (80 = 64 + 16)
    (2, 32, 16, 128, 32),       # decoder post-ResBlock shape (1 chunk, 32-cout tiles)
    (1, 40, 8, 64, 24),         # cin padded 40 -> 64, cout 24 < 32
    (1, 64, 24, 64, 64),        # 64-wide, 64 couts: not a pipelined shape (falls back)
]


@pytest.mark.parametrize('case', PIPE_CASES)
def test_conv2d_pipelined(ops, case):
    """Pipelined persistent 3x3 kernel (algo 3 forces it) against the two-barrier tiled and generic
    kernels and a torch fp32 conv on the same bf16-rounded operands."""
    from dbsr_amd import _lib
    N, Cin, H, W, Cout = case
    gen = torch.Generator().manual_seed(Cin * 7 + Cout + H)
    x = torch.randn(N, Cin, H, W, generator=gen)
    w = torch.randn(Cout, Cin, 3, 3, generator=gen) / (Cin * 9) ** 0.5
    b = torch.randn(Cout, generator=gen) * 0.1
    res = torch.randn(N, Cout, H, W, generator=gen)
    xb, wb, rb = (t.to(torch.bfloat16).float() for t in (x, w, res))
    ref = F.relu(F.relu(F.conv2d(xb, wb, b, padding=1)) + rb)
    outs = {}
    try:
        for algo in (3, 1, 0):
            _lib.lib().dbsr_set_conv_algo(algo)
            outs[algo] = ops.conv2d(x.to(DEV), w.to(DEV), b.to(DEV), padding=1, act=1, residual=res.to(DEV),
                                    post_act=1, compute_dtype=torch.bfloat16).float().cpu()
    finally:
        _lib.lib().dbsr_set_conv_algo(2)
    # bf16 outputs: one rounding of the fp32 sum (+ one of the pre-residual value) -> ~2^-8 relative
    np.testing.assert_allclose(outs[3].numpy(), ref.numpy(), atol=3e-2, rtol=2e-2)
    np.testing.assert_allclose(outs[3].numpy(), outs[1].numpy(), atol=3e-2, rtol=2e-2)
    np.testing.assert_allclose(outs[3].numpy(), outs[0].numpy(), atol=3e-2, rtol=2e-2)
    assert (outs[3] - ref).abs().mean() < 3e-3


@pytest.mark.parametrize('case', [(2, 32, 16, 128, 3), (1, 32, 24, 64, 1), (3, 32, 8, 192, 4)])
def test_conv2d_fused_head(ops, case):
    """Last decoder ResBlock conv2 + RGB predictor in one pipelined kernel (dbsr_conv2d_head) against
    torch fp32 on the same bf16-rounded operands: relu(W_h . relu(conv(x) + b + res) + b_h)."""
    from dbsr_amd import _lib
    N, C, H, W, hc = case
    gen = torch.Generator().manual_seed(H * 31 + W + hc)
    x = torch.randn(N, C, H, W, generator=gen)
    w = torch.randn(C, C, 3, 3, generator=gen) / (C * 9) ** 0.5
    b = torch.randn(C, generator=gen) * 0.1
    res = torch.randn(N, C, H, W, generator=gen)
    hw = torch.randn(hc, C, 1, 1, generator=gen) / C ** 0.5
    hb = torch.randn(hc, generator=gen) * 0.1
    xb, wb, rb = (t.to(torch.bfloat16).float() for t in (x, w, res))
    ref = F.relu(F.conv2d(F.relu(F.conv2d(xb, wb, b, padding=1) + rb), hw, hb))
    try:
        _lib.lib().dbsr_set_conv_algo(3)      # pipelined kernel at any tile count
        out = ops.conv2d(x.to(DEV), w.to(DEV), b.to(DEV), padding=1, act=0, residual=res.to(DEV), post_act=1,
                         compute_dtype=torch.bfloat16, head=(hw.to(DEV), hb.to(DEV))).cpu()
    finally:
        _lib.lib().dbsr_set_conv_algo(2)
    assert out.shape == (N, hc, H, W)
    # fp32 head on the fp32 ResBlock output: only the bf16 operands of the 3x3 conv differ from torch
    np.testing.assert_allclose(out.numpy(), ref.numpy(), atol=2e-3, rtol=2e-3)


def test_conv2d_head_rejects_ineligible(ops):
    """A conv the fused head cannot serve (64 couts) is refused with an error, never silently run."""
    x = torch.randn(1, 64, 8, 64, device=DEV)
    w = torch.randn(64, 64, 3, 3, device=DEV)
    with pytest.raises(RuntimeError, match='conv2d_head'):
        ops.conv2d(x, w, None, padding=1, residual=torch.randn(1, 64, 8, 64, device=DEV), post_act=1,
                   compute_dtype=torch.bfloat16, head=(torch.randn(3, 64, 1, 1, device=DEV), None))


@pytest.mark.parametrize('case', [(2, 64, 6, 10, 8), (1, 64, 48, 48, 8), (3, 32, 5, 7, 4), (1, 128, 4, 9, 8)])
def test_conv1x1_pixelshuffle(ops, case):
    """PixelShuffle upsampler (1x1 conv + ReLU + shuffle, upsampling.py:51-66): the dedicated bf16 kernel
    (dbsr_conv_kernel_for == 3) against torch on the same bf16-rounded operands and against the generic
    kernel's shuffle epilogue (algo 0).  The dedicated kernel starts its accumulators at the bias (the order
    dbsr_conv_shuffle_blur shares), the generic kernel adds the bias after the K sum: one fp32 rounding apart,
    so at most one bf16 rounding step (rtol 2^-7)."""
    from dbsr_amd import _lib
    N, Cin, H, W, s = case
    Cout = 32 * s * s
    gen = torch.Generator().manual_seed(Cin + H * W + s)
    x = torch.randn(N, Cin, H, W, generator=gen)
    w = torch.randn(Cout, Cin, 1, 1, generator=gen) / Cin ** 0.5
    b = torch.randn(Cout, generator=gen) * 0.1
    xb, wb = x.to(torch.bfloat16).float(), w.to(torch.bfloat16).float()
    ref = F.pixel_shuffle(F.relu(F.conv2d(xb, wb, b)), s)
    outs = {}
    try:
        for algo in (2, 0):
            _lib.lib().dbsr_set_conv_algo(algo)
            outs[algo] = ops.conv2d(x.to(DEV), w.to(DEV), b.to(DEV), act=1, compute_dtype=torch.bfloat16,
                                    shuffle=s).float().cpu()
    finally:
        _lib.lib().dbsr_set_conv_algo(2)
    assert outs[2].shape == ref.shape
    np.testing.assert_allclose(outs[2].numpy(), ref.numpy(), atol=2e-2, rtol=1e-2)
    np.testing.assert_allclose(outs[2].numpy(), outs[0].numpy(), rtol=2.0 ** -7, atol=1e-6)


@pytest.mark.parametrize('case', [(2, 512, 64, 48, 48, torch.bfloat16, 1, True),    # merge projection shape
                                  (3, 512, 64, 37, 41, torch.float16, 1, True),     # ragged pixel count
                                  (5, 128, 32, 29, 33, torch.bfloat16, 0, False),   # 32 couts, no bias/act
                                  (1, 256, 64, 64, 64, torch.bfloat16, 1, True)])
def test_conv1x1_pointwise(ops, case):
    """Pointwise projection kernel (merging.py:34 feat_project_layer, dbsr_conv_kernel_for == 5) against
    torch on the same 16-bit operands and against the generic kernel (algo 0)."""
    from dbsr_amd import _lib
    N, Cin, Cout, H, W, dt, act, with_bias = case
    gen = torch.Generator().manual_seed(Cin + Cout + H * W)
    x = torch.randn(N, Cin, H, W, generator=gen)
    w = torch.randn(Cout, Cin, 1, 1, generator=gen) / Cin ** 0.5
    b = torch.randn(Cout, generator=gen) * 0.1 if with_bias else None
    xb, wb = x.to(dt).float(), w.to(dt).float()
    ref = F.conv2d(xb, wb, b)
    if act:
        ref = F.relu(ref)
    outs = {}
    try:
        for algo in (2, 0):
            _lib.lib().dbsr_set_conv_algo(algo)
            outs[algo] = ops.conv2d(x.to(DEV), w.to(DEV), b.to(DEV) if b is not None else None, act=act,
                                    compute_dtype=dt).float().cpu()
            if algo == 2:
                assert ops.conv2d.last_kernel == 5
    finally:
        _lib.lib().dbsr_set_conv_algo(2)
    np.testing.assert_allclose(outs[2].numpy(), ref.numpy(), atol=2e-2, rtol=1e-2)
    np.testing.assert_allclose(outs[2].numpy(), outs[0].numpy(), atol=1e-2, rtol=8e-3)


@pytest.mark.parametrize('dt', [torch.bfloat16, torch.float16])
@pytest.mark.parametrize('case', [(3, 565, 16, 16, 2, 1, False),    # PWC level-2 flow head (pwcnet.py:156)
                                  (2, 256, 16, 16, 2, 1, True),     # the smallest K served (4 chunks), residual
                                  (2, 400, 13, 11, 3, 1, True),     # ragged tiles, residual, 32-channel tail chunk
                                  (1, 272, 9, 20, 4, 1, False),     # two 16-pixel tiles across, the last partial
                                  (2, 1000, 5, 7, 1, 1, False)])    # 16 chunks, one output channel
def test_conv3x3_narrow(ops, dt, case):
    """Narrow-output 3x3 kernel (dbsr_conv_kernel_for == 6, cout <= 4, cin >= 256) against torch fp32 on the same
    16-bit operands (fp32 output, as the flow heads write it) and against the generic kernel (algo 0)."""
    from dbsr_amd import _lib
    N, Cin, H, W, Cout, d, with_res = case
    gen = torch.Generator().manual_seed(Cin * 10 + Cout + H)
    x = torch.randn(N, Cin, H, W, generator=gen)
    w = torch.randn(Cout, Cin, 3, 3, generator=gen) / (Cin * 9) ** 0.5
    b = torch.randn(Cout, generator=gen) * 0.1
    res = torch.randn(N, Cout, H, W, generator=gen) if with_res else None
    ref = F.conv2d(x.to(dt).float(), w.to(dt).float(), b, padding=d, dilation=d)
    if with_res:
        ref = ref + res
    outs = {}
    try:
        for algo in (2, 0):
            _lib.lib().dbsr_set_conv_algo(algo)
            outs[algo] = ops.conv2d(x.to(DEV), w.to(DEV), b.to(DEV), padding=d, dilation=d, compute_dtype=dt,
                                    out_f32=True, residual=res.to(DEV) if with_res else None).cpu()
            assert ops.conv2d.last_kernel == (6 if algo == 2 else 0)
    finally:
        _lib.lib().dbsr_set_conv_algo(2)
    np.testing.assert_allclose(outs[2].numpy(), ref.numpy(), atol=1e-4, rtol=1e-4)
    np.testing.assert_allclose(outs[2].numpy(), outs[0].numpy(), atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize('dt', [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize('shape', [(2, 32, 384, 384), (1, 16, 13, 21), (3, 8, 9, 4)])
def test_gauss_blur3(shape, dt):
    """Sliding-window 3x3 Gaussian (upsampling.py:59-65, filtering.py:29-40) against the oracle's blur
    (16-bit: on the rounded input, fp32 sums, one rounding of the output).  The 16-bit kernel sums the separable
    pair (blur_row / blur_col) where torch sums the 9 taps: the fp32 sums differ by roundings, which can move the
    16-bit output by one rounding step (rtol 2 ulps of the dtype)."""
    from dbsr_amd import _lib as L
    N, C, H, W = shape
    x = torch.randn(N, C, H, W, generator=torch.Generator().manual_seed(H + W + C)).to(dt).float()
    kern = orc.gauss_kernel(3, 1.0).reshape(3, 3).float()
    ref = F.conv2d(x, kern.expand(C, 1, 3, 3).contiguous(), padding=1, groups=C)
    if dt != torch.float32:
        ref = ref.to(dt).float()
    xs = x.permute(0, 2, 3, 1).contiguous().to(dt).to(DEV)
    out = torch.zeros_like(xs)
    import ctypes
    kb = (ctypes.c_float * 9)(*kern.flatten().tolist())
    L.check(L.lib().dbsr_gauss_blur3(N, H, W, C, L.tensor_desc(xs, C), kb, L.tensor_desc(out, C),
                                     L.stream_ptr(xs.device)), 'blur')
    tol = 1e-5 if dt == torch.float32 else (2 ** -7 if dt == torch.bfloat16 else 2 ** -10)
    np.testing.assert_allclose(out.permute(0, 3, 1, 2).float().cpu().numpy(), ref.numpy(), atol=1e-5, rtol=tol)
