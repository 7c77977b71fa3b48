"""The K-split weight-stationary 128 -> 128 3x3 kernel (csrc/conv128.hip, dbsr_conv2d's kernel 7: the weight
predictor's input conv and ResBlocks, merging.py:86-90, 98-101) against torch fp32 on the same 16-bit-rounded
operands and against the pipelined kernel it replaces (dbsr_set_conv_algo(5)), for every compiled epilogue, both
16-bit dtypes, full and partial rounds of the persistent grid, and frames whose tiles touch every border."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = 'cuda'

# (N, H, W): tiles of 16 x 8 = N * H/8 * W/16
SHAPES = [
    (8, 48, 48),     # 144 tiles: one partial round (the decoder-side batch)
    (16, 32, 64),    # 256 tiles: exactly one XCD-ordered round
    (20, 48, 48),    # 360 tiles: one full round + a partial one
    (13, 16, 176),   # 286 tiles, wide frames
]
# (act, residual, post_act): epilogues 1 (ResBlock conv1), 2 (conv2 / wp.init), 3 (plain), 0 (leaky, run time)
EPIS = [(1, False, 0), (0, True, 1), (0, False, 0), (2, True, 2)]


def _ref(x, w, b, res, act, post):
    def a(v, k):
        return F.relu(v) if k == 1 else F.leaky_relu(v, 0.1) if k == 2 else v
    y = a(F.conv2d(x, w, b, padding=1), act)
    return a(y + res, post) if res is not None else y


@pytest.mark.parametrize('dt', [torch.float16, torch.bfloat16])
@pytest.mark.parametrize('shape', SHAPES)
@pytest.mark.parametrize('epi', EPIS)
def test_ks128_vs_torch_and_pipe(dt, shape, epi):
    from dbsr_amd import _lib, ops
    N, H, W = shape
    act, use_res, post = epi
    gen = torch.Generator().manual_seed(N * 1000 + H + W + act * 7 + post)
    x = torch.randn(N, 128, H, W, generator=gen)
    w = torch.randn(128, 128, 3, 3, generator=gen) / (128 * 9) ** 0.5
    b = torch.randn(128, generator=gen) * 0.1
    res = torch.randn(N, 128, H, W, generator=gen) if use_res else None
    xr, wr = x.to(dt).float(), w.to(dt).float()
    rr = res.to(dt).float() if use_res else None
    ref = _ref(xr, wr, b, rr, act, post)
    outs = {}
    try:
        for algo in (2, 5):
            _lib.lib().dbsr_set_conv_algo(algo)
            outs[algo] = ops.conv2d(x.to(DEV), w.to(DEV), b.to(DEV), padding=1, act=act,
                                    residual=res.to(DEV) if use_res else None, post_act=post,
                                    compute_dtype=dt).float().cpu()
            if algo == 2:
                assert ops.conv2d.last_kernel == 7 and ops.conv2d.last_variant == 7001608
            else:
                assert ops.conv2d.last_kernel != 7
    finally:
        _lib.lib().dbsr_set_conv_algo(2)
    ulp = 2.0 ** (-10 if dt == torch.float16 else -7)
    # one rounding of the fp32 sum to 16 bits (+ one of the pre-residual value), fp32 accumulation both ways
    np.testing.assert_allclose(outs[2].numpy(), ref.numpy(), atol=4 * ulp, rtol=2 * ulp)
    np.testing.assert_allclose(outs[2].numpy(), outs[5].numpy(), atol=4 * ulp, rtol=2 * ulp)
    assert (outs[2] - ref).abs().mean() < 0.25 * ulp
    # the two kernels differ only by the fp32 summation order: most elements are bitwise equal (the rest by an ulp
    # where the order moved the fp32 sum across a 16-bit rounding boundary: 14.5 % with fp16 + residual, r06k)
    assert (outs[2] == outs[5]).float().mean() > 0.7


@pytest.mark.parametrize('dt', [torch.float16, torch.bfloat16])
@pytest.mark.parametrize('use_res', [False, True])
def test_ks128_gated_dgrad_epilogue(dt, use_res):
    """Epilogue 5, the training step's gated dgrads of the weight predictor's ResBlocks (training.py res_bwd):
    dX = conv_input_grad(dY) [+ residual], times (gate > 0), no bias, at the training shape's frame size."""
    from dbsr_amd import _lib, ops
    N, H, W = 3, 128, 128
    gen = torch.Generator().manual_seed(11 + use_res)
    dy = torch.randn(N, 128, H, W, generator=gen)
    w = torch.randn(128, 128, 3, 3, generator=gen) / (128 * 9) ** 0.5
    res = torch.randn(N, 128, H, W, generator=gen) if use_res else None
    gate = torch.randn(N, 128, H, W, generator=gen)
    dyr, wr, gr = dy.to(dt).float(), w.to(dt).float(), gate.to(dt).float()
    ref = torch.nn.grad.conv2d_input((N, 128, H, W), wr, dyr, padding=1)
    if use_res:
        ref = ref + res.to(dt).float()
    ref = ref * (gr > 0)
    outs = {}
    try:
        for algo in (2, 5):
            _lib.lib().dbsr_set_conv_algo(algo)
            outs[algo] = ops.conv2d_dgrad(dy.to(DEV), w.to(DEV), residual=res.to(DEV) if use_res else None,
                                          gate=gate.to(DEV), compute_dtype=dt).float().cpu()
            assert (ops.conv2d_dgrad.last_kernel == 7) == (algo == 2)
    finally:
        _lib.lib().dbsr_set_conv_algo(2)
    ulp = 2.0 ** (-10 if dt == torch.float16 else -7)
    np.testing.assert_allclose(outs[2].numpy(), ref.numpy(), atol=4 * ulp, rtol=2 * ulp)
    np.testing.assert_allclose(outs[2].numpy(), outs[5].numpy(), atol=4 * ulp, rtol=2 * ulp)
    assert ((outs[2] == 0) | (gr > 0)).all()


def test_ks128_not_picked_off_shape():
    """Shapes outside the kernel's contract go elsewhere: cout != 128, a frame width not a multiple of 16, too
    few tiles, cin 64."""
    from dbsr_amd import ops
    for (N, cin, H, W, cout) in [(16, 128, 32, 64, 96), (16, 128, 32, 56, 128), (2, 128, 48, 48, 128),
                                 (16, 64, 32, 64, 128)]:
        x = torch.randn(N, cin, H, W, device=DEV)
        w = torch.randn(cout, cin, 3, 3, device=DEV) / 34.0
        ops.conv2d(x, w, None, padding=1, compute_dtype=torch.float16)
        assert ops.conv2d.last_kernel != 7, (N, cin, H, W, cout)


# (N, Cin, H, W, Cout, expected K split): the LDS-tiled kernel's split-K (conv2d.hip tiled_ksplit) -- the decoder's
# first conv (512 -> 64, 8 frames of 48x48), a partial cout tile (96 couts) with a ragged frame, and a cout < 64
# conv (PWC-Net's last level-2 DenseNet conv, 533 -> 32) that stays unsplit
TILED_SPLIT = [(8, 512, 48, 48, 64, 8), (3, 320, 20, 17, 96, 5), (104, 533, 16, 16, 32, 0)]


@pytest.mark.parametrize('dt', [torch.float16, torch.bfloat16])
@pytest.mark.parametrize('case', TILED_SPLIT)
def test_tiled_split_k(dt, case):
    """Split-K LDS-tiled 3x3 (fp32 slice partials + in-order finalize) against torch fp32 on the same 16-bit
    operands, with bias + ReLU and with the residual / post-ReLU epilogue; the dispatch variant names the split."""
    from dbsr_amd import ops
    N, Cin, H, W, Cout, sp = case
    gen = torch.Generator().manual_seed(Cin + Cout + H)
    x = torch.randn(N, Cin, H, W, generator=gen)
    w = torch.randn(Cout, Cin, 3, 3, generator=gen) / (Cin * 9) ** 0.5
    b = torch.randn(Cout, generator=gen) * 0.1
    res = torch.randn(N, Cout, H, W, generator=gen)
    xr, wr, rr = x.to(dt).float(), w.to(dt).float(), res.to(dt).float()
    ulp = 2.0 ** (-10 if dt == torch.float16 else -7)
    for use_res in (False, True):
        ref = F.conv2d(xr, wr, b, padding=1)
        ref = F.relu(ref + rr) if use_res else F.relu(ref)
        out = ops.conv2d(x.to(DEV), w.to(DEV), b.to(DEV), padding=1, act=0 if use_res else 1,
                         residual=res.to(DEV) if use_res else None, post_act=1 if use_res else 0,
                         compute_dtype=dt).float().cpu()
        assert ops.conv2d.last_kernel == 1 and ops.conv2d.last_variant % 1000000 // 100000 == sp, ops.conv2d.last_variant
        np.testing.assert_allclose(out.numpy(), ref.numpy(), atol=4 * ulp, rtol=2 * ulp)
        assert (out - ref).abs().mean() < 0.25 * ulp


# (N, Cin, H, W, Cout): the small-input 3x3 kernel (conv2d.hip conv3x3_small_kernel, kernel_for 8) -- the encoder's
# first conv (4 raw channels -> 64), the offset-feature extractor's (2 offset channels -> 64), a ragged frame width
# and a 16-cout conv
SMALL = [(14, 4, 48, 48, 64), (13, 2, 48, 48, 64), (3, 8, 20, 37, 32), (2, 3, 16, 16, 16)]


@pytest.mark.parametrize('dt', [torch.float16, torch.bfloat16])
@pytest.mark.parametrize('case', SMALL)
def test_small_input_conv(dt, case):
    """conv3x3_small_kernel against torch fp32 on the same 16-bit operands (bias + ReLU, and no activation)."""
    from dbsr_amd import ops
    N, Cin, H, W, Cout = case
    gen = torch.Generator().manual_seed(Cin * 13 + Cout + W)
    x = torch.randn(N, Cin, H, W, generator=gen)
    w = torch.randn(Cout, Cin, 3, 3, generator=gen) / (Cin * 9) ** 0.5
    b = torch.randn(Cout, generator=gen) * 0.1
    xr, wr = x.to(dt).float(), w.to(dt).float()
    ulp = 2.0 ** (-10 if dt == torch.float16 else -7)
    for act in (1, 0):
        ref = F.conv2d(xr, wr, b, padding=1)
        if act:
            ref = F.relu(ref)
        out = ops.conv2d(x.to(DEV), w.to(DEV), b.to(DEV), padding=1, act=act, compute_dtype=dt).float().cpu()
        assert ops.conv2d.last_kernel == 8
        np.testing.assert_allclose(out.numpy(), ref.numpy(), atol=4 * ulp, rtol=2 * ulp)
