"""torch.ops.dbsr.* on the GPU: each operator against the oracle / torch on the same inputs, and its
registered autograd formula against torch autograd of the oracle's restatement (correlation K3/K4,
warp, fusion)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import dbsr_oracle as orc

pytestmark = pytest.mark.gpu
DEV = 'cuda'


@pytest.fixture(scope='module')
def dbsr():
    from dbsr_amd import torch_ops
    return torch_ops.load()


def _rel(a, b):
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-12))


@pytest.mark.parametrize('shape', [(2, 32, 16, 16), (3, 196, 1, 1), (1, 20, 5, 7)])
@pytest.mark.parametrize('leaky', [False, True])
def test_correlation_op_and_grad(dbsr, shape, leaky):
    gen = torch.Generator().manual_seed(shape[1] + leaky)
    a = torch.randn(*shape, generator=gen, requires_grad=True)
    b = torch.randn(*shape, generator=gen, requires_grad=True)
    ref = orc.correlation(a, b)
    if leaky:
        ref = F.leaky_relu(ref, 0.1)
    g = torch.randn(ref.shape, generator=gen)
    ref.backward(g)
    ad, bd = a.detach().to(DEV).requires_grad_(), b.detach().to(DEV).requires_grad_()
    out = dbsr.correlation(ad, bd, leaky)
    out.backward(g.to(DEV))
    np.testing.assert_allclose(out.detach().cpu().numpy(), ref.detach().numpy(), atol=1e-5, rtol=1e-5)
    assert _rel(ad.grad.cpu(), a.grad) <= 1e-5
    assert _rel(bd.grad.cpu(), b.grad) <= 1e-5


def test_warp_op_and_grad(dbsr):
    gen = torch.Generator().manual_seed(9)
    x = torch.randn(2, 24, 10, 14, generator=gen, requires_grad=True)
    fl = torch.randn(2, 2, 10, 14, generator=gen) * 2.5
    y = orc.warp(x, fl)
    g = torch.randn(y.shape, generator=gen)
    y.backward(g)
    xd = x.detach().to(DEV).requires_grad_()
    yd = dbsr.warp_bilinear(xd, fl.to(DEV))
    yd.backward(g.to(DEV))
    assert _rel(yd.detach().cpu(), y.detach()) <= 1e-5
    assert _rel(xd.grad.cpu(), x.grad) <= 1e-5


@pytest.mark.parametrize('N', [4, 20])        # 20: beyond the register-resident kernels (any burst size)
def test_fuse_softmax_op_and_grad(dbsr, N):
    gen = torch.Generator().manual_seed(10 + N)
    B, C, H, W = 2, 32, 5, 6
    lg = torch.randn(B, N, C, H, W, generator=gen, requires_grad=True)
    f = torch.randn(B, N, C, H, W, generator=gen, requires_grad=True)
    w = F.softmax(lg, dim=1)
    fused = (f * w).sum(dim=1)
    g = torch.randn(fused.shape, generator=gen)
    fused.backward(g)
    lgd, fd = lg.detach().to(DEV).requires_grad_(), f.detach().to(DEV).requires_grad_()
    fu, wd = dbsr.fuse_softmax(lgd, fd, True)
    fu.backward(g.to(DEV))
    assert _rel(fu.detach().cpu(), fused.detach()) <= 1e-5
    assert _rel(wd.detach().cpu(), w.detach()) <= 1e-5
    assert _rel(lgd.grad.cpu(), lg.grad) <= 1e-5
    assert _rel(fd.grad.cpu(), f.grad) <= 1e-5


def test_backwarp_op(dbsr, golden):
    g = golden('ops')
    x = torch.from_numpy(g['bw8_x']).to(DEV)
    fl = torch.from_numpy(g['bw8_flow']).to(DEV) * float(g['bw8_scale'])
    np.testing.assert_allclose(dbsr.backwarp(x, fl).cpu().numpy(), g['bw8_out'], atol=1e-5, rtol=0)


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16, torch.float16])
def test_conv2d_fused_op(dbsr, dtype):
    """conv + bias + ReLU + residual + ReLU (ResBlock conv2 shape, blocks.py:94-96); the packed weights are
    cached per (storage, version) and repacked after an in-place update."""
    gen = torch.Generator().manual_seed(12)
    x = torch.randn(2, 64, 16, 24, generator=gen)
    w = torch.randn(64, 64, 3, 3, generator=gen) / 24.0
    b = torch.randn(64, generator=gen) * 0.1
    r = torch.randn(2, 64, 16, 24, generator=gen)
    xr, wr, rr = (t.to(dtype).float() for t in (x, w, r))
    ref = F.relu(F.relu(F.conv2d(xr, wr, b, padding=1)) + rr)
    wd = w.to(DEV)
    out = dbsr.conv2d_fused(x.to(DEV).to(dtype), wd, b.to(DEV), 1, 1, 1, 1, r.to(DEV).to(dtype), 1).float().cpu()
    tol = 1e-4 if dtype == torch.float32 else 2e-2
    assert _rel(out, ref) <= tol
    with torch.no_grad():
        wd.mul_(0.5)                                     # in-place update -> new version -> repack
    out2 = dbsr.conv2d_fused(x.to(DEV).to(dtype), wd, b.to(DEV), 1, 1, 1, 1, r.to(DEV).to(dtype), 1).float().cpu()
    ref2 = F.relu(F.relu(F.conv2d(xr, (w * 0.5).to(dtype).float(), b, padding=1)) + rr)
    assert _rel(out2, ref2) <= tol


def test_conv2d_fused_cache_bias_and_address_reuse(dbsr):
    """the packed-weight cache must not serve (a) a bias-less packing to a call with a bias,
    (b) one weight's packing to another weight that reuses its address, (c) stale entries of freed weights."""
    gen = torch.Generator().manual_seed(21)
    x = torch.randn(1, 32, 8, 8, generator=gen)
    b = torch.randn(16, generator=gen)
    xd = x.to(DEV)
    torch.ops.dbsr.clear_pack_cache()
    w = torch.randn(16, 32, 3, 3, generator=gen) / 17.0
    wd = w.to(DEV)
    o0 = dbsr.conv2d_fused(xd, wd, None, 1, 1, 1, 0, None, 0).cpu()
    o1 = dbsr.conv2d_fused(xd, wd, b.to(DEV), 1, 1, 1, 0, None, 0).cpu()
    assert _rel(o0, F.conv2d(x, w, None, padding=1)) <= 1e-4
    assert _rel(o1, F.conv2d(x, w, b, padding=1)) <= 1e-4
    b2 = b.to(DEV)
    o2 = dbsr.conv2d_fused(xd, wd, b2, 1, 1, 1, 0, None, 0).cpu()
    with torch.no_grad():
        b2.add_(1.0)                                     # bias update -> repack
    o3 = dbsr.conv2d_fused(xd, wd, b2, 1, 1, 1, 0, None, 0).cpu()
    assert _rel(o2, F.conv2d(x, w, b, padding=1)) <= 1e-4
    assert _rel(o3, F.conv2d(x, w, b + 1.0, padding=1)) <= 1e-4
    # fresh weights allocated in a loop reuse the caching allocator's address, all at version 0
    ptrs = set()
    for i in range(4):
        cout = 16 if i % 2 == 0 else 24
        wi = torch.randn(cout, 32, 3, 3, generator=gen) / 17.0
        wdi = wi.to(DEV)
        ptrs.add(wdi.data_ptr())
        oi = dbsr.conv2d_fused(xd, wdi, None, 1, 1, 1, 0, None, 0).cpu()
        assert oi.shape[1] == cout
        assert _rel(oi, F.conv2d(x, wi, None, padding=1)) <= 1e-4, i
        del wdi
    assert torch.ops.dbsr.pack_cache_size() <= 2         # freed weights' entries are evicted
