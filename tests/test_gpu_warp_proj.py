"""dbsr_warp_project (the DBSR warp fused with the feature projection of the warped frames, encoders.py:80 then
merging.py:34-36,75) against dbsr_warp_bilinear + torch's 1x1 conv on the same 16-bit operands.

Tolerances.  The warped frames are the same arithmetic as dbsr_warp_bilinear: bitwise.  The projection sums the 512
products of the stored 16-bit warped values and 16-bit weights in fp32 (MFMA order) and rounds ReLU(sum + b) once to
the dtype; torch sums the same products in fp32 in its own order: atol 1e-3 + 2 ulps of the dtype."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

DEV = 'cuda'
pytestmark = pytest.mark.gpu


def _run(P, H, W, dt, pcout, seed, mapped=False, bias=True):
    """mapped: the engine's layout -- the features of frames 1..N-1 of bursts of N = 3 read through the frame map
    (N-1, N, 1, 1) from an embedding buffer holding every frame, the projections written into channels [0, pcout)
    of a wider weight-predictor input buffer through the same map."""
    from dbsr_amd import _lib as L
    from dbsr_amd.engine import NHWC, PackedConv
    gen = torch.Generator().manual_seed(seed)
    C = 512
    dev = torch.device(DEV)
    s = torch.cuda.current_stream().cuda_stream
    N = 3
    B = (P + N - 2) // (N - 1) if mapped else 0
    nimg = B * N if mapped else P
    E = NHWC(nimg, H, W, C, dt, dev)
    E.t.copy_(torch.randn(nimg, H, W, C, generator=gen).to(dt))
    flow = (torch.randn(P, 2, H, W, generator=gen) * 3.0).to(dev)
    flow[0, :, :2, :2] = 0.0                       # integer taps
    flow[-1, 0, -1, :] = 40.0                      # past the border: all taps outside
    conv = torch.nn.Conv2d(C, pcout, 1, bias=bias)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(pcout, C, 1, 1, generator=gen) * (2.0 / C ** 0.5))
        if bias:
            conv.bias.copy_(torch.randn(pcout, generator=gen) * 0.1)
    pc = PackedConv(conv.to(dev), dt, dev, s)
    fmap = (N - 1, N, 1, 1) if mapped else (1, 1, 0, 1)
    Wf0, Wf1 = NHWC(P, H, W, C, dt, dev), NHWC(P, H, W, C, dt, dev)
    ld = pcout + 64 if mapped else pcout
    Y = NHWC(nimg, H, W, ld, dt, dev)
    L.check(L.lib().dbsr_warp_bilinear(P, H, W, C, E.d(0, fmap), flow.data_ptr(), 2 * H * W, Wf0.d(0), s), 'warp')
    L.check(L.lib().dbsr_warp_project(P, H, W, C, E.d(0, fmap), flow.data_ptr(), 2 * H * W, Wf1.d(0), pc.w.data_ptr(),
                                      pc.bias.data_ptr() if bias else None, pcout, Y.d(0, fmap), s), 'warp_project')
    torch.cuda.synchronize()
    assert torch.equal(Wf0.t, Wf1.t)
    x = Wf0.t.float().permute(0, 3, 1, 2)
    wq = conv.weight.detach().to(dev).to(dt).float()
    ref = F.relu(F.conv2d(x, wq, conv.bias.detach().to(dev) if bias else None)).permute(0, 2, 3, 1)
    if mapped:
        idx = torch.tensor([(f // (N - 1)) * N + 1 + f % (N - 1) for f in range(P)], device=dev)
        got = Y.t[idx, :, :, :pcout].float()
        others = torch.ones(nimg, dtype=torch.bool, device=dev)
        others[idx] = False
        assert Y.t[others].abs().max() == 0 and Y.t[..., pcout:].abs().max() == 0   # nothing outside the map
    else:
        got = Y.t.float()
    eps = 2.0 ** -8 if dt == torch.bfloat16 else 2.0 ** -11
    np.testing.assert_allclose(got.cpu().numpy(), ref.cpu().numpy(), atol=1e-3, rtol=2 * eps)
    return got


@pytest.mark.parametrize('case', [(5, 16, 24, torch.float16, 64), (5, 16, 24, torch.bfloat16, 64),
                                  (3, 7, 9, torch.float16, 32),          # 189 pixels: a partial last tile
                                  (13, 48, 48, torch.float16, 64),       # one burst of the bench shape
                                  (4, 8, 8, torch.bfloat16, 48)])
def test_warp_project_vs_warp_and_conv(case):
    P, H, W, dt, pcout = case
    _run(P, H, W, dt, pcout, seed=P * 100 + H)


@pytest.mark.parametrize('dt', [torch.float16, torch.bfloat16])
def test_warp_project_frame_maps(dt):
    _run(6, 12, 20, dt, 64, seed=5, mapped=True)
    _run(5, 9, 11, dt, 32, seed=6, mapped=True, bias=False)


def test_warp_project_rejects():
    from dbsr_amd import _lib as L
    nt = L.Tensor(1, L.DBSR_F16, 64 * 512, 512, 0, L.FrameMap(1, 1, 0, 1))
    f32 = L.Tensor(1, L.DBSR_F32, 64 * 512, 512, 0, L.FrameMap(1, 1, 0, 1))
    lib = L.lib()
    assert lib.dbsr_warp_project(1, 8, 8, 256, nt, 1, 128, nt, 1, None, 64, nt, None) == -1      # c != 512
    assert lib.dbsr_warp_project(1, 8, 8, 512, f32, 1, 128, f32, 1, None, 64, f32, None) == -1   # fp32
    assert lib.dbsr_warp_project(1, 8, 8, 512, nt, 1, 128, nt, 1, None, 80, nt, None) == -1      # proj_cout
    assert lib.dbsr_warp_project(1, 8, 8, 512, nt, 1, 128, nt, None, None, 64, nt, None) == -1   # no weights


@pytest.mark.parametrize('dt', [torch.float16, torch.bfloat16])
def test_engine_fused_warp_proj_matches_unfused(synth_sd, dt):
    """The whole 16-bit forward with DBSREngine.FUSED_WARP_PROJ on and off, B=2 N=14 48x48: offsets bitwise (the
    flow is upstream), the fusion weights and the prediction within the bench-shape parity bounds (the projection's
    K order differs from the 1x1 conv kernel's)."""
    import dbsr_amd
    from dbsr_amd.burst import synthetic_bursts
    from dbsr_amd.engine import DBSREngine
    burst, _ = synthetic_bursts(2, 14, 48, 48, sr_factor=8, seed=78)
    burst = burst.to(DEV)
    outs = {}
    old = DBSREngine.FUSED_WARP_PROJ
    try:
        for flag in (True, False):
            DBSREngine.FUSED_WARP_PROJ = flag
            net = dbsr_amd.dbsrnet_cvpr2021(**dbsr_amd.DBSR_SYNTHETIC_KWARGS)
            net.load_state_dict(synth_sd)
            net = net.to(DEV).eval().set_compute_dtype(dt)
            with torch.no_grad():
                pred, aux = net(burst)
            names = [name for _, _, name, _ in net._engine.plans[(2, 14, 48, 48)].ops]
            assert ('warp+proj' in names) == flag and ('merge.proj_oth' in names) == (not flag), names
            outs[flag] = (pred.float().cpu(), aux['offsets'].cpu(), aux['fusion_weights'].float().cpu())
    finally:
        DBSREngine.FUSED_WARP_PROJ = old
    (p1, o1, w1), (p0, o0, w0) = outs[True], outs[False]
    assert torch.equal(o1, o0)
    dq = ((p1 - p0).abs() * 2 ** 14).flatten()
    assert torch.quantile(dq[:2 ** 24].float(), 0.999) <= 320 and dq.max() <= 800, (dq.max().item(),)
    np.testing.assert_allclose(w1.numpy(), w0.numpy(), atol=2e-3, rtol=5e-2 if dt == torch.bfloat16 else 1e-2)
