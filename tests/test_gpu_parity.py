"""Parity at the benchmarked workloads (BASELINE.json configs[1], configs[2]) against the oracle run
in-test on the same seeded bursts, and element-wise checks of the pipelined conv kernel's compile-time
epilogues (the variants the bench-shape forward dispatches).

Tolerances (north_star: fp32 <= 1e-3 max-abs; 16-bit: PSNR within 0.01 dB of the reference):
  * the precision bar at the reference's operating point: the published SyntheticBurst
    PSNR is 39.17 dB (README.md:250,255), MSE 1.211e-4; moving it by 0.01 dB takes dMSE = 2.79e-7, i.e. an
    RMS prediction error of RMS_BAR = 5.3e-4 (for an error uncorrelated with the residual).  Gate: the RMS
    of (pred - pred_oracle) on the predictions the metric scores (clamped to [0,1], compute_score.py:110-111)
    <= RMS_BAR at the bench workload in the bench's dtype (fp16); the unclamped RMS and the fusion-weight
    errors are reported beside it.  bf16 storage misses the bar (~2.9e-3) and is held only to the loose
    bounds below (it is a supported mode, not the bench's).
  * configs[1] (B=8): per-burst |PSNR - PSNR_ref| <= 0.01 dB against the synthetic ground truth
    with compute_score's 2^14 quantisation and boundary_ignore=40; offsets max-abs <= OFFS_TOL px
    (bf16 PWC-Net features, fp32 flow accumulation); quantised pred: 99.9 % of values within
    PRED_Q_TOL quanta of the oracle's and none beyond PRED_Q_MAX (bf16 activations through ~70 convs
    with seeded random weights; measured on MI355X: p99.9 234, max 463 quanta, PSNR delta 0.0047 dB,
    offsets 0.013 px).
  * configs[2] (fp32, B=4, 80x80): pred and offsets max-abs <= 1e-3.
"""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = 'cuda'
OFFS_TOL = 0.05
PRED_Q_TOL = 320          # 320 of 2^14 quanta = 0.0195 in [0, 1]
PRED_Q_MAX = 800          # 0.049
RMS_BAR = 5.3e-4          # see the module docstring


def _net(synth_sd, dtype):
    import dbsr_amd
    net = dbsr_amd.dbsrnet_cvpr2021(**dbsr_amd.DBSR_SYNTHETIC_KWARGS)
    net.load_state_dict(synth_sd)
    return net.to(DEV).eval().set_compute_dtype(dtype)


def _psnr_q(pred, gt, bi=40):
    """compute_score.py:110-115 quantisation + PSNR(boundary_ignore=40) (image_quality_v2.py:69-101)."""
    q = (pred.clamp(0.0, 1.0) * 2 ** 14).short().float() / 2 ** 14
    return [float(10 * torch.log10(1.0 / ((p - g_)[..., bi:-bi, bi:-bi] ** 2).mean())) for p, g_ in zip(q, gt)]


@pytest.fixture(scope='module')
def bench_case(synth_sd):
    """configs[1] inputs and the oracle's fp32 forward of them (computed once per module)."""
    from dbsr_amd.burst import synthetic_bursts
    from oracle import dbsr_oracle as orc
    burst, gt = synthetic_bursts(8, 14, 48, 48, sr_factor=8, seed=101)
    with torch.no_grad():
        ref, raux = orc.dbsr_forward(burst, synth_sd)
    return burst, gt, ref, raux['offsets'], raux['fusion_weights']


def precision_report(pred, ref, fw=None, rfw=None):
    """RMS / max errors of a prediction against the oracle's, and of the fusion weights."""
    pred = pred.float().cpu()
    d = pred - ref
    dc = pred.clamp(0, 1) - ref.clamp(0, 1)
    rep = {'rms': float(d.pow(2).mean().sqrt()), 'rms_clamped': float(dc.pow(2).mean().sqrt()),
           'max': float(d.abs().max()), 'max_clamped': float(dc.abs().max())}
    if fw is not None:
        e = fw.float().cpu() - rfw                          # [B,N,C,H,W]
        rep.update({'fw_rms': float(e.pow(2).mean().sqrt()), 'fw_mean': float(e.mean()),
                    'fw_max_per_channel_max': float(e.abs().amax(dim=(0, 1, 3, 4)).max()),
                    'fw_max_per_channel_median': float(e.abs().amax(dim=(0, 1, 3, 4)).median())})
    return rep


def _check_bench(pred, offs, bench_case, loose=False):
    burst, gt, ref, roffs = bench_case[:4]
    pred, offs = pred.float().cpu(), offs.cpu()
    od = (offs - roffs).abs().max().item()
    q = (pred.clamp(0, 1) * 2 ** 14).short().int()
    rq = (ref.clamp(0, 1) * 2 ** 14).short().int()
    qd = (q - rq).abs().float()
    mine, theirs = _psnr_q(pred, gt), _psnr_q(ref, gt)
    dpsnr = max(abs(a - b) for a, b in zip(mine, theirs))
    print('offsets max-abs %.4g  pred quanta max %d p99.9 %.1f mean %.2f  PSNR delta max %.5f dB' % (
        od, int(qd.max()), float(torch.quantile(qd.flatten()[::7], 0.999)), float(qd.mean()), dpsnr))
    assert od <= OFFS_TOL
    assert float((qd > PRED_Q_TOL).float().mean()) <= 1e-3
    assert float(qd.max()) <= PRED_Q_MAX
    if not loose:
        assert dpsnr <= 0.01


@pytest.mark.parametrize('dtype', [torch.float16, torch.bfloat16])
def test_bench_shape_vs_oracle(synth_sd, bench_case, dtype):
    """configs[1] exactly as bench.py runs it (B=8, N=14, 48x48, HIP-graph replay, default kernel dispatch)
    against the oracle.  fp16 (the bench's dtype): the RMS bar at 39.17 dB plus the PSNR-delta and element
    bounds; bf16: the element bounds only, its RMS printed (it misses the bar)."""
    net = _net(synth_sd, dtype)
    net.use_graph = True
    with torch.no_grad():
        net(bench_case[0].to(DEV))                 # capture
        pred, aux = net(bench_case[0].to(DEV))     # replay
    rep = precision_report(pred, bench_case[2], aux['fusion_weights'], bench_case[4])
    print('%s precision vs oracle: %s' % (dtype, ' '.join('%s %.3e' % kv for kv in rep.items())))
    _check_bench(pred, aux['offsets'], bench_case, loose=dtype == torch.bfloat16)
    if dtype == torch.float16:
        assert rep['rms_clamped'] <= RMS_BAR, rep
        # the margin under the bar: with the DBSR weights' error-diffusion rounding (DBSREngine.
        # WEIGHT_ROUNDING, measured 3.19e-4; round-to-nearest 4.50e-4)
        assert rep['rms_clamped'] <= 4.0e-4, rep
        assert rep['fw_rms'] <= 1e-3, rep


def test_bench_shape_two_lanes_bitwise(synth_sd, bench_case):
    """PWC-Net on a side stream beside the encoder (two lanes, eager and graph) gives bit-identical
    results to the single-stream forward at the bench shape, over repeated forwards."""
    from dbsr_amd import engine
    burst = bench_case[0].to(DEV)
    outs = {}
    old = engine.Plan.MULTI_STREAM
    try:
        for multi in (False, True):
            engine.Plan.MULTI_STREAM = multi
            net = _net(synth_sd, torch.float16)
            res = []
            with torch.no_grad():
                for use_graph in (False, False, False, True, True, True):
                    net.use_graph = use_graph
                    pred, aux = net(burst)
                    res.append((pred, aux['offsets'], aux['fusion_weights']))
            outs[multi] = res
    finally:
        engine.Plan.MULTI_STREAM = old
    ref = outs[False][0]
    for multi in (False, True):
        for i, o in enumerate(outs[multi]):
            for a, b, name in zip(o, ref, ('pred', 'offsets', 'fusion_weights')):
                assert torch.equal(a, b), (multi, i, name, (a.float() - b.float()).abs().max().item())


def test_cfg3_batch4_fp32_vs_oracle(synth_sd):
    """configs[2] at its stated batch (BurstSR real crops: B=4, 14 frames, 80x80, fp32; 1/1023 RAW
    quantisation) against the oracle: max-abs <= 1e-3 on pred and offsets."""
    from dbsr_amd.burst import synthetic_bursts
    from oracle import dbsr_oracle as orc
    burst, _ = synthetic_bursts(4, 14, 80, 80, sr_factor=8, seed=13)
    burst = (burst * 1023).round() / 1023
    net = _net(synth_sd, torch.float32)
    with torch.no_grad():
        pred, aux = net(burst.to(DEV))
        ref, raux = orc.dbsr_forward(burst, synth_sd)
    assert pred.shape == (4, 3, 640, 640)
    assert (aux['offsets'].cpu() - raux['offsets']).abs().max().item() <= 1e-3
    assert (pred.cpu() - ref).abs().max().item() <= 1e-3


# (act, residual, post_act, cin, cout): the pipelined kernel's compile-time epilogues at the widths the
# forward uses -- EPI 1 act(ReLU) no residual (encoder init-out, ResBlock conv1, wp.init),
# EPI 2 no act + residual + ReLU (ResBlock conv2), EPI 3 plain (wp.out 128 -> 512)
PIPE_EPI = [
    (1, False, 0, 64, 64), (1, False, 0, 64, 512), (1, False, 0, 192, 128),
    (0, True, 1, 64, 64), (0, True, 1, 128, 128), (0, True, 1, 32, 32),
    (0, False, 0, 128, 512), (0, False, 0, 64, 64), (1, False, 0, 32, 32),
]


# the 16x16-frame tile (PWC level 2 / refiner: 117 - 565 input channels, LeakyReLU)
PIPE16 = [(2, False, 0, 117, 128, 16), (2, False, 0, 565, 128, 16), (2, False, 0, 373, 96, 16),
          (2, False, 0, 469, 64, 16)]


# the 32x16 tile (frame widths that are multiples of 32 but not 48: the training step's 128x128 frames)
PIPE32 = [(1, False, 0, 128, 128, 32), (0, True, 1, 128, 128, 64), (0, False, 0, 128, 512, 64),
          (1, False, 0, 192, 128, 64)]


@pytest.mark.parametrize('case', PIPE_EPI + PIPE16 + PIPE32)
def test_pipe_epilogue_variants(ops_mod, case):
    from dbsr_amd import _lib
    act, use_res, post, cin, cout = case[:5]
    H, W = (case[5], case[5]) if len(case) > 5 else ((8, 96) if cout > 32 else (8, 128))
    N = 2
    gen = torch.Generator().manual_seed(cin * 13 + cout + act * 7 + post)
    x = torch.randn(N, cin, H, W, generator=gen)
    w = torch.randn(cout, cin, 3, 3, generator=gen) / (cin * 9) ** 0.5
    b = torch.randn(cout, generator=gen) * 0.1
    res = torch.randn(N, cout, H, W, generator=gen) if use_res else None
    xb, wb = x.to(torch.bfloat16).float(), w.to(torch.bfloat16).float()
    ref = F.conv2d(xb, wb, b, padding=1)
    if act == 1:
        ref = F.relu(ref)
    elif act == 2:
        ref = F.leaky_relu(ref, 0.1)
    if use_res:
        # the kernel adds the residual to the fp32 conv value and rounds once
        ref = ref + res.to(torch.bfloat16).float()
    if post:
        ref = F.relu(ref)
    outs = {}
    try:
        for algo in (3, 0):
            _lib.lib().dbsr_set_conv_algo(algo)
            outs[algo] = ops_mod.conv2d(x.to(DEV), w.to(DEV), b.to(DEV), padding=1, act=act,
                                        residual=res.to(DEV) if use_res else None, post_act=post,
                                        compute_dtype=torch.bfloat16).float().cpu()
            if algo == 3:
                assert ops_mod.conv2d.last_kernel == 2, ops_mod.conv2d.last_kernel
    finally:
        _lib.lib().dbsr_set_conv_algo(2)
    # bf16 output: one rounding of the fp32 result (2^-8 relative)
    np.testing.assert_allclose(outs[3].numpy(), ref.numpy(), atol=2e-2, rtol=1e-2)
    np.testing.assert_allclose(outs[3].numpy(), outs[0].numpy(), atol=2e-2, rtol=1e-2)
    assert (outs[3] - ref).abs().mean() < 2e-3


# (act, residual, post_act, cin, cout, dtype): the weight-stationary kernel (dbsr_conv_kernel_for == 4,
# Cin <= 64): compile-time epilogues 1/2/3, the run-time one (LeakyReLU + residual + ReLU), one-chunk
# Cin 32, a partial 64-cout tile (96: the second tile's upper wave has no couts), 512 couts (8 cout
# tiles sharing a spatial tile's halo), fp16
WS_EPI = [
    (1, False, 0, 64, 64, torch.bfloat16), (1, False, 0, 64, 512, torch.bfloat16),
    (0, True, 1, 64, 64, torch.bfloat16), (0, False, 0, 64, 64, torch.bfloat16),
    (1, False, 0, 32, 64, torch.bfloat16), (0, True, 1, 64, 96, torch.bfloat16),
    (2, True, 1, 64, 128, torch.bfloat16), (0, True, 1, 64, 64, torch.float16),
    (1, False, 0, 48, 64, torch.float16),
]


# the 32-cout variant on 64x8 tiles (the decoder's 384x384 post-ResBlocks): act, residual, post, cin, cout, dtype
WS32_EPI = [
    (1, False, 0, 32, 32, torch.bfloat16), (0, True, 1, 32, 32, torch.bfloat16), (0, False, 0, 32, 32, torch.bfloat16),
    (1, False, 0, 24, 16, torch.bfloat16), (0, True, 1, 32, 24, torch.float16), (2, True, 1, 32, 32, torch.float16),
]


@pytest.mark.parametrize('case', WS_EPI + WS32_EPI)
def test_ws_conv_variants(ops_mod, case):
    """Weight-stationary 3x3 conv against torch on the same 16-bit-rounded operands, and against the
    generic kernel; WM 64: frames 48x48 (the encoder's) and 32x16 (non-square, edge tiles on both axes),
    on 16x8 tiles where the 16x16 grid is under 128 tiles (12 and 40 frames at cin > 32) and on 16x16 tiles;
    WM 32 (cout <= 32, 64x8 tiles): 64x64 and 48x192 frames."""
    from dbsr_amd import _lib
    act, use_res, post, cin, cout, dt = case
    shapes = ((12, 48, 48), (40, 32, 16), (26, 48, 48)) if cout > 32 else ((8, 64, 64), (4, 48, 192))
    for (N, H, W) in shapes:
        gen = torch.Generator().manual_seed(cin * 13 + cout + act * 7 + post + H)
        x = torch.randn(N, cin, H, W, generator=gen)
        w = torch.randn(cout, cin, 3, 3, generator=gen) / (cin * 9) ** 0.5
        b = torch.randn(cout, generator=gen) * 0.1
        res = torch.randn(N, cout, H, W, generator=gen) if use_res else None
        xb, wb = x.to(dt).float(), w.to(dt).float()
        ref = F.conv2d(xb, wb, b, padding=1)
        if act == 1:
            ref = F.relu(ref)
        elif act == 2:
            ref = F.leaky_relu(ref, 0.1)
        if use_res:
            ref = ref + res.to(dt).float()
        if post:
            ref = F.relu(ref)
        outs = {}
        try:
            for algo in (2, 0):
                _lib.lib().dbsr_set_conv_algo(algo)
                outs[algo] = ops_mod.conv2d(x.to(DEV), w.to(DEV), b.to(DEV), padding=1, act=act,
                                            residual=res.to(DEV) if use_res else None, post_act=post,
                                            compute_dtype=dt).float().cpu()
                if algo == 2:
                    assert ops_mod.conv2d.last_kernel == 4, (N, H, W, ops_mod.conv2d.last_kernel)
        finally:
            _lib.lib().dbsr_set_conv_algo(2)
        # 16-bit output: one rounding of the fp32 result (bf16 2^-8, fp16 2^-11 relative)
        np.testing.assert_allclose(outs[2].numpy(), ref.numpy(), atol=2e-2, rtol=1e-2)
        np.testing.assert_allclose(outs[2].numpy(), outs[0].numpy(), atol=2e-2, rtol=1e-2)
        assert (outs[2] - ref).abs().mean() < 2e-3


@pytest.mark.parametrize('dt', [torch.float16, torch.bfloat16])
@pytest.mark.parametrize('epi', [(1, False, 0), (0, True, 1), (0, False, 0)])
def test_ws_tile_heights_bitwise(ops_mod, dt, epi):
    """The weight-stationary kernel's 16x8 tiles (12 frames of 48x48: a 108-tile grid) and 16x16 tiles (26
    frames: 234 tiles) give bitwise the same outputs on the same frames: the tile shape changes which pixels a
    block owns, never the order a pixel's K is summed in."""
    act, use_res, post = epi
    gen = torch.Generator().manual_seed(77 + act + 3 * post)
    x = torch.randn(26, 64, 48, 48, generator=gen)
    w = torch.randn(64, 64, 3, 3, generator=gen) / 24.0
    b = torch.randn(64, generator=gen) * 0.1
    res = torch.randn(26, 64, 48, 48, generator=gen) if use_res else None
    outs, var = {}, {}
    for n in (12, 26):
        outs[n] = ops_mod.conv2d(x[:n].to(DEV), w.to(DEV), b.to(DEV), padding=1, act=act,
                                 residual=res[:n].to(DEV) if use_res else None, post_act=post, compute_dtype=dt)
        var[n] = ops_mod.conv2d.last_variant
    assert var == {12: 4001608, 26: 4001616}, var
    assert torch.equal(outs[12], outs[26][:12])


@pytest.fixture(scope='module')
def ops_mod():
    from dbsr_amd import ops as O
    return O


@pytest.fixture(scope='module')
def cfg4_case():
    """configs[4]: SyntheticBurst 14 frames 96x96 -> x8 of full resolution (upsample_factor 16, 1536x1536
    output; SURVEY §8d's reading of '8x'), seeded weights of that architecture, and the oracle's fp32
    forward."""
    import dbsr_amd
    from dbsr_amd import arch
    from dbsr_amd.weights import generate_state_dict
    from dbsr_amd.burst import synthetic_bursts
    from oracle import dbsr_oracle as orc
    kw = dict(dbsr_amd.DBSR_SYNTHETIC_KWARGS, upsample_factor=16)
    net = dbsr_amd.dbsrnet_cvpr2021(**kw)
    sd = {k: torch.from_numpy(v) for k, v in generate_state_dict(arch.state_dict_shapes(net), seed=0).items()}
    net.load_state_dict(sd)
    burst, gt = synthetic_bursts(1, 14, 96, 96, sr_factor=16, seed=31)
    okw = dict(orc.DBSR_SYNTHETIC_KWARGS, upsample_factor=16)
    with torch.no_grad():
        ref, raux = orc.dbsr_forward(burst, sd, kw=okw)
    return net, burst, gt, ref, raux['offsets']


def _psnr_delta(pred, ref, gt):
    return max(abs(a - b) for a, b in zip(_psnr_q(pred.float().cpu(), gt), _psnr_q(ref, gt)))


def test_cfg5_fp16_x16_unsharded(cfg4_case):
    """configs[4]'s network (x16, 96x96, fp16 compute on the f16 MFMA kernels) in one piece vs the oracle."""
    net, burst, gt, ref, roffs = cfg4_case
    net = net.to(DEV).set_compute_dtype(torch.float16)
    with torch.no_grad():
        pred, aux = net(burst.to(DEV))
    assert pred.shape == (1, 3, 1536, 1536)
    od = (aux['offsets'].cpu() - roffs).abs().max().item()
    dp = _psnr_delta(pred, ref, gt)
    rep = precision_report(pred, ref)
    print('fp16 x16: offsets max-abs %.4g PSNR delta %.5f dB %s' % (od, dp, ' '.join('%s %.3e' % kv for kv in rep.items())))
    assert od <= OFFS_TOL
    assert dp <= 0.01
    assert rep['rms_clamped'] <= RMS_BAR, rep


def test_cfg5_frame_sharded_4_ranks_fp16(cfg4_case):
    """configs[4] as specified: frames split over 4 ranks (simulated on one device: each rank's
    forward_partial on its frame shard, statistics stacked as the RCCL all-gather lays them out), fp16,
    x16 upsampling, 96x96 -> the decoder split by rows (each rank its 24 LR rows + the decoder halo, as
    parallel.frame_sharded_forward runs it): the assembled prediction equals the one-rank decoder up to
    summation order and the unsharded oracle forward within the bar."""
    from dbsr_amd.parallel import frame_shard, shard_range
    net, burst, gt, ref, _ = cfg4_case
    net = net.to(DEV).set_compute_dtype(torch.float16)
    eng = net._get_engine()
    b = burst.to(DEV)
    with torch.no_grad():
        stats = []
        for r in range(4):
            frames, first = frame_shard(14, r, 4)
            st, _ = eng.forward_partial(b[:, frames], first)
            stats.append(st.clone())
        g = torch.stack(stats)
        whole = eng.combine_decode(g)
        slabs = [eng.combine_decode(g, rows=shard_range(96, r, 4)) for r in range(4)]
    pred = torch.cat(slabs, dim=2)
    assert pred.shape == (1, 3, 1536, 1536) and all(sl.shape[2] == 384 for sl in slabs)
    # every slab conv dispatches as on the whole image (dbsr_conv_desc.plan_h): the same kernel, tile and K
    # split, hence the same summation order per pixel -- the assembled rows are bitwise the unsplit decoder's
    d = (pred.float() - whole.float()).abs()
    print('row-split decoder vs whole: max %.3g mean %.3g' % (float(d.max()), float(d.mean())))
    assert float(d.max()) == 0.0
    dp = _psnr_delta(pred, ref, gt)
    rep = precision_report(pred, ref)
    print('fp16 x16 4-rank frame-sharded: PSNR delta %.5f dB %s' % (dp, ' '.join('%s %.3e' % kv for kv in rep.items())))
    assert dp <= 0.01
    assert rep['rms_clamped'] <= RMS_BAR, rep


def test_cfg5_slab_plans_dispatch_as_whole(cfg4_case):
    """Each row slab's decoder plan (4 ranks at configs[4]) launches, conv for conv, the kernel variant (kernel,
    tile, K split: dbsr_conv_dispatch_variant) the whole-image decoder plan launches -- the property that keeps
    a frame-sharded prediction independent of the rank count (decoders.py:54-62 decodes all rows at once)."""
    from dbsr_amd import _lib as L
    from dbsr_amd.parallel import frame_shard, shard_range
    net, burst, _, _, _ = cfg4_case
    net = net.to(DEV).set_compute_dtype(torch.float16)
    eng = net._get_engine()
    b = burst.to(DEV)
    with torch.no_grad():
        frames, first = frame_shard(14, 0, 4)
        eng.forward_partial(b[:, frames], first)
    lib = L.lib()
    whole = eng.plans.get(('combine', 4, 1, 96, 96, None)) or eng._build_combine(4, 1, 96, 96)
    wv = [lib.dbsr_conv_dispatch_variant(ctypes.byref(d)) for d, _ in whole.convs]
    assert len(wv) >= 10
    for r in range(4):
        rows = shard_range(96, r, 4)
        slab = eng._build_combine(4, 1, 96, 96, rows)
        sv = [lib.dbsr_conv_dispatch_variant(ctypes.byref(d)) for d, _ in slab.convs]
        assert sv == wv, (r, rows, sv, wv)
        assert [bool(getattr(d, 'fused_head', False)) for d, _ in slab.convs] == \
            [bool(getattr(d, 'fused_head', False)) for d, _ in whole.convs]


@pytest.mark.parametrize('size', [(96, 80), (48, 48)])      # 48x48: the per-level specialised dense kernels
@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float16])
def test_pwc_fused_dense_levels(synth_sd, dtype, size):
    """The fused coarse-level DenseNet (dbsr_pwc_dense, levels 6..3) against the per-conv path on the same
    16-bit inputs, and both against the fp32 oracle PWC-Net (pwcnet.py:248-281): the fused path may not
    be further from the oracle than the per-conv one (the two differ only in summation order and in
    where activations round to 16 bits)."""
    from dbsr_amd.engine import PWCPlanner
    from dbsr_amd.pwcnet import PWCNet
    from oracle import dbsr_oracle as orc
    pre = 'encoder.alignment_net.'
    gen = torch.Generator().manual_seed(5)
    src = torch.rand(6, 3, *size, generator=gen)
    tgt = (src + 0.05 * torch.randn(6, 3, *size, generator=gen)).clamp(0, 1)
    ref = orc.pwcnet(src, tgt, synth_sd)
    flows = {}
    try:
        for fused in (True, False):
            PWCPlanner.FUSED_DENSE = fused
            net = PWCNet(load_pretrained=False)
            net.load_state_dict({k[len(pre):]: v for k, v in synth_sd.items() if k.startswith(pre)})
            net = net.to(DEV)
            net.compute_dtype = dtype
            with torch.no_grad():
                flows[fused] = net(src.to(DEV), tgt.to(DEV)).cpu()
    finally:
        PWCPlanner.FUSED_DENSE = True
    e_f = (flows[True] - ref).abs().max().item()
    e_u = (flows[False] - ref).abs().max().item()
    d = (flows[True] - flows[False]).abs().max().item()
    scale = ref.abs().max().item()
    print('fused err %.4g unfused err %.4g diff %.4g (|flow| max %.3g)' % (e_f, e_u, d, scale))
    assert e_f <= max(1.5 * e_u, 2e-3 * scale)
    assert d <= 0.02 * scale


@pytest.mark.parametrize('dtype', [torch.float16, torch.bfloat16])
def test_pwc_fused_extractor(synth_sd, dtype):
    """The one-launch feature pyramid (dbsr_pwc_extract, pwcnet.py:45-111) against the per-conv path on the same
    16-bit inputs and both against the fp32 oracle PWC-Net: 48x56 frames (resized to 64x64, pwcnet.py:262-271),
    the flows may differ only by summation order / 16-bit rounding placement."""
    from dbsr_amd.engine import PWCPlanner
    from dbsr_amd.pwcnet import PWCNet
    from oracle import dbsr_oracle as orc
    pre = 'encoder.alignment_net.'
    gen = torch.Generator().manual_seed(15)
    src = torch.rand(10, 3, 48, 56, generator=gen)
    tgt = (src + 0.05 * torch.randn(10, 3, 48, 56, generator=gen)).clamp(0, 1)
    ref = orc.pwcnet(src, tgt, synth_sd)
    flows = {}
    try:
        for fused in (True, False):
            PWCPlanner.FUSED_EXTRACT = fused
            net = PWCNet(load_pretrained=False)
            net.load_state_dict({k[len(pre):]: v for k, v in synth_sd.items() if k.startswith(pre)})
            net = net.to(DEV)
            net.compute_dtype = dtype
            with torch.no_grad():
                flows[fused] = net(src.to(DEV), tgt.to(DEV)).cpu()
            names = [n for _, _, n, _ in next(iter(net._engine.plans.values())).ops]
            assert ('pwc.extract' in names) == fused, names
    finally:
        PWCPlanner.FUSED_EXTRACT = True
    e_f = (flows[True] - ref).abs().max().item()
    e_u = (flows[False] - ref).abs().max().item()
    d = (flows[True] - flows[False]).abs().max().item()
    scale = ref.abs().max().item()
    print('fused extractor err %.4g unfused err %.4g diff %.4g (|flow| max %.3g)' % (e_f, e_u, d, scale))
    assert e_f <= max(1.5 * e_u, 2e-3 * scale)
    assert d <= 0.02 * scale
