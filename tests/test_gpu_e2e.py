"""End-to-end parity of the MI355X DBSR forward against fixtures produced by the reference itself
(tests/golden/make_golden.py).  Tolerances (north_star): fp32 max-abs <= 1e-3; bf16: PSNR delta
against the reference's PSNR on the same synthetic ground truth."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'
E2E = ['e2e_b1n4', 'e2e_b1n14', 'e2e_b2n4_zeroflow', 'e2e_b1n3_h40w56']


def _net(synth_sd, dtype=torch.float32, zero_flow=False):
    import dbsr_amd
    net = dbsr_amd.dbsrnet_cvpr2021(**dbsr_amd.DBSR_SYNTHETIC_KWARGS)
    net.load_state_dict(synth_sd)
    net = net.to(DEV).eval()
    net.set_compute_dtype(dtype)
    net.zero_flow = zero_flow
    return net


def psnr_q(pred, gt, bi=40):
    """compute_score.py:110-115 quantisation + PSNR(boundary_ignore=40) (image_quality_v2.py:69-101)."""
    q = (pred.clamp(0.0, 1.0) * 2 ** 14).short().float() / 2 ** 14
    return [float(10 * torch.log10(1.0 / ((p - g_)[..., bi:-bi, bi:-bi] ** 2).mean())) for p, g_ in zip(q, gt)]


@pytest.mark.parametrize('name', E2E)
def test_e2e_fp32(golden, synth_sd, name):
    g = golden(name)
    net = _net(synth_sd, torch.float32, bool(g['zero_flow']))
    burst = torch.from_numpy(g['burst']).to(DEV)
    with torch.no_grad():
        pred, aux = net(burst)
    pred = pred.cpu()
    np.testing.assert_allclose(aux['offsets'].cpu().numpy(), g['offsets'], atol=1e-3, rtol=0)
    np.testing.assert_allclose(pred[..., 100:164, 100:164].numpy(), g['pred_crop'], atol=1e-3, rtol=0)
    fw = aux['fusion_weights'].cpu()
    np.testing.assert_allclose(fw[:, :, :16, 8:16, 8:16].numpy(), g['fw_crop'], atol=1e-3, rtol=0)
    np.testing.assert_allclose(pred.double().sum(dim=(-2, -1)).numpy(), g['pred_sum'], rtol=1e-4)
    if 'pred_q' in g:
        q = (pred.clamp(0, 1) * 2 ** 14).short().numpy().astype(np.int64)
        assert np.abs(q - g['pred_q'].astype(np.int64)).max() <= 20   # 1e-3 * 2^14 = 16.4 quanta


@pytest.mark.parametrize('dtype', [torch.float16, torch.bfloat16])
@pytest.mark.parametrize('name', ['e2e_b1n14', 'e2e_b1n4'])
def test_e2e_16bit_psnr(golden, synth_sd, name, dtype):
    g = golden(name)
    burst = torch.from_numpy(g['burst'])
    gt = torch.from_numpy(g['gt_u16'].astype(np.float32)) / 65535.0
    net = _net(synth_sd, dtype)
    with torch.no_grad():
        pred, _ = net(burst.to(DEV))
    mine = psnr_q(pred.float().cpu(), gt)
    delta = max(abs(a - b) for a, b in zip(mine, g['ref_psnr']))
    print(dtype, 'PSNR', mine, 'ref', list(g['ref_psnr']), 'delta', delta)
    assert delta <= 0.01          # north_star: PSNR within 0.01 dB of the reference


def test_graph_replay_matches_eager(golden, synth_sd):
    g = golden('e2e_b1n4')
    burst = torch.from_numpy(g['burst']).to(DEV)
    net = _net(synth_sd, torch.bfloat16)
    with torch.no_grad():
        p0, a0 = net(burst)
        net.use_graph = True
        p1, a1 = net(burst)
        p1, o1 = p1.clone(), a1['offsets'].clone()
        p2, _ = net(burst * 0.5)
    assert torch.equal(p0, p1) and torch.equal(a0['offsets'], o1)
    assert not torch.equal(p1, p2)


def test_cfg3_burstsr_shape_fp32(synth_sd):
    """configs[2] shape (BurstSR real crops: 14 frames, 80x80, fp32) against the oracle on the same
    input.  Real-RAW layout: black-level-subtracted 10-bit values /1023 (burstsr_dataset.py:57,78-90),
    emulated by quantising a synthetic burst to 1/1023 steps.  80 is not a multiple of 64, so PWC-Net's
    resize-to-128 path (pwcnet.py:256-259) and the W/W64 flow rescale are exercised."""
    from dbsr_amd.burst import synthetic_bursts
    from oracle import dbsr_oracle as orc
    burst, _ = synthetic_bursts(1, 14, 80, 80, sr_factor=8, seed=11)
    burst = (burst * 1023).round() / 1023
    net = _net(synth_sd, torch.float32)
    with torch.no_grad():
        pred, aux = net(burst.to(DEV))
    ref, raux = orc.dbsr_forward(burst, synth_sd)
    assert pred.shape == (1, 3, 640, 640)
    assert (aux['offsets'].cpu() - raux['offsets']).abs().max().item() <= 1e-3
    assert (pred.cpu() - ref).abs().max().item() <= 1e-3


def test_burst_longer_than_16_fp32(synth_sd):
    """A 20-frame burst (the reference accepts any burst size, merging.py:116-124): the fusion takes the
    any-N kernel; fp32 against the oracle at the north_star's 1e-3."""
    from dbsr_amd.burst import synthetic_bursts
    from oracle import dbsr_oracle as orc
    burst, _ = synthetic_bursts(1, 20, 32, 32, sr_factor=8, seed=21)
    net = _net(synth_sd, torch.float32)
    with torch.no_grad():
        pred, aux = net(burst.to(DEV))
    ref, raux = orc.dbsr_forward(burst, synth_sd)
    assert aux['fusion_weights'].shape[1] == 20
    assert (aux['offsets'].cpu() - raux['offsets']).abs().max().item() <= 1e-3
    assert (pred.cpu() - ref).abs().max().item() <= 1e-3


def test_compute_score_hip_vs_oracle(tmp_path, synth_sd):
    """SyntheticBurstVal-layout files -> evaluation.compute_score with the HIP bf16 network (batched)
    vs the same scoring of the oracle's fp32 forward, per image within the 0.01 dB bar."""
    from dbsr_amd import evaluation as ev
    from dbsr_amd.burst import synthetic_bursts
    from oracle import dbsr_oracle as orc
    burst, gt = synthetic_bursts(2, 14, 48, 48, sr_factor=8, seed=21)
    ev.write_synthetic_burst_val(str(tmp_path), burst, gt)
    ds = ev.SyntheticBurstVal(str(tmp_path))
    net = _net(synth_sd, torch.bfloat16)
    mine = ev.compute_score(net, ds, boundary_ignore=40, device=DEV, batch=2)
    psnr = ev.PSNR(boundary_ignore=40)
    for i in range(len(ds)):
        b, g, meta = ds[i]
        ref, _ = orc.dbsr_forward(b.unsqueeze(0), synth_sd)
        r = float(psnr(ev.quantize_prediction(ref), g.unsqueeze(0)))
        print(meta['burst_name'], mine['per_image'][meta['burst_name']], r)
        assert abs(mine['per_image'][meta['burst_name']] - r) <= 0.01


@pytest.mark.parametrize('world', [1, 2, 3])
def test_frame_sharded_fusion_hip(golden, synth_sd, world):
    """configs[4]'s frame-sharded path on one device: each simulated rank runs forward_partial on its
    frame shard (dbsr_fuse_partial), the statistics are stacked as the all-gather would lay them out, and
    combine_decode (dbsr_fuse_combine + decoder) must reproduce the reference forward (fp32, 1e-3)."""
    from dbsr_amd.parallel import frame_shard
    g = golden('e2e_b1n4')
    burst = torch.from_numpy(g['burst']).to(DEV)
    net = _net(synth_sd, torch.float32)
    eng = net._get_engine()
    B, N, _, H, W = burst.shape
    with torch.no_grad():
        stats = []
        for r in range(world):
            frames, first = frame_shard(N, r, world)
            st, _ = eng.forward_partial(burst[:, frames], first)
            stats.append(st.clone())
        pred = eng.combine_decode(torch.stack(stats)).cpu()
    np.testing.assert_allclose(pred[..., 100:164, 100:164].numpy(), g['pred_crop'], atol=1e-3, rtol=0)
    np.testing.assert_allclose(pred.double().sum(dim=(-2, -1)).numpy(), g['pred_sum'], rtol=1e-4)


def test_bench_shape_forward_is_deterministic(synth_sd):
    """configs[1] shape (bf16, B=8, N=14, 48x48): the first forward of a plan and the steady-state
    forwards (eager and HIP-graph replay) give bitwise identical offsets, predictions and weights."""
    from dbsr_amd.burst import synthetic_bursts
    burst, _ = synthetic_bursts(8, 14, 48, 48, sr_factor=8, seed=9)
    burst = burst.to(DEV)
    net = _net(synth_sd, torch.bfloat16)
    outs = []
    with torch.no_grad():
        for use_graph in (False, False, True, True):
            net.use_graph = use_graph
            pred, aux = net(burst)
            outs.append((pred.clone(), aux['offsets'].clone(), aux['fusion_weights'].clone()))
    for o in outs[1:]:
        assert all(torch.equal(a, b) for a, b in zip(o, outs[0]))


@pytest.mark.parametrize('use_graph', [False, True])
def test_output_slots_zero_copy_and_no_aliasing(synth_sd, use_graph):
    """Outputs are views of a slot's static buffers when nothing from that slot's previous forward is still
    referenced (no copy in the steady state), and never alias outputs the caller still holds."""
    from dbsr_amd.burst import synthetic_bursts
    net = _net(synth_sd, torch.float16)
    net.use_graph = use_graph
    b1, _ = synthetic_bursts(2, 4, 32, 32, sr_factor=8, seed=71)
    b2, _ = synthetic_bursts(2, 4, 32, 32, sr_factor=8, seed=72)
    b1, b2 = b1.to(DEV), b2.to(DEV)
    with torch.no_grad():
        ptrs = set()
        for _ in range(3):                       # results dropped each time: one slot, zero copy
            pred, aux = net(b1)
            ptrs.add(pred.data_ptr())
            del pred, aux
        assert len(ptrs) == 1
        held = []
        for i in range(5):                       # every result held: distinct storage each time
            pred, aux = net(b1 if i % 2 == 0 else b2)
            held.append((pred, aux['offsets'], aux['fusion_weights']))
        assert len({h[0].data_ptr() for h in held}) == 5
        assert len({h[2].data_ptr() for h in held}) == 5
        ref1, ref2 = net(b1), net(b2)
        for i, (p, o, f) in enumerate(held):
            r = ref1 if i % 2 == 0 else ref2
            assert torch.equal(p, r[0]) and torch.equal(o, r[1]['offsets']), i
            assert torch.equal(f, r[1]['fusion_weights']), i


def test_fusion_weights_reference_contract(synth_sd):
    """aux['fusion_weights'] is the reference's tensor (merging.py:117-126): fp32, contiguous [B,N,C,H,W],
    the softmax over the burst (sums to 1 over N), equal to the engine's channels-last buffer
    (aux.native_fusion_weights, the zero-copy view) -- in 16-bit compute mode too."""
    from dbsr_amd.burst import synthetic_bursts
    burst, _ = synthetic_bursts(2, 5, 32, 48, sr_factor=8, seed=81)
    net = _net(synth_sd, torch.float16)
    with torch.no_grad():
        _, aux = net(burst.to(DEV))
    fw = aux['fusion_weights']
    assert fw.dtype == torch.float32 and fw.is_contiguous() and fw.shape == (2, 5, 512, 32, 48)
    nat = aux.native_fusion_weights
    assert nat.shape == fw.shape and nat.dtype == torch.float16
    assert torch.equal(fw, nat.float())
    s = fw.sum(dim=1)
    assert float((s - 1).abs().max()) <= 5e-3            # 16-bit stored weights, fp32 softmax
    assert set(aux.keys()) == {'offsets', 'fusion_weights'} and aux.get('fusion_weights') is fw
