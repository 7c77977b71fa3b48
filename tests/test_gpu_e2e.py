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


@pytest.mark.parametrize('name', ['e2e_b1n14', 'e2e_b1n4'])
def test_e2e_bf16_psnr(golden, synth_sd, name):
    g = golden(name)
    burst = torch.from_numpy(g['burst'])
    gt = torch.from_numpy(g['gt_u16'].astype(np.float32)) / 65535.0
    net = _net(synth_sd, torch.bfloat16)
    with torch.no_grad():
        pred, _ = net(burst.to(DEV))
    mine = psnr_q(pred.float().cpu(), gt)
    delta = max(abs(a - b) for a, b in zip(mine, g['ref_psnr']))
    print('bf16 PSNR', mine, 'ref', list(g['ref_psnr']), 'delta', delta)
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
