"""BurstSR scoring path on the HIP kernels (csrc/sca_ops.hip + the PWC engine + the warp kernel) against
the oracle restatement, which test_burstsr.py pins to the reference's own SpatialColorAlignment outputs.

Tolerances: resampling / smoothing fp32 vs torch fp32 1e-5 abs; colour matrix 1e-4 relative (normal
equations in fp64 vs LAPACK least squares, then fp32 smoothing differences); the validity mask is a
threshold of computed errors, so it must agree on >= 99.5 % of pixels (exactly where no error sits
within rounding of the threshold); the full forward uses the fp32 HIP PWC-Net (flow within 1e-3 of the
reference, as the e2e PWC fixture)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = 'cuda'


@pytest.fixture(scope='module')
def bs():
    from dbsr_amd import burstsr
    return burstsr


@pytest.mark.parametrize('shape,scale,mul', [((2, 3, 128, 128), 1 / 8, 1.0), ((1, 2, 640, 640), 1 / 8, 1 / 8),
                                             ((3, 1, 80, 72), 8.0, 1.0), ((1, 3, 33, 47), 0.5, 2.0)])
def test_resize_bilinear(bs, shape, scale, mul):
    x = torch.randn(*shape, generator=torch.Generator().manual_seed(shape[-1]))
    ref = F.interpolate(x, scale_factor=scale, mode='bilinear') * mul
    out = bs.resize_bilinear(x.to(DEV), scale, mul=mul).cpu()
    assert out.shape == ref.shape
    np.testing.assert_allclose(out.numpy(), ref.numpy(), atol=1e-5, rtol=1e-5)


def test_gauss_reflect(bs):
    from oracle import dbsr_oracle as orc
    x = torch.rand(2, 3, 80, 64, generator=torch.Generator().manual_seed(1))
    K, ksz = bs.get_gaussian_kernel(1.5)
    ref = orc.apply_kernel(x, ksz, K)
    out = bs.apply_kernel(x.to(DEV), ksz, K).cpu()
    np.testing.assert_allclose(out.numpy(), ref.numpy(), atol=1e-6)


def test_match_colors_vs_reference_fixture(bs, golden):
    g = golden('burstsr')
    K, ksz = bs.get_gaussian_kernel(1.5)
    out, valid = bs.match_colors(torch.from_numpy(g['b_ref']).to(DEV), torch.from_numpy(g['b_q']).to(DEV),
                                 torch.from_numpy(g['b_test']).to(DEV), ksz, K)
    np.testing.assert_allclose(bs.match_colors.last_cmat.cpu().numpy(), g['b_cmat'], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(out.cpu().numpy(), g['b_out'], rtol=1e-4, atol=1e-5)
    agree = (valid.cpu().numpy() == g['b_valid']).mean()
    assert agree >= 0.995, agree
    assert 0.2 < g['b_valid'].mean() < 0.9            # the fixture exercises both sides of the mask


def _pwc(synth_sd):
    from dbsr_amd.pwcnet import PWCNet
    pre = 'encoder.alignment_net.'
    net = PWCNet(load_pretrained=False)
    net.load_state_dict({k[len(pre):]: v for k, v in synth_sd.items() if k.startswith(pre)})
    return net.to(DEV)


def test_sca_forward_vs_reference_fixture(bs, golden, synth_sd):
    g = golden('burstsr')
    sca = bs.SpatialColorAlignment(_pwc(synth_sd), sr_factor=4)
    pred, gt, burst = (torch.from_numpy(g[k]).to(DEV) for k in ('a_pred', 'a_gt', 'a_burst'))
    out, valid = sca(pred, gt, burst)
    flow = sca.alignment_net(pred / (pred.max() + 1e-6), gt / (gt.max() + 1e-6))
    assert (flow.cpu() - torch.from_numpy(g['a_flow'])).abs().max().item() <= 1e-3
    np.testing.assert_allclose(bs.match_colors.last_cmat.cpu().numpy(), g['a_cmat'], rtol=2e-3, atol=2e-3)
    v = valid.cpu().numpy()
    assert (v == g['a_valid']).mean() >= 0.99
    both = v & g['a_valid']
    d = np.abs(out.cpu().numpy() - g['a_out'])[np.broadcast_to(both, g['a_out'].shape)]
    assert d.max() <= 5e-3, d.max()


def test_compute_score_burstsr_end_to_end(bs, tmp_path, synth_sd):
    """Two synthetic bursts written in the BurstSR layout -> HIP network (fp32, x8) -> quantise -> HIP
    spatial-colour alignment -> masked PSNR, against the same chain on the oracle."""
    import dbsr_amd
    from dbsr_amd.burst import synthetic_bursts
    from dbsr_amd.evaluation import PSNR, quantize_prediction
    from oracle import dbsr_oracle as orc
    from tests.test_burstsr import _meta_canon, _meta_samsung
    bursts, gts = synthetic_bursts(2, 14, 40, 40, sr_factor=8, seed=21)
    exp_scale = ((1 / 50) * 200 / 1.7 ** 2) / ((1 / 100) * 100 / 4.0 ** 2)     # the two metas' light factors
    for b in range(2):
        fr = (bursts[b].numpy() * 1023 + 64).round().clip(0, 65535).astype(np.uint16)
        gt = (gts[b].numpy() * 16383 / exp_scale + 512).round().clip(0, 65535).astype(np.uint16)
        bs.write_burstsr_sample(str(tmp_path), '00%02d_0000' % b, fr, gt, _meta_samsung(), _meta_canon())
    ds = bs.BurstSRDataset(str(tmp_path), processing=bs.BurstSRProcessing(crop_sz=40))
    net = dbsr_amd.dbsrnet_cvpr2021(**dbsr_amd.DBSR_SYNTHETIC_KWARGS)
    net.load_state_dict(synth_sd)
    net = net.to(DEV).set_compute_dtype(torch.float32)
    res = bs.compute_score_burstsr(net, ds, _pwc(synth_sd))
    psnr_fn = PSNR(boundary_ignore=40)
    for i in range(2):
        burst, gt, info = ds[i]
        with torch.no_grad():
            pred, _ = orc.dbsr_forward(burst.unsqueeze(0), synth_sd)
        pred = quantize_prediction(pred)
        out, valid, _, _ = orc.spatial_color_alignment(pred, gt.unsqueeze(0), burst.unsqueeze(0), synth_sd)
        ref = float(psnr_fn(out, gt.unsqueeze(0), valid=valid))
        mine = res['per_image'][info['burst_name']]
        print(info['burst_name'], mine, ref)
        assert abs(mine - ref) <= 0.05, (mine, ref)
