"""The oracle (oracle/dbsr_oracle.py) pinned against fixtures produced by the reference itself
(tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest
import torch

from oracle import dbsr_oracle as orc

E2E = ['e2e_b1n4', 'e2e_b1n14', 'e2e_b2n4_zeroflow', 'e2e_b1n3_h40w56']


@pytest.mark.parametrize('name', E2E)
def test_oracle_e2e_matches_reference(golden, synth_sd, name):
    g = golden(name)
    burst = torch.from_numpy(g['burst'])
    with torch.no_grad():
        pred, aux = orc.dbsr_forward(burst, synth_sd, zero_flow=bool(g['zero_flow']), return_intermediates=True)
    np.testing.assert_allclose(aux['offsets'].numpy(), g['offsets'], atol=1e-5, rtol=0)
    np.testing.assert_allclose(pred[..., 100:164, 100:164].numpy(), g['pred_crop'], atol=1e-5, rtol=0)
    np.testing.assert_allclose(aux['fused_enc'][:, :64, 8:24, 8:24].numpy(), g['fused_crop'], atol=1e-5, rtol=0)
    fw = aux['fusion_weights']
    np.testing.assert_allclose(fw[:, :, :16, 8:16, 8:16].numpy(), g['fw_crop'], atol=1e-6, rtol=0)
    np.testing.assert_allclose(fw.double().sum(dim=(-2, -1)).float().numpy(), g['fw_sum'], rtol=1e-5, atol=1e-4)
    np.testing.assert_allclose(pred.double().sum(dim=(-2, -1)).float().numpy(), g['pred_sum'], rtol=1e-5)


def test_oracle_correlation_vs_k2_loops(golden):
    g = golden('ops')
    out = orc.correlation(torch.from_numpy(g['corr_f1']), torch.from_numpy(g['corr_f2']))
    np.testing.assert_allclose(out.numpy(), g['corr_out'], atol=1e-5, rtol=0)


@pytest.mark.parametrize('tag', ['bw8', 'bw2'])
def test_oracle_backwarp(golden, tag):
    g = golden('ops')
    out = orc.backwarp(torch.from_numpy(g[f'{tag}_x']), torch.from_numpy(g[f'{tag}_flow']) * float(g[f'{tag}_scale']))
    np.testing.assert_allclose(out.numpy(), g[f'{tag}_out'], atol=1e-6, rtol=0)


def test_oracle_warp(golden):
    g = golden('ops')
    out = orc.warp(torch.from_numpy(g['warp_x']), torch.from_numpy(g['warp_flow']))
    np.testing.assert_allclose(out.numpy(), g['warp_out'], atol=1e-6, rtol=0)


def test_oracle_pwcnet(golden, synth_sd):
    g = golden('ops')
    with torch.no_grad():
        fl = orc.pwcnet(torch.from_numpy(g['pwc_src']), torch.from_numpy(g['pwc_tgt']), synth_sd)
    np.testing.assert_allclose(fl.numpy(), g['pwc_flow'], atol=1e-5, rtol=0)


def test_oracle_pixshuffle_blur(golden):
    import torch.nn.functional as F
    g = golden('ops')
    x, w = torch.from_numpy(g['up_x']), torch.from_numpy(g['up_w'])
    out = F.pixel_shuffle(F.relu(F.conv2d(x, w)), 4)
    K = orc.gauss_kernel(3, 1.0)
    shp = out.shape
    out = F.conv2d(out.reshape(-1, 1, *shp[-2:]), K, padding=1).view(shp)
    np.testing.assert_allclose(out.numpy(), g['up_out'], atol=1e-6, rtol=0)


# ---------------- WeightedSum constructor variants (tests/golden/make_golden_variants.py) ----------------
VARIANTS = {'relu': dict(softmax=False), 'mean': dict(use_base_frame=False), 'nomod': dict(offset_modulo=None),
            'all': dict(softmax=False, use_base_frame=False, offset_modulo=None)}


@pytest.mark.parametrize('case', list(VARIANTS))
def test_oracle_merging_variants(golden, case):
    """oracle.merging with softmax / use_base_frame / offset_modulo against the reference WeightedSum module
    (merging.py:61-127) on offsets reaching past [-3, 3)."""
    g = golden('variants')
    sd = {'merging.' + k[len('merging_sd.'):]: torch.from_numpy(g[k]) for k in g if k.startswith('merging_sd.')}
    kw = {**dict(num_weight_predictor_res=1, num_offset_feat_extractor_res=1, offset_modulo=1.0, use_base_frame=True),
          **VARIANTS[case]}
    x = {'ref_feat': torch.from_numpy(g['merging_ref_feat']), 'oth_feat': torch.from_numpy(g['merging_oth_feat']),
         'offsets': torch.from_numpy(g['merging_offsets'])}
    with torch.no_grad():
        r = orc.merging(x, sd, kw)
    np.testing.assert_allclose(r['fused_enc'].numpy(), g[f'merging_{case}_fused'], atol=1e-6, rtol=0)
    np.testing.assert_allclose(r['fusion_weights'].numpy(), g[f'merging_{case}_weights'], atol=1e-6, rtol=0)


@pytest.mark.parametrize('case', ['relu', 'all'])
def test_oracle_e2e_variants(golden, synth_sd, case):
    """The whole oracle forward with the variant flags against the reference dbsrnet_cvpr2021 built with them."""
    g = golden('variants')
    kw = dict(orc.DBSR_SYNTHETIC_KWARGS, **VARIANTS[case])
    with torch.no_grad():
        pred, aux = orc.dbsr_forward(torch.from_numpy(g['e2e_burst']), synth_sd, kw=kw)
    np.testing.assert_allclose(aux['offsets'].numpy(), g['e2e_offsets'], atol=1e-5, rtol=0)
    np.testing.assert_allclose(pred[..., 100:164, 100:164].numpy(), g[f'e2e_{case}_pred_crop'], atol=1e-5, rtol=0)
    fw = aux['fusion_weights']
    np.testing.assert_allclose(fw[:, :, :16, 8:16, 8:16].numpy(), g[f'e2e_{case}_fw_crop'], atol=1e-6, rtol=0)
    np.testing.assert_allclose(pred.double().sum(dim=(-2, -1)).float().numpy(), g[f'e2e_{case}_pred_sum'], rtol=1e-5)
