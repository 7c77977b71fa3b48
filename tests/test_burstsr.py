"""BurstSR scoring path, CPU side: the oracle's SpatialColorAlignment restatement against the reference's
own outputs (tests/golden/make_golden_burstsr.py ran spatial_color_alignment.py on torch-CPU), the
Samsung / Canon readers, BurstSRProcessing and the restricted meta_info.pkl loader.  The HIP path is
checked against these in test_gpu_burstsr.py."""
import io
import json
import pickle
import sys
import types

import numpy as np
import pytest
import torch

from dbsr_amd import burstsr as bs
from oracle import dbsr_oracle as orc


def test_oracle_match_colors_vs_reference(golden):
    g = golden('burstsr')
    K, ksz = orc.gaussian_kernel_2d(1.5)
    out, valid, cmat = orc.match_colors(torch.from_numpy(g['b_ref']), torch.from_numpy(g['b_q']),
                                        torch.from_numpy(g['b_test']), ksz, K)
    np.testing.assert_allclose(cmat.numpy(), g['b_cmat'], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(out.numpy(), g['b_out'], rtol=1e-5, atol=1e-6)
    np.testing.assert_array_equal(valid.numpy(), g['b_valid'])


def test_oracle_sca_forward_vs_reference(golden, synth_sd):
    g = golden('burstsr')
    out, valid, flow, cmat = orc.spatial_color_alignment(torch.from_numpy(g['a_pred']), torch.from_numpy(g['a_gt']),
                                                         torch.from_numpy(g['a_burst']), synth_sd)
    np.testing.assert_allclose(flow.numpy(), g['a_flow'], atol=1e-5)
    np.testing.assert_allclose(cmat.numpy(), g['a_cmat'], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(out.numpy(), g['a_out'], atol=1e-5)
    np.testing.assert_array_equal(valid.numpy(), g['a_valid'])


def test_gaussian_kernel_matches_oracle():
    K, ksz = bs.get_gaussian_kernel(1.5)
    K2, ksz2 = orc.gaussian_kernel_2d(1.5)
    assert ksz == ksz2 == 7
    assert torch.equal(K, K2)


def _meta_samsung():
    return {'black_level': [64, 64, 64, 64], 'cam_wb': [2.0, 1.0, 1.0, 1.6], 'daylight_wb': [2.1, 1.0, 1.0, 1.5],
            'color_matrix': [[1.5, -0.4, -0.1], [-0.2, 1.4, -0.2], [0.0, -0.6, 1.6]],
            'exif_data': {'Image ExposureTime': [[1, 50]], 'Image FNumber': [[17, 10]],
                          'Image ISOSpeedRatings': [200], 'Image Tag 0xC761': [[1e-4], [2e-6], [1e-4], [2e-6],
                                                                                [1e-4], [2e-6]]}}


def _meta_canon():
    return {'black_level': [512, 512, 512, 512], 'cam_wb': [2048, 1024, 1024, 1700],
            'daylight_wb': [2000, 1024, 1024, 1650], 'rgb_xyz_matrix': np.eye(3).tolist(),
            'exif_data': {'EXIF ExposureTime': [[1, 100]], 'EXIF FNumber': [[4, 1]], 'EXIF ISOSpeedRatings': [100]}}


def test_reader_and_processing(tmp_path):
    rng = np.random.default_rng(5)
    frames = rng.integers(64, 1023, size=(14, 4, 96, 88)).astype(np.uint16)
    gt = rng.integers(512, 16383, size=(3, 768, 704)).astype(np.uint16)
    bs.write_burstsr_sample(str(tmp_path), '0003_0001', frames, gt, _meta_samsung(), _meta_canon())
    bs.write_burstsr_sample(str(tmp_path), '0007_0002', frames[:, :, :80, :80], gt[:, :640, :640], _meta_samsung(),
                            _meta_canon())
    ds = bs.BurstSRDataset(str(tmp_path), split='val', seq_ids=['0003', '0007'])
    assert ds.burst_list == ['0003_0001', '0007_0002']
    burst, gtd, info = ds[0]
    assert burst.shape == (14, 4, 80, 80) and gtd.shape == (3, 640, 640)
    # centre crop (processing.py:176-189 with random_crop=False): rows 8..88, cols 4..84; gt x8
    exp = (frames[:, :, 8:88, 4:84].astype(np.float32) - 64) / 1023.0
    np.testing.assert_allclose(burst.numpy(), exp, rtol=1e-6, atol=1e-7)
    lf_b = (1 / 50) * 200 / 1.7 ** 2
    lf_c = (1 / 100) * 100 / 4.0 ** 2
    exp_gt = (gt[:, 64:704, 32:672].astype(np.float32) - 512) / 16383.0 * (lf_b / lf_c)
    np.testing.assert_allclose(gtd.numpy(), exp_gt, rtol=1e-5, atol=1e-6)
    assert info['burst_name'] == '0003_0001' and abs(info['exp_scale_factor'] - lf_b / lf_c) < 1e-12
    # already crop-sized: no crop
    burst2, gt2, _ = ds[1]
    np.testing.assert_allclose(burst2.numpy(), (frames[:, :, :80, :80].astype(np.float32) - 64) / 1023.0, atol=1e-7)
    im = bs.SamsungRAWImage.load(str(tmp_path / 'val' / '0003_0001' / 'samsung_00'))
    assert im.im_raw.dtype == torch.int16 and np.allclose(im.get_noise_profile()[:, 0], 1e-4)


class _FakeTag:
    pass


def test_meta_pickle_restricted_loader(tmp_path):
    """A meta_info.pkl shaped like the dataset's (numpy arrays, exifread IfdTag / Ratio objects) loads
    through stand-ins; any other global is refused."""
    from fractions import Fraction
    mod_c = types.ModuleType('exifread.classes')
    mod_u = types.ModuleType('exifread.utils')

    class IfdTag:
        pass

    class Ratio(Fraction):
        pass
    IfdTag.__module__, IfdTag.__qualname__ = 'exifread.classes', 'IfdTag'
    Ratio.__module__, Ratio.__qualname__ = 'exifread.utils', 'Ratio'
    mod_c.IfdTag, mod_u.Ratio = IfdTag, Ratio
    sys.modules.update({'exifread': types.ModuleType('exifread'), 'exifread.classes': mod_c, 'exifread.utils': mod_u})
    try:
        t_exp, t_iso = IfdTag(), IfdTag()
        t_exp.values, t_iso.values = [Ratio(1, 50)], [200]
        meta = {'black_level': [64, 64, 64, 64], 'color_matrix': np.eye(3, dtype=np.float32),
                'exif_data': {'Image ExposureTime': t_exp, 'Image ISOSpeedRatings': t_iso}}
        blob = pickle.dumps(meta, protocol=4)
    finally:
        for k in ('exifread', 'exifread.classes', 'exifread.utils'):
            sys.modules.pop(k, None)
    (tmp_path / 'meta_info.pkl').write_bytes(blob)
    m = bs.load_meta(str(tmp_path))
    assert m['black_level'] == [64, 64, 64, 64] and np.array_equal(m['color_matrix'], np.eye(3))
    assert abs(bs.exif_value(m['exif_data'], 'Image ExposureTime') - 0.02) < 1e-12
    assert bs.exif_value(m['exif_data'], 'Image ISOSpeedRatings') == 200
    evil = pickle.dumps({'x': _FakeTag()})
    (tmp_path / 'meta_info.pkl').write_bytes(evil)
    with pytest.raises(pickle.UnpicklingError, match='not allowed'):
        bs.load_meta(str(tmp_path))


def test_sca_refuses_cpu_tensors():
    with pytest.raises(NotImplementedError, match='HIP'):
        bs.resize_bilinear(torch.zeros(1, 2, 8, 8), 0.5)
