"""Eval-harness counterpart (dbsr_amd.evaluation): PNG codec with cv2 channel conventions, the
SyntheticBurstVal reader, and the reference's metric semantics pinned to values produced by the
reference's own image_quality_v2.py (tests/golden/make_golden_eval.py)."""
import os

import numpy as np
import pytest
import torch
from PIL import Image

from dbsr_amd import evaluation as ev


@pytest.mark.parametrize('ftype', [0, 1, 2, 3, 4])
@pytest.mark.parametrize('shape,dtype', [((7, 9, 4), np.uint16), ((5, 11, 3), np.uint16), ((6, 4), np.uint8),
                                         ((3, 5, 3), np.uint8), ((4, 6, 2), np.uint16)])
def test_png_roundtrip_all_filters(tmp_path, ftype, shape, dtype):
    rng = np.random.default_rng(ftype)
    img = rng.integers(0, np.iinfo(dtype).max, size=shape, endpoint=True).astype(dtype)
    p = str(tmp_path / 'x.png')
    ev.png_write(p, img, filter_type=ftype)
    out = ev.png_read(p)
    np.testing.assert_array_equal(out.reshape(img.shape), img)


def test_png_decodes_pillow_files(tmp_path):
    """Files written by an independent encoder (Pillow's adaptive filtering) decode identically."""
    rng = np.random.default_rng(1)
    smooth = (np.add.outer(np.arange(40), np.arange(52)) * 3 % 256).astype(np.uint8)
    rgb = np.stack([smooth, smooth[::-1], rng.integers(0, 255, (40, 52), dtype=np.uint8)], -1)
    Image.fromarray(rgb, 'RGB').save(tmp_path / 'rgb.png', optimize=True)
    np.testing.assert_array_equal(ev.png_read(str(tmp_path / 'rgb.png')), rgb)
    g16 = (np.add.outer(np.arange(33), np.arange(21)) * 911 % 65536).astype(np.uint16)
    Image.fromarray(g16.astype(np.int32)).convert('I;16').save(tmp_path / 'g16.png')
    np.testing.assert_array_equal(ev.png_read(str(tmp_path / 'g16.png'))[..., 0], g16)


def test_png_written_files_open_in_pillow(tmp_path):
    rgb = np.random.default_rng(2).integers(0, 255, (9, 13, 3), dtype=np.uint8)
    ev.png_write(str(tmp_path / 'a.png'), rgb, filter_type=4)
    np.testing.assert_array_equal(np.asarray(Image.open(tmp_path / 'a.png')), rgb)


def test_cv2_channel_order(tmp_path):
    """cv2.imwrite stores an array's channels 0,1,2(,3) as the file's B,G,R(,A) planes."""
    arr = np.zeros((2, 3, 4), np.uint16)
    for c in range(4):
        arr[..., c] = 1000 * (c + 1)
    ev.imwrite(str(tmp_path / 'a.png'), arr)
    on_disk = ev.png_read(str(tmp_path / 'a.png'))
    assert list(on_disk[0, 0]) == [3000, 2000, 1000, 4000]      # file RGBA = array [2,1,0,3]
    np.testing.assert_array_equal(ev.imread_unchanged(str(tmp_path / 'a.png')), arr)


def test_png_rejects_bad_input(tmp_path):
    p = tmp_path / 'bad.png'
    p.write_bytes(b'not a png')
    with pytest.raises(ValueError):
        ev.png_read(str(p))
    ev.png_write(str(tmp_path / 'ok.png'), np.zeros((2, 2, 3), np.uint8))
    data = bytearray((tmp_path / 'ok.png').read_bytes())
    data[-20] ^= 0xff                                            # corrupt the IDAT payload / CRC
    (tmp_path / 'c.png').write_bytes(bytes(data))
    with pytest.raises(ValueError):
        ev.png_read(str(tmp_path / 'c.png'))


def test_synthetic_burst_val_reader(tmp_path):
    from dbsr_amd.burst import synthetic_bursts
    burst, gt = synthetic_bursts(2, 3, 12, 10, sr_factor=8, seed=5)
    ev.write_synthetic_burst_val(str(tmp_path), burst, gt)
    ds = ev.SyntheticBurstVal(str(tmp_path), burst_size=3)
    assert len(ds) == 2
    b, g, meta = ds[1]
    assert b.shape == (3, 4, 12, 10) and g.shape == (3, 96, 80) and meta == {'burst_name': '0001'}
    assert (b - burst[1]).abs().max() <= 0.5 / 2 ** 14 + 1e-7
    assert (g - gt[1]).abs().max() <= 0.5 / 2 ** 14 + 1e-7
    assert os.path.isfile(tmp_path / 'bursts' / '0000' / 'im_raw_02.png')


def test_metrics_match_reference(golden):
    g = golden('eval')
    pred, gt, valid = (torch.from_numpy(g[k]) for k in ('pred', 'gt', 'valid'))
    assert abs(float(ev.PSNR(boundary_ignore=40)(pred, gt)) - g['psnr_b40']) < 1e-5
    assert abs(float(ev.PSNR()(pred[:2], gt[:2])) - g['psnr_none']) < 1e-5
    assert abs(float(ev.PSNR(boundary_ignore=8)(pred[:2], gt[:2], valid[:2])) - g['psnr_b8_valid']) < 1e-5
    assert abs(float(ev.PSNR(boundary_ignore=40, max_value=None)(pred[:2], gt[:2])) - g['psnr_b40_maxnone']) < 1e-5
    for m in ('l1', 'l2', 'l2_sqrt', 'charbonnier'):
        assert abs(float(ev.PixelWiseError(m, boundary_ignore=40)(pred, gt)) - g['err_' + m]) < 1e-7
    np.testing.assert_array_equal(ev.quantize_prediction(pred).numpy(), g['quantized'])


def test_psnr_all_invalid_is_zero():
    x = torch.rand(2, 3, 8, 8)
    assert ev.PSNR()(x, x.clone()) == 0


class _StubNet:
    """CPU stand-in for the network in the harness-plumbing test only (the product forward is GPU-only):
    predicts the nearest-upsampled green plane of frame 0."""
    def __call__(self, burst):
        g = burst[:, 0, 1:3].mean(1, keepdim=True).repeat(1, 3, 1, 1)
        return torch.nn.functional.interpolate(g, scale_factor=8), {}


def test_compute_score_and_save_results_plumbing(tmp_path):
    from dbsr_amd.burst import synthetic_bursts
    burst, gt = synthetic_bursts(3, 2, 12, 12, sr_factor=8, seed=1)
    ev.write_synthetic_burst_val(str(tmp_path / 'ds'), burst, gt)
    ds = ev.SyntheticBurstVal(str(tmp_path / 'ds'), burst_size=2)
    s = ev.compute_score(_StubNet(), ds, boundary_ignore=8, device='cpu', batch=2)
    assert sorted(s['per_image']) == ['0000', '0001', '0002']
    # same numbers one burst at a time, the reference's loop (compute_score.py:92-117)
    psnr = ev.PSNR(boundary_ignore=8)
    for i in range(3):
        b, g, meta = ds[i]
        p, _ = _StubNet()(b.unsqueeze(0))
        assert abs(float(psnr(ev.quantize_prediction(p), g.unsqueeze(0))) - s['per_image'][meta['burst_name']]) < 1e-5
    ev.save_results(_StubNet(), ds, str(tmp_path / 'out'), device='cpu', batch=2)
    saved = ev.load_saved_prediction(str(tmp_path / 'out' / '0001.png'))
    p, _ = _StubNet()(ds[1][0].unsqueeze(0))
    # save_results truncates (astype uint16) like compute_score's .short(): identical quantisation
    np.testing.assert_array_equal(saved.numpy(), ev.quantize_prediction(p).numpy())
