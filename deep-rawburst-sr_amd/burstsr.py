"""BurstSR scoring path: the real-data counterpart of `evaluation.compute_score`.

The reference scores a network on the BurstSR validation crops (evaluation/burstsr/compute_score.py:38-136)
by reading Samsung RAW bursts and a Canon ground truth (dataset/burstsr_dataset.py:35-302, cv2 + pickled
metadata), normalising them (data/processing.py:126-278), running the network, quantising the prediction
to 2^14, aligning it to the ground truth spatially (PWC-Net flow + warp) and in colour (a per-image 3x3
least-squares fit, models/loss/spatial_color_alignment.py:23-108) and reporting the masked PSNR.  Here:

  * `SamsungRAWImage` / `CanonImage` (burstsr_dataset.py:35-240): im_raw.png through the cv2-convention
    PNG codec of evaluation.py; meta_info through `load_meta` -- a JSON sidecar, or the dataset's
    meta_info.pkl through a restricted unpickler that only builds plain containers, numpy arrays and
    inert stand-ins for exifread's tag / ratio classes (nothing in the file is executed).
  * `BurstSRProcessing` (processing.py:126-278, evaluation settings: no flip, no noise, no white balance).
  * `BurstSRDataset` + `IndexedBurst` ordering (burstsr_dataset.py:243-291; sampler.py:99-150).
  * `SpatialColorAlignment` / `match_colors` on the HIP path: PWC flow from the engine, warps from the
    warp kernel, resampling / smoothing / colour fit / mask from csrc/sca_ops.hip.
  * `compute_score_burstsr` (compute_score.py:96-134, PSNR column; SSIM / LPIPS are out of scope).

Inputs to the HIP path must be on the device; the product path has no CPU fallback.
"""
import io
import json
import math
import os
import pickle
from fractions import Fraction

import numpy as np
import torch
import torch.nn as nn

from . import _lib as L
from . import ops
from .evaluation import PSNR, imread_unchanged, imwrite, quantize_prediction


# ------------------------------------------------------------------------------------- Gaussian kernel

def get_gaussian_kernel(sd, ksz=None):
    """filtering.py:20-51: normalised 2-D Gaussian density on an odd ksz grid (default int(4 sd + 1)),
    float32 like the reference's torch ops.  Returns ([1, ksz, ksz], ksz)."""
    if ksz is None:
        ksz = int(4 * sd + 1)
    assert ksz % 2 == 1
    k = torch.arange(-(ksz - 1) / 2, (ksz + 1) / 2).reshape(1, -1)
    g = torch.exp(-1.0 / (2 * sd ** 2) * (k - torch.zeros(1, 1)) ** 2) / (math.sqrt(2 * math.pi) * sd)
    K = g.reshape(1, 1, -1) * g.reshape(1, -1, 1)
    K = K / K.sum()
    return K, ksz


# ------------------------------------------------------------------------------------- HIP helpers

def _dev_check(*ts):
    for t in ts:
        if not t.is_cuda:
            raise NotImplementedError('SpatialColorAlignment runs on the HIP device only (no CPU fallback)')


def resize_bilinear(x, scale_factor, mul=1.0):
    """F.interpolate(x, scale_factor=s, mode='bilinear') (align_corners=False) * mul, fp32 NCHW."""
    _dev_check(x)
    x = x.float().contiguous()
    n, c, h, w = x.shape
    oh, ow = int(math.floor(h * scale_factor)), int(math.floor(w * scale_factor))
    out = torch.empty(n, c, oh, ow, dtype=torch.float32, device=x.device)
    r = float(np.float32(1.0 / scale_factor))
    L.check(L.lib().dbsr_resize_bilinear(n * c, h, w, x.data_ptr(), oh, ow, r, r, float(mul), out.data_ptr(),
                                         L.stream_ptr(x.device)), 'dbsr_resize_bilinear')
    return out


def apply_kernel(im, ksz, kernel):
    """filtering.py:54-63 (reflect padding + ksz x ksz filter per plane)."""
    _dev_check(im)
    im = im.float().contiguous()
    h, w = im.shape[-2:]
    out = torch.empty_like(im)
    k = kernel.reshape(-1).to(torch.float32).cpu().contiguous()
    L.check(L.lib().dbsr_gauss_reflect(im.numel() // (h * w), h, w, ksz, k.data_ptr(), im.data_ptr(),
                                       out.data_ptr(), L.stream_ptr(im.device)), 'dbsr_gauss_reflect')
    return out


def match_colors(im_ref, im_q, im_test, ksz, gauss_kernel, bi=5, thresh=20.0):
    """spatial_color_alignment.py:23-67: C = argmin ||smooth(im_q) C - smooth(im_ref)|| on the crop
    [bi:-bi] per image; returns (im_test^T C, valid) with valid the bilinear-upsampled
    (err * 255 < thresh) mask thresholded > 0.9.  The fitted matrices stay on `match_colors.last_cmat`."""
    _dev_check(im_ref, im_q, im_test)
    n, _, h, w = im_ref.shape
    assert im_q.shape == im_ref.shape and im_ref.shape[1] == 3 and im_test.shape[1] == 3
    ref_s = apply_kernel(im_ref, ksz, gauss_kernel)
    q_s = apply_kernel(im_q, ksz, gauss_kernel)
    dev = im_ref.device
    s = L.stream_ptr(dev)
    cmat = torch.empty(n, 3, 3, dtype=torch.float32, device=dev)
    L.check(L.lib().dbsr_color_fit(n, h, w, bi, ref_s.data_ptr(), q_s.data_ptr(), cmat.data_ptr(), s), 'dbsr_color_fit')
    test = im_test.float().contiguous()
    oh, ow = test.shape[-2:]
    # valid is [n, h - 2bi, w - 2bi] padded back by (w_q - w_valid) // 2 = bi, then upsampled by
    # im_test.shape[-1] / valid.shape[-1] (:52-59)
    f = ow / w
    if (int(math.floor(h * f)), int(math.floor(w * f))) != (oh, ow):
        raise ValueError('match_colors: the upsampled mask (%d x %d) * %.4g does not cover the test image %dx%d'
                         % (h, w, f, oh, ow))
    r = float(np.float32(1.0 / f))
    out = torch.empty_like(test)
    valid = torch.empty(n, 1, oh, ow, dtype=torch.uint8, device=dev)
    L.check(L.lib().dbsr_color_apply(n, h, w, bi, ref_s.data_ptr(), q_s.data_ptr(), cmat.data_ptr(), float(thresh),
                                     test.data_ptr(), oh, ow, r, r, out.data_ptr(), valid.data_ptr(), s),
            'dbsr_color_apply')
    match_colors.last_cmat = cmat
    return out, valid.bool()


class SpatialColorAlignment(nn.Module):
    """spatial_color_alignment.py:70-108: flow pred -> gt from the alignment network, warp of the
    prediction, x1/(2 sr_factor) warp of the base frame's (R, G, B) planes, colour match."""

    def __init__(self, alignment_net, sr_factor=4):
        super().__init__()
        self.sr_factor = sr_factor
        self.alignment_net = alignment_net
        self.gauss_kernel, self.ksz = get_gaussian_kernel(sd=1.5)

    def forward(self, pred, gt, burst_input):
        _dev_check(pred, gt, burst_input)
        with torch.no_grad():
            flow = self.alignment_net(pred / (pred.max() + 1e-6), gt / (gt.max() + 1e-6))
        pred_warped = ops.warp(pred.float().contiguous(), flow)
        ds_factor = 1.0 / float(2.0 * self.sr_factor)
        flow_ds = resize_bilinear(flow, ds_factor, mul=ds_factor)
        burst_0 = burst_input[:, 0, [0, 1, 3]].float().contiguous()
        burst_0_warped = ops.warp(burst_0, flow_ds)
        frame_gt_ds = resize_bilinear(gt, ds_factor)
        return match_colors(frame_gt_ds, burst_0_warped, pred_warped, self.ksz, self.gauss_kernel)


# ------------------------------------------------------------------------------------- metadata

class _ExifStandIn:
    """Inert stand-in for an exifread class (IfdTag, ...): keeps the pickled attribute dict."""

    def __setstate__(self, state):
        if isinstance(state, tuple) and len(state) == 2:       # (dict, slots)
            state = {**(state[0] or {}), **(state[1] or {})}
        if isinstance(state, dict):
            self.__dict__.update(state)

    def decimal(self):
        if hasattr(self, 'num') and hasattr(self, 'den'):
            return float(self.num) / float(self.den)
        raise AttributeError('decimal')


class _RatioStandIn(Fraction):
    """exifread.utils.Ratio (a Fraction subclass in exifread >= 2.3): pickled as Ratio(num, den)."""

    def decimal(self):
        return float(self)


_SAFE_GLOBALS = {
    ('builtins', n) for n in ('dict', 'list', 'tuple', 'set', 'frozenset', 'float', 'int', 'str', 'bytes',
                              'bytearray', 'complex', 'bool', 'object')
} | {
    ('collections', 'OrderedDict'), ('fractions', 'Fraction'), ('copyreg', '_reconstructor'),
    ('copyreg', '__newobj__'), ('numpy', 'ndarray'), ('numpy', 'dtype'),
    ('numpy.core.multiarray', '_reconstruct'), ('numpy._core.multiarray', '_reconstruct'),
    ('numpy.core.multiarray', 'scalar'), ('numpy._core.multiarray', 'scalar'),
}


class _MetaUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        if (module, name) in _SAFE_GLOBALS:
            return super().find_class(module, name)
        if module.split('.')[0] == 'exifread':
            return _RatioStandIn if name == 'Ratio' else type(name, (_ExifStandIn,), {})
        raise pickle.UnpicklingError('meta_info.pkl: global %s.%s is not allowed' % (module, name))


def load_meta(path):
    """meta_info of one image directory: meta_info.json (this package's sidecar) if present, else
    meta_info.pkl through the restricted unpickler."""
    js = os.path.join(path, 'meta_info.json')
    if os.path.exists(js):
        with open(js) as f:
            return json.load(f)
    with open(os.path.join(path, 'meta_info.pkl'), 'rb') as f:
        return _MetaUnpickler(io.BytesIO(f.read())).load()


def exif_value(exif, key):
    """exif[key].values[0] (.decimal() for rationals) as the reference's accessors read it, for exifread
    tags, their stand-ins, or JSON values: a list of values, each a number or [numerator, denominator]."""
    v = exif[key]
    vals = v.values if hasattr(v, 'values') else v
    x = vals[0] if isinstance(vals, (list, tuple)) else vals
    if hasattr(x, 'decimal'):
        return x.decimal()
    if isinstance(x, (list, tuple)) and len(x) == 2:
        return x[0] / x[1]
    return float(x)


# ------------------------------------------------------------------------------------- images

class SamsungRAWImage:
    """burstsr_dataset.py:35-111: packed RGGB int16 [4, H, W], black level, norm factor 1023."""

    def __init__(self, im_raw, black_level, cam_wb, daylight_wb, color_matrix, exif_data, im_preview=None):
        self.im_raw = im_raw
        self.black_level = black_level
        self.cam_wb = cam_wb
        self.daylight_wb = daylight_wb
        self.color_matrix = color_matrix
        self.exif_data = exif_data
        self.im_preview = im_preview
        self.norm_factor = 1023.0

    @staticmethod
    def load(path):
        im = imread_unchanged(os.path.join(path, 'im_raw.png'))
        im_raw = torch.from_numpy(np.transpose(im, (2, 0, 1)).astype(np.int16))
        m = load_meta(path)
        return SamsungRAWImage(im_raw, m['black_level'], m['cam_wb'], m['daylight_wb'], m['color_matrix'],
                               m['exif_data'], m.get('im_preview', None))

    def get_all_meta_data(self):
        return {'black_level': self.black_level, 'cam_wb': self.cam_wb, 'daylight_wb': self.daylight_wb,
                'color_matrix': np.asarray(self.color_matrix).tolist()}

    def get_exposure_time(self):
        return exif_value(self.exif_data, 'Image ExposureTime')

    def get_noise_profile(self):
        noise = self.exif_data['Image Tag 0xC761']
        noise = noise.values if hasattr(noise, 'values') else noise
        return np.array([n[0] for n in noise]).reshape(3, 2)

    def get_f_number(self):
        return exif_value(self.exif_data, 'Image FNumber')

    def get_iso(self):
        return exif_value(self.exif_data, 'Image ISOSpeedRatings')

    def get_image_data(self, substract_black_level=False, white_balance=False, normalize=False):
        im_raw = self.im_raw.float()
        if substract_black_level:
            im_raw = im_raw - torch.tensor(self.black_level).view(4, 1, 1)
        if white_balance:
            im_raw = im_raw * torch.tensor(self.cam_wb).view(4, 1, 1)
        if normalize:
            im_raw = im_raw / self.norm_factor
        return im_raw

    def shape(self):
        return (4, self.im_raw.shape[1], self.im_raw.shape[2])

    def get_crop(self, r1, r2, c1, c2):
        prev = self.im_preview[2 * r1:2 * r2, 2 * c1:2 * c2] if self.im_preview is not None else None
        return SamsungRAWImage(self.im_raw[:, r1:r2, c1:c2], self.black_level, self.cam_wb, self.daylight_wb,
                               self.color_matrix, self.exif_data, im_preview=prev)


class CanonImage:
    """burstsr_dataset.py:114-240: RGB int16 [3, H, W] (R, G, B of the RGGB black level / white balance),
    norm factor 16383."""

    def __init__(self, im_raw, black_level, cam_wb, daylight_wb, rgb_xyz_matrix, exif_data):
        self.im_raw = im_raw
        if len(black_level) == 4:
            black_level = [black_level[0], black_level[1], black_level[3]]
        self.black_level = black_level
        if len(cam_wb) == 4:
            cam_wb = [cam_wb[0], cam_wb[1], cam_wb[3]]
        self.cam_wb = cam_wb
        if len(daylight_wb) == 4:
            daylight_wb = [daylight_wb[0], daylight_wb[1], daylight_wb[3]]
        self.daylight_wb = daylight_wb
        self.rgb_xyz_matrix = rgb_xyz_matrix
        self.exif_data = exif_data
        self.norm_factor = 16383

    @staticmethod
    def load(path):
        im = imread_unchanged(os.path.join(path, 'im_raw.png'))
        im_raw = torch.from_numpy(np.transpose(im, (2, 0, 1)).astype(np.int16))
        m = load_meta(path)
        return CanonImage(im_raw.float(), m['black_level'], m['cam_wb'], m['daylight_wb'], m['rgb_xyz_matrix'],
                          m['exif_data'])

    def get_all_meta_data(self):
        return {'black_level': self.black_level, 'cam_wb': self.cam_wb, 'daylight_wb': self.daylight_wb,
                'rgb_xyz_matrix': np.asarray(self.rgb_xyz_matrix).tolist(), 'norm_factor': self.norm_factor}

    def get_exposure_time(self):
        return exif_value(self.exif_data, 'EXIF ExposureTime')

    def get_f_number(self):
        return exif_value(self.exif_data, 'EXIF FNumber')

    def get_iso(self):
        return exif_value(self.exif_data, 'EXIF ISOSpeedRatings')

    def get_image_data(self, substract_black_level=False, white_balance=False, normalize=False):
        im_raw = self.im_raw.float()
        if substract_black_level:
            im_raw = im_raw - torch.tensor(self.black_level).view(3, 1, 1)
        if white_balance:
            im_raw = im_raw * torch.tensor(self.cam_wb).view(3, 1, 1) / 1024.0
        if normalize:
            im_raw = im_raw / self.norm_factor
        return im_raw

    def shape(self):
        return (3, self.im_raw.shape[1], self.im_raw.shape[2])

    def get_crop(self, r1, r2, c1, c2):
        return CanonImage(self.im_raw[:, r1:r2, c1:c2], self.black_level, self.cam_wb, self.daylight_wb,
                          self.rgb_xyz_matrix, self.exif_data)


# ------------------------------------------------------------------------------------- dataset

class BurstSRProcessing:
    """processing.py:126-278 with the evaluation settings of get_burstsr_val_set (burstsr_dataset.py:294-302):
    crop to crop_sz (centre, or seeded random) if needed, black level subtracted, /norm_factor, no flip, no
    synthetic noise; the ground truth is scaled by the exposure ratio (light factors exposure * ISO / f^2)."""

    def __init__(self, crop_sz=80, substract_black_level=True, white_balance=False, random_crop=False, seed=0):
        self.crop_sz = crop_sz
        self.substract_black_level = substract_black_level
        self.white_balance = white_balance
        self.random_crop = random_crop
        self.rng = np.random.default_rng(seed)

    def __call__(self, frames, gt):
        if frames[0].shape()[-1] != self.crop_sz:
            H, W = frames[0].shape()[-2:]
            if self.random_crop:
                r1 = int(self.rng.integers(0, H - self.crop_sz + 1))
                c1 = int(self.rng.integers(0, W - self.crop_sz + 1))
            else:
                r1, c1 = (H - self.crop_sz) // 2, (W - self.crop_sz) // 2
            r2, c2 = r1 + self.crop_sz, c1 + self.crop_sz
            sf = gt.shape()[-1] // frames[0].shape()[-1]
            frames = [im.get_crop(r1, r2, c1, c2) for im in frames]
            gt = gt.get_crop(sf * r1, sf * r2, sf * c1, sf * c2)
        burst = torch.stack([im.get_image_data(normalize=True, substract_black_level=self.substract_black_level,
                                               white_balance=self.white_balance) for im in frames], 0)
        gt_data = gt.get_image_data(normalize=True, white_balance=self.white_balance,
                                    substract_black_level=self.substract_black_level)
        lf_burst = frames[0].get_exposure_time() * frames[0].get_iso() / (frames[0].get_f_number() ** 2)
        lf_canon = gt.get_exposure_time() * gt.get_iso() / (gt.get_f_number() ** 2)
        exp_scale = lf_burst / lf_canon
        return burst.float(), (gt_data * exp_scale).float(), {'exp_scale_factor': exp_scale}


class BurstSRDataset(torch.utils.data.Dataset):
    """burstsr_dataset.py:243-291 + sampler.IndexedBurst (sampler.py:99-150) for evaluation: root/split/<burst>/
    samsung_00..13 and canon.  `seq_ids`: sequence-id prefixes (burst name[:4]) to keep -- the reference
    takes them from data_specs/burstsr_<split>.txt; pass that list (or None for every burst on disk).
    Frame order: the base frame 0 then frames 1..13 (the reference samples 1..13 in an unseeded random
    order; fusion is permutation-invariant, so only the summation order differs)."""

    def __init__(self, root, split='val', seq_ids=None, burst_size=14, processing=None):
        self.root, self.split, self.burst_size = root, split, burst_size
        names = sorted(os.listdir(os.path.join(root, split)))
        if seq_ids is not None:
            names = [b for b in names if b[:4] in set(seq_ids)]
        self.burst_list = names
        self.processing = processing or BurstSRProcessing(crop_sz=80, substract_black_level=True)

    def __len__(self):
        return len(self.burst_list)

    def __getitem__(self, idx):
        d = os.path.join(self.root, self.split, self.burst_list[idx])
        frames = [SamsungRAWImage.load(os.path.join(d, 'samsung_{:02d}'.format(i))) for i in range(self.burst_size)]
        gt = CanonImage.load(os.path.join(d, 'canon'))
        burst, gt_data, info = self.processing(frames, gt)
        info['burst_name'] = self.burst_list[idx]
        return burst, gt_data, info


def write_burstsr_sample(root, name, frames_raw, gt_raw, meta_samsung, meta_canon, split='val'):
    """Write one burst in the BurstSR directory layout (im_raw.png via the cv2-convention codec +
    meta_info.json): frames_raw uint16 [N, 4, h, w], gt_raw uint16 [3, H, W].  For tests / demos; the
    real dataset's meta_info.pkl is read by `load_meta`."""
    d = os.path.join(root, split, name)
    for i, fr in enumerate(frames_raw):
        p = os.path.join(d, 'samsung_{:02d}'.format(i))
        os.makedirs(p, exist_ok=True)
        imwrite(os.path.join(p, 'im_raw.png'), np.transpose(np.asarray(fr, dtype=np.uint16), (1, 2, 0)))
        with open(os.path.join(p, 'meta_info.json'), 'w') as f:
            json.dump(meta_samsung, f)
    p = os.path.join(d, 'canon')
    os.makedirs(p, exist_ok=True)
    imwrite(os.path.join(p, 'im_raw.png'), np.transpose(np.asarray(gt_raw, dtype=np.uint16), (1, 2, 0)))
    with open(os.path.join(p, 'meta_info.json'), 'w') as f:
        json.dump(meta_canon, f)


# ------------------------------------------------------------------------------------- harness

def compute_score_burstsr(net, dataset, alignment_net, boundary_ignore=40, burst_sz=None, device='cuda'):
    """compute_score.py:96-134 (PSNR column): per burst net(burst) -> quantise to 2^14 -> spatial + colour
    alignment to the ground truth -> PSNR over the valid mask with boundary_ignore; mean over the set.
    Returns {'psnr': mean, 'per_image': {burst_name: psnr}}."""
    sca = SpatialColorAlignment(alignment_net, sr_factor=4)
    psnr_fn = PSNR(boundary_ignore=boundary_ignore)
    per = {}
    for idx in range(len(dataset)):
        burst, gt, info = dataset[idx]
        burst = burst.unsqueeze(0).to(device)
        gt = gt.unsqueeze(0).to(device)
        if burst_sz is not None:
            burst = burst[:, :burst_sz]
        with torch.no_grad():
            pred, _ = net(burst)
            pred = quantize_prediction(pred.float())
            pred_m, valid = sca(pred, gt, burst)
        per[info['burst_name']] = float(psnr_fn(pred_m, gt, valid=valid))
    return {'psnr': sum(per.values()) / max(1, len(per)), 'per_image': per}
