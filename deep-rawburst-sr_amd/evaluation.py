"""Evaluation-harness counterpart for the DBSR forward.

The reference's SyntheticBurstVal scoring cannot run on this stack (dataset/synthetic_burst_val_set.py
needs cv2; evaluation/synburst/compute_score.py needs cv2, lpips and torch._six via the dataset
package).  This module restates the parts that decide the reported number, so a user of the reference
can score the drop-in network on the same files:

  * a 16-bit PNG codec with cv2's channel conventions (`imread_unchanged`, `imwrite`): cv2 stores
    arrays as BGR(A), so the on-disk RGB(A) planes are the array's channels in [2,1,0(,3)] order
    (synthetic_burst_val_set.py:43-54 reads with cv2.IMREAD_UNCHANGED; save_results.py:63-67 writes
    with cv2.imwrite).  Pillow is not usable for this: it reduces 16-bit RGB(A) to 8 bits.
  * `SyntheticBurstVal` (synthetic_burst_val_set.py:20-79): bursts/NNNN/im_raw_KK.png (4-channel
    RGGB, /2^14), gt/NNNN/im_rgb.png (3-channel, /2^14).  meta_info.pkl is NOT unpickled here (it is
    only used for sRGB visualisation, which is out of scope); meta_info carries 'burst_name' only.
  * `quantize_prediction` (compute_score.py:109-111) and `PSNR` / `PixelWiseError`
    (models/loss/image_quality_v2.py:24-101), `compute_score` (compute_score.py:36-122, PSNR column)
    and `save_results` (save_results.py:36-67).

Host-side Python only: the network forward is the HIP path; metrics run as torch ops on whatever
device the predictions live on (they are reductions over one image, not part of the hot path).
"""
import math
import os
import struct
import zlib

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

_PNG_SIG = b'\x89PNG\r\n\x1a\n'
_COLOR_CHANNELS = {0: 1, 2: 3, 4: 2, 6: 4}       # PNG colour type -> samples per pixel


# ------------------------------------------------------------------------------------------ PNG codec

def _paeth(a, b, c):
    p = a + b - c
    pa, pb, pc = np.abs(p - a), np.abs(p - b), np.abs(p - c)
    return np.where((pa <= pb) & (pa <= pc), a, np.where(pb <= pc, b, c))


def png_read(path):
    """Decode a non-interlaced 8/16-bit gray/gray-alpha/RGB/RGBA PNG into an [H,W,C] array holding the
    FILE's channel order (uint8 or uint16).  Raises ValueError on anything else (palette,
    interlace, bit depths < 8), which SyntheticBurstVal/BurstSR files never use."""
    with open(path, 'rb') as f:
        data = f.read()
    if data[:8] != _PNG_SIG:
        raise ValueError(f'{path}: not a PNG file')
    pos, idat, hdr = 8, [], None
    while pos < len(data):
        ln, typ = struct.unpack('>I4s', data[pos:pos + 8])
        body = data[pos + 8:pos + 8 + ln]
        if zlib.crc32(typ + body) & 0xffffffff != struct.unpack('>I', data[pos + 8 + ln:pos + 12 + ln])[0]:
            raise ValueError(f'{path}: CRC mismatch in {typ!r} chunk')
        if typ == b'IHDR':
            hdr = struct.unpack('>IIBBBBB', body)
        elif typ == b'IDAT':
            idat.append(body)
        elif typ == b'IEND':
            break
        pos += 12 + ln
    if hdr is None:
        raise ValueError(f'{path}: missing IHDR')
    w, h, depth, ctype, _, _, interlace = hdr
    if depth not in (8, 16) or ctype not in _COLOR_CHANNELS or interlace != 0:
        raise ValueError(f'{path}: unsupported PNG (depth {depth}, colour type {ctype}, interlace {interlace})')
    ch = _COLOR_CHANNELS[ctype]
    bpp = ch * depth // 8
    stride = w * bpp
    raw = np.frombuffer(zlib.decompress(b''.join(idat)), dtype=np.uint8)
    if raw.size != h * (stride + 1):
        raise ValueError(f'{path}: image data size {raw.size} != {h}*({stride}+1)')
    rows = raw.reshape(h, stride + 1)
    out = np.zeros((h, stride), dtype=np.uint8)
    prev = np.zeros(stride, dtype=np.int32)
    for y in range(h):
        ft, line = rows[y, 0], rows[y, 1:].astype(np.int32)
        if ft == 0:
            cur = line
        elif ft == 1:     # Sub: running sum along the row, per byte lane of a pixel
            cur = np.cumsum(line.reshape(w, bpp), axis=0).reshape(-1) & 0xff
        elif ft == 2:     # Up
            cur = (line + prev) & 0xff
        elif ft in (3, 4):  # Average / Paeth: sequential along the row, vectorised over the pixel's bytes
            cur = np.empty(stride, dtype=np.int32)
            left = np.zeros(bpp, dtype=np.int32)
            upleft = np.zeros(bpp, dtype=np.int32)
            for x in range(0, stride, bpp):
                up = prev[x:x + bpp]
                pred = (left + up) >> 1 if ft == 3 else _paeth(left, up, upleft)
                left = (line[x:x + bpp] + pred) & 0xff
                cur[x:x + bpp] = left
                upleft = up
        else:
            raise ValueError(f'{path}: bad filter type {ft} in row {y}')
        out[y] = cur
        prev = cur
    if depth == 16:
        return out.view('>u2').astype(np.uint16).reshape(h, w, ch)
    return out.reshape(h, w, ch)


def png_write(path, img, filter_type=0, level=6):
    """Encode an [H,W] or [H,W,C] uint8/uint16 array (FILE channel order, C in 1..4) as a PNG.
    `filter_type` 0..4 applies that filter to every row (tests use it to cover the decoder)."""
    img = np.ascontiguousarray(img)
    if img.ndim == 2:
        img = img[:, :, None]
    h, w, ch = img.shape
    if img.dtype == np.uint16:
        depth, buf = 16, img.astype('>u2').view(np.uint8)
    elif img.dtype == np.uint8:
        depth, buf = 8, img
    else:
        raise ValueError(f'png_write: dtype {img.dtype} (want uint8 or uint16)')
    ctype = {1: 0, 2: 4, 3: 2, 4: 6}[ch]
    bpp = ch * depth // 8
    cur = buf.reshape(h, w * bpp).astype(np.int32)
    up = np.vstack([np.zeros((1, w * bpp), np.int32), cur[:-1]])
    left = np.hstack([np.zeros((h, bpp), np.int32), cur[:, :-bpp]])
    upleft = np.hstack([np.zeros((h, bpp), np.int32), up[:, :-bpp]])
    pred = {0: 0, 1: left, 2: up, 3: (left + up) >> 1, 4: _paeth(left, up, upleft)}[filter_type]
    filt = ((cur - pred) & 0xff).astype(np.uint8)
    raw = np.hstack([np.full((h, 1), filter_type, np.uint8), filt]).tobytes()

    def chunk(typ, body):
        return struct.pack('>I', len(body)) + typ + body + struct.pack('>I', zlib.crc32(typ + body) & 0xffffffff)
    with open(path, 'wb') as f:
        f.write(_PNG_SIG + chunk(b'IHDR', struct.pack('>IIBBBBB', w, h, depth, ctype, 0, 0, 0))
                + chunk(b'IDAT', zlib.compress(raw, level)) + chunk(b'IEND', b''))


def _bgr_order(ch):
    return [2, 1, 0, 3][:ch] if ch >= 3 else list(range(ch))


def imread_unchanged(path):
    """cv2.imread(path, cv2.IMREAD_UNCHANGED): [H,W] for gray, else [H,W,C] in BGR(A) order."""
    img = png_read(path)
    if img.shape[2] == 1:
        return img[:, :, 0]
    return np.ascontiguousarray(img[:, :, _bgr_order(img.shape[2])])


def imwrite(path, img):
    """cv2.imwrite(path, img) for PNG: the array is BGR(A), the file stores RGB(A)."""
    img = np.asarray(img)
    if img.ndim == 3 and img.shape[2] >= 3:
        img = img[:, :, _bgr_order(img.shape[2])]
    png_write(path, img)


# ------------------------------------------------------------------------------------------ dataset

class SyntheticBurstVal(torch.utils.data.Dataset):
    """dataset/synthetic_burst_val_set.py:20-79 (cv2 replaced by `imread_unchanged`)."""

    def __init__(self, root, initialize=True, burst_size=14, num_bursts=None):
        self.root = root
        if num_bursts is None:   # the reference hard-codes 300 (:32); count what is on disk instead
            bdir = os.path.join(root, 'bursts')
            num_bursts = len([d for d in os.listdir(bdir) if d.isdigit()]) if os.path.isdir(bdir) else 300
        self.burst_list = list(range(num_bursts))
        self.burst_size = burst_size

    def initialize(self):
        pass

    def __len__(self):
        return len(self.burst_list)

    def _read_burst_image(self, index, image_id):
        im = imread_unchanged('{}/bursts/{:04d}/im_raw_{:02d}.png'.format(self.root, index, image_id))
        return torch.from_numpy(im.astype(np.float32)).permute(2, 0, 1).float() / (2 ** 14)

    def _read_gt_image(self, index):
        gt = imread_unchanged('{}/gt/{:04d}/im_rgb.png'.format(self.root, index))
        return (torch.from_numpy(gt.astype(np.float32)) / 2 ** 14).permute(2, 0, 1).float()

    def __getitem__(self, index):
        burst = torch.stack([self._read_burst_image(index, i) for i in range(self.burst_size)], 0)
        gt = self._read_gt_image(index)
        return burst, gt, {'burst_name': '{:04d}'.format(index)}


def write_synthetic_burst_val(root, bursts, gts, start=0):
    """Write bursts [B,N,4,H,W] and gts [B,3,sH,sW] (values in [0,1]) in the SyntheticBurstVal layout,
    quantised to 2^14 the way the dataset's PNGs are.  Used to exercise the reader and the scorer
    without the (unavailable) dataset."""
    for b in range(bursts.shape[0]):
        name = '{:04d}'.format(start + b)
        os.makedirs(os.path.join(root, 'bursts', name), exist_ok=True)
        os.makedirs(os.path.join(root, 'gt', name), exist_ok=True)
        for i in range(bursts.shape[1]):
            im = (bursts[b, i].permute(1, 2, 0).clamp(0, 1) * 2 ** 14).round().numpy().astype(np.uint16)
            imwrite(os.path.join(root, 'bursts', name, 'im_raw_{:02d}.png'.format(i)), im)
        gt = (gts[b].permute(1, 2, 0).clamp(0, 1) * 2 ** 14).round().numpy().astype(np.uint16)
        imwrite(os.path.join(root, 'gt', name, 'im_rgb.png'), gt)


# ------------------------------------------------------------------------------------------ metrics

def quantize_prediction(pred):
    """compute_score.py:109-111: (clamp(0,1)*2^14).short() / 2^14."""
    return (pred.clamp(0.0, 1.0) * 2 ** 14).short().float() / (2 ** 14)


class PixelWiseError(nn.Module):
    """models/loss/image_quality_v2.py:24-66."""

    def __init__(self, metric='l1', boundary_ignore=None):
        super().__init__()
        self.boundary_ignore = boundary_ignore
        if metric == 'l1':
            self.loss_fn = F.l1_loss
        elif metric == 'l2':
            self.loss_fn = F.mse_loss
        elif metric == 'l2_sqrt':
            self.loss_fn = lambda pred, gt: (((pred - gt) ** 2).sum(dim=-3)).sqrt().mean()
        elif metric == 'charbonnier':
            self.loss_fn = lambda pred, gt: ((pred - gt) ** 2 + 1e-3 ** 2).sqrt().mean()
        else:
            raise ValueError(f'unknown metric {metric!r}')

    def forward(self, pred, gt, valid=None):
        if self.boundary_ignore is not None:
            bi = self.boundary_ignore
            pred = pred[..., bi:-bi, bi:-bi]
            gt = gt[..., bi:-bi, bi:-bi]
            if valid is not None:
                valid = valid[..., bi:-bi, bi:-bi]
        if valid is None:
            return self.loss_fn(pred, gt)
        err = self.loss_fn(pred, gt, reduction='none')
        elem_ratio = err.numel() / valid.numel()
        return (err * valid.float()).sum() / (valid.float().sum() * elem_ratio + 1e-12)


class PSNR(nn.Module):
    """models/loss/image_quality_v2.py:69-101: per-image PSNR, inf/nan images dropped, then the mean."""

    def __init__(self, boundary_ignore=None, max_value=1.0):
        super().__init__()
        self.l2 = PixelWiseError(metric='l2', boundary_ignore=boundary_ignore)
        self.max_value = max_value

    def psnr(self, pred, gt, valid=None):
        mse = self.l2(pred, gt, valid=valid)
        if self.max_value is not None:
            return 20 * math.log10(self.max_value) - 10.0 * mse.log10()
        return 20 * gt.max().log10() - 10.0 * mse.log10()

    def forward(self, pred, gt, valid=None):
        if valid is None:
            vals = [self.psnr(p.unsqueeze(0), g.unsqueeze(0)) for p, g in zip(pred, gt)]
        else:
            vals = [self.psnr(p.unsqueeze(0), g.unsqueeze(0), v.unsqueeze(0)) for p, g, v in zip(pred, gt, valid)]
        vals = [p for p in vals if not (torch.isinf(p) or torch.isnan(p))]
        return 0 if not vals else sum(vals) / len(vals)


# ------------------------------------------------------------------------------------------ harness

def _batches(dataset, batch, burst_sz):
    for s in range(0, len(dataset), batch):
        items = [dataset[i] for i in range(s, min(s + batch, len(dataset)))]
        bursts = torch.stack([it[0] for it in items])
        if burst_sz is not None:
            bursts = bursts[:, :burst_sz]
        yield bursts, torch.stack([it[1] for it in items]), [it[2]['burst_name'] for it in items]


def compute_score(net, dataset, boundary_ignore=40, burst_sz=None, device='cuda', batch=8):
    """PSNR column of evaluation/synburst/compute_score.py:36-122 for one network: forward each
    burst, quantise like :109-111, per-image PSNR with `boundary_ignore`, mean over the set.
    Bursts go through the engine `batch` at a time (bursts are independent); scores stay per image.
    Returns {'psnr': mean, 'per_image': {burst_name: psnr}}."""
    psnr_fn = PSNR(boundary_ignore=boundary_ignore)
    per = {}
    for bursts, gts, names in _batches(dataset, batch, burst_sz):
        with torch.no_grad():
            pred, _ = net(bursts.to(device))
        pred = quantize_prediction(pred.float())
        gts = gts.to(pred.device)
        for i, name in enumerate(names):
            per[name] = float(psnr_fn(pred[i:i + 1], gts[i:i + 1]))
    return {'psnr': sum(per.values()) / max(1, len(per)), 'per_image': per}


def save_results(net, dataset, out_dir, burst_sz=None, device='cuda', batch=8):
    """evaluation/synburst/save_results.py:36-67: uint16 PNG of clamp(pred,0,1)*2^14 per burst, written
    the way cv2.imwrite writes an [H,W,3] array (array channels read as BGR)."""
    os.makedirs(out_dir, exist_ok=True)
    for bursts, _, names in _batches(dataset, batch, burst_sz):
        with torch.no_grad():
            pred, _ = net(bursts.to(device))
        arr = (pred.float().permute(0, 2, 3, 1).clamp(0.0, 1.0) * 2 ** 14).cpu().numpy().astype(np.uint16)
        for i, name in enumerate(names):
            imwrite('{}/{}.png'.format(out_dir, name), arr[i])


def load_saved_prediction(path):
    """compute_score.py:102-104: a saved prediction back to [1,3,H,W] float /2^14."""
    im = imread_unchanged(path)
    return (torch.from_numpy(im.astype(np.float32)) / 2 ** 14).permute(2, 0, 1).float().unsqueeze(0)
