"""Generate tests/golden/eval.npz by running the REFERENCE metric code (models/loss/image_quality_v2.py).

Build container only (needs /root/reference).  Same in-process import stubs as make_golden.py
(SURVEY.md §8c).  Inputs are seeded numpy arrays; outputs are the reference's PSNR / PixelWiseError
values, and the compute_score quantisation (compute_score.py:109-111) of a seeded prediction.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_eval.py
"""
import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REF = '/root/reference'

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    sys.path.insert(0, HERE)
    import make_golden
    make_golden._install_stubs()
    sys.path.insert(0, REF)
    from models.loss.image_quality_v2 import PSNR, PixelWiseError

    rng = np.random.default_rng(7)
    d = {}
    gt = rng.random((3, 3, 96, 104), dtype=np.float32)
    pred = np.clip(gt + rng.normal(0, 0.05, gt.shape).astype(np.float32), -0.1, 1.2).astype(np.float32)
    pred[2] = gt[2]                                   # identical pair -> inf PSNR, dropped by PSNR.forward
    valid = (rng.random((3, 1, 96, 104)) > 0.3)
    d['gt'], d['pred'], d['valid'] = gt, pred, valid
    tp, tg, tv = torch.from_numpy(pred), torch.from_numpy(gt), torch.from_numpy(valid)
    d['psnr_b40'] = np.float64(PSNR(boundary_ignore=40)(tp, tg))
    d['psnr_none'] = np.float64(PSNR()(tp[:2], tg[:2]))
    d['psnr_b8_valid'] = np.float64(PSNR(boundary_ignore=8)(tp[:2], tg[:2], tv[:2]))
    d['psnr_b40_maxnone'] = np.float64(PSNR(boundary_ignore=40, max_value=None)(tp[:2], tg[:2]))
    for m in ('l1', 'l2', 'l2_sqrt', 'charbonnier'):
        d['err_' + m] = np.float64(PixelWiseError(metric=m, boundary_ignore=40)(tp, tg))
    # compute_score.py:109-111 quantisation of an unclamped prediction
    q = torch.from_numpy(pred)
    d['quantized'] = ((q.clamp(0.0, 1.0) * 2 ** 14).short().float() / (2 ** 14)).numpy()
    np.savez_compressed(os.path.join(HERE, 'eval.npz'), **d)
    print({k: (v if np.ndim(v) == 0 else v.shape) for k, v in d.items()})


if __name__ == '__main__':
    main()
