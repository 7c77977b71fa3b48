"""Generate tests/golden/burstsr.npz by running the REFERENCE SpatialColorAlignment
(models/loss/spatial_color_alignment.py:23-108) on torch-CPU.

Build container only (needs /root/reference).  Same in-process import stubs as make_golden.py (SURVEY.md
§8c), plus two stand-ins the reference needs on torch 2.10:
  * torch.lstsq (removed in torch 2.x; spatial_color_alignment.py:40) -> the least-squares solution of
    torch.linalg.lstsq, returned as `.solution` with the row layout torch.lstsq had ((max(m, n), k), the
    first n rows the solution; the reference keeps [:3]).  For the full-rank systems here the
    least-squares solution is unique, so the shim changes no result beyond rounding.
  * FunctionCorrelation -> the oracle's K2 restatement (as make_golden.py).
PWC-Net weights: the alignment-net part of dbsr_amd.weights.generate_state_dict(seed=0) (the same
weights the e2e fixtures use).

Fixture parts:
  A) the whole SCA forward on a synthetic 128x128 prediction / ground truth / 16x16 base frame: flow,
     pred_warped_m, valid;
  B) match_colors alone on 48x48 smooth images related by a known 3x3 colour matrix + noise and a
     corrupted patch (a well-posed fit; mask upsampled x2 to a 96x96 test image):
     c_mat, output, valid.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_burstsr.py
"""
import os
import sys
import types

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = '/root/reference'

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def smooth_image(rng, n, h, w):
    """Sum of low-frequency sinusoids per channel, in [0.05, 0.95]."""
    yy, xx = np.meshgrid(np.linspace(0, 1, h), np.linspace(0, 1, w), indexing='ij')
    out = np.zeros((n, 3, h, w), np.float32)
    for b in range(n):
        for c in range(3):
            acc = np.zeros((h, w))
            for _ in range(4):
                fy, fx, ph = rng.uniform(0.5, 3.0), rng.uniform(0.5, 3.0), rng.uniform(0, 2 * np.pi)
                acc += rng.uniform(0.2, 1.0) * np.sin(2 * np.pi * (fy * yy + fx * xx) + ph)
            acc = (acc - acc.min()) / (acc.max() - acc.min() + 1e-9)
            out[b, c] = 0.05 + 0.9 * acc
    return out


def main():
    sys.path.insert(0, HERE)
    sys.path.insert(0, REPO)
    import make_golden
    from oracle import dbsr_oracle as orc
    import dbsr_amd
    from dbsr_amd import arch
    from dbsr_amd.weights import generate_state_dict
    make_golden._install_stubs()

    solutions = []

    def lstsq(B, A):
        sol = torch.linalg.lstsq(A, B).solution
        solutions.append(sol.clone())
        m, n = A.shape
        full = torch.zeros(max(m, n), B.shape[1], dtype=sol.dtype)
        full[:n] = sol
        return types.SimpleNamespace(solution=full)
    torch.lstsq = lstsq

    sys.path.insert(0, REF)
    import models.alignment.pwcnet as ref_pwc
    import models.loss.spatial_color_alignment as ref_sca
    ref_pwc.correlation.FunctionCorrelation = lambda tenFirst, tenSecond: orc.correlation(tenFirst, tenSecond)

    torch.set_num_threads(os.cpu_count())
    net = dbsr_amd.dbsrnet_cvpr2021(**dbsr_amd.DBSR_SYNTHETIC_KWARGS)
    sd = generate_state_dict(arch.state_dict_shapes(net), seed=0)
    pre = 'encoder.alignment_net.'
    pwc = ref_pwc.PWCNet(load_pretrained=False).eval()
    pwc.load_state_dict({k[len(pre):]: torch.from_numpy(v) for k, v in sd.items() if k.startswith(pre)})

    rng = np.random.default_rng(11)
    d = {}
    # ---- A: the whole forward
    gt = torch.from_numpy(smooth_image(rng, 1, 128, 128))
    cm = torch.tensor([[0.9, 0.05, 0.0], [0.1, 1.05, 0.05], [0.0, -0.05, 0.95]])
    shifted = F.grid_sample(gt, F.affine_grid(torch.tensor([[[1.0, 0.0, 0.02], [0.0, 1.0, -0.015]]]), gt.shape,
                                              align_corners=False), align_corners=False, padding_mode='border')
    pred = torch.einsum('bkhw,kj->bjhw', shifted, cm) + torch.from_numpy(rng.normal(0, 0.005, gt.shape).astype(np.float32))
    pred = (pred.clamp(0, 1) * 2 ** 14).short().float() / 2 ** 14
    burst0 = F.interpolate(gt, scale_factor=1 / 8, mode='bilinear')           # the base frame's R, G, B
    burst = torch.stack([burst0[:, 0], burst0[:, 1], burst0[:, 1], burst0[:, 2]], 1).unsqueeze(1)
    burst = burst + torch.from_numpy(rng.normal(0, 0.002, burst.shape).astype(np.float32))
    sca = ref_sca.SpatialColorAlignment(pwc, sr_factor=4)
    with torch.no_grad():
        flow = pwc(pred / (pred.max() + 1e-6), gt / (gt.max() + 1e-6))
        solutions.clear()
        out, valid = sca(pred, gt, burst)
    d.update(a_pred=pred.numpy(), a_gt=gt.numpy(), a_burst=burst.numpy(), a_flow=flow.numpy(), a_out=out.numpy(),
             a_valid=valid.numpy(), a_cmat=torch.stack(solutions).numpy())
    print('A: |flow| max %.3f  valid %.3f  cmat %s' % (flow.abs().max(), valid.float().mean(), solutions[0].numpy().round(3)))

    # ---- B: match_colors alone, 2 images
    ref = torch.from_numpy(smooth_image(rng, 2, 48, 48))
    cms = torch.tensor([[[1.1, 0.1, -0.05], [0.0, 0.9, 0.1], [0.05, 0.0, 1.2]],
                        [[0.8, -0.1, 0.0], [0.2, 1.0, 0.0], [0.0, 0.1, 0.9]]])
    inv = torch.linalg.inv(cms)
    q = torch.einsum('bkhw,bkj->bjhw', ref, inv) + torch.from_numpy(rng.normal(0, 0.02, ref.shape).astype(np.float32))
    q[:, :, 20:28, 18:32] += 0.3                                              # a region the mask must reject
    test = torch.from_numpy(smooth_image(rng, 2, 96, 96))
    K, ksz = ref_sca.get_gaussian_kernel(sd=1.5)
    solutions.clear()
    out_b, valid_b = ref_sca.match_colors(ref, q, test, ksz, K)
    d.update(b_ref=ref.numpy(), b_q=q.numpy(), b_test=test.numpy(), b_out=out_b.numpy(), b_valid=valid_b.numpy(),
             b_cmat=torch.stack(solutions).numpy())
    print('B: valid %.3f' % valid_b.float().mean())
    np.savez_compressed(os.path.join(HERE, 'burstsr.npz'), **d)
    print('wrote', os.path.join(HERE, 'burstsr.npz'), os.path.getsize(os.path.join(HERE, 'burstsr.npz')))


if __name__ == '__main__':
    main()
