"""Generate the golden fixtures under tests/golden/ by running the REFERENCE implementation.

Runs only in the build container (needs /root/reference; the GPU box never runs this).  The
reference is imported read-only with three in-process stubs, exactly as SURVEY.md §8(c) describes:
  cupy        -- only `cupy.util.memoize` is touched at import (correlation.py:5,273)
  lpips       -- imported by models/loss/image_quality_v2.py:21, unused on the forward path
  admin.local -- environment.py:42-50 would otherwise try to write admin/local.py into the tree
The reference has no CPU correlation (correlation.py:324-325), so `FunctionCorrelation` is
monkeypatched with the oracle's K2 restatement (oracle/dbsr_oracle.py::correlation); everything
else (convs, grid_sample, interpolate, softmax, pixel_shuffle) executes reference code on torch-CPU.
PWC-Net is built with load_pretrained=False (no weights offline) and all weights come from
dbsr_amd.weights.generate_state_dict(seed=0).

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
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


def _install_stubs():
    cupy = types.ModuleType('cupy')
    cupy.util = types.SimpleNamespace(memoize=lambda **kw: (lambda f: f))
    sys.modules['cupy'] = cupy
    sys.modules['lpips'] = types.ModuleType('lpips')
    loc = types.ModuleType('admin.local')

    class EnvironmentSettings:
        def __init__(self):
            self.pretrained_nets_dir = '/nonexistent'
            self.workspace_dir = '/tmp'
    loc.EnvironmentSettings = EnvironmentSettings
    sys.modules['admin.local'] = loc


def quantize(pred):
    """evaluation/synburst/compute_score.py:110-111: (clamp(0,1)*2^14).short()."""
    return (pred.clamp(0.0, 1.0) * 2 ** 14).short().numpy().astype(np.uint16)


def quantize_f(pred):
    return (pred.clamp(0.0, 1.0) * 2 ** 14).short().float() / 2 ** 14


def main():
    sys.path.insert(0, REPO)
    from oracle import dbsr_oracle as orc
    import dbsr_amd
    from dbsr_amd import arch
    from dbsr_amd.weights import generate_state_dict
    from dbsr_amd.burst import synthetic_bursts

    _install_stubs()
    sys.path.insert(0, REF)
    import models.alignment.pwcnet as ref_pwc
    import models.dbsr.dbsrnet as ref_dbsrnet
    import models.layers.warp as ref_warp
    import models.layers.upsampling as ref_up

    ref_pwc.correlation.FunctionCorrelation = lambda tenFirst, tenSecond: orc.correlation(tenFirst, tenSecond)
    ref_dbsrnet.PWCNet = lambda load_pretrained=True, weights_path=None: ref_pwc.PWCNet(load_pretrained=False)

    torch.manual_seed(0)
    torch.set_num_threads(os.cpu_count())
    kw = dict(orc.DBSR_SYNTHETIC_KWARGS)
    ref_net = ref_dbsrnet.dbsrnet_cvpr2021(**kw).eval()
    mine = dbsr_amd.dbsrnet_cvpr2021(**kw)
    shapes = arch.state_dict_shapes(mine)
    ref_shapes = arch.state_dict_shapes(ref_net)
    assert list(shapes.keys()) == list(ref_shapes.keys()) and shapes == ref_shapes, 'state_dict mismatch'
    sd = generate_state_dict(shapes, seed=0)
    ref_net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})

    out = {}
    # ---------------- end-to-end forwards ----------------
    cases = [('e2e_b1n4', 1, 4, 48, 48, 11, False),
             ('e2e_b1n14', 1, 14, 48, 48, 12, False),
             ('e2e_b2n4_zeroflow', 2, 4, 48, 48, 13, True),
             ('e2e_b1n3_h40w56', 1, 3, 40, 56, 14, False)]
    for name, B, N, H, W, seed, zf in cases:
        burst, gt = synthetic_bursts(B, N, H, W, sr_factor=8, seed=seed)
        if zf:
            saved = ref_net.encoder.alignment_net.forward
            ref_net.encoder.alignment_net.forward = lambda s, t: torch.zeros(s.shape[0], 2, s.shape[-2], s.shape[-1])
        with torch.no_grad():
            pred, aux = ref_net(burst)
            enc = ref_net.encoder(burst)
            fused = ref_net.merging(enc)['fused_enc']
        if zf:
            ref_net.encoder.alignment_net.forward = saved
        fw = aux['fusion_weights']
        # ground truth stored as uint16 (/65535): torch's CPU randn differs across CPU ISAs, so the
        # GPU box cannot regenerate it bit-identically
        gt_u16 = (gt.clamp(0, 1) * 65535).round().to(torch.int32).numpy().astype(np.uint16)
        gt = torch.from_numpy(gt_u16.astype(np.float32)) / 65535.0
        psnr = [float(10 * torch.log10(1.0 / ((p - q)[..., 40:-40, 40:-40] ** 2).mean()))
                for p, q in zip(quantize_f(pred), gt)]           # image_quality_v2.py:69-101, bi=40
        d = dict(burst=burst.numpy(), seed=np.int64(seed), ref_psnr=np.array(psnr, dtype=np.float64),
                 pred_crop=pred[..., 100:164, 100:164].numpy(),
                 offsets=aux['offsets'].numpy(),
                 fused_crop=fused[:, :64, 8:24, 8:24].numpy(),
                 fw_sum=fw.double().sum(dim=(-2, -1)).float().numpy(),          # [B,N,C]
                 fw_crop=fw[:, :, :16, 8:16, 8:16].numpy(),
                 pred_sum=pred.double().sum(dim=(-2, -1)).float().numpy(),
                 zero_flow=np.array(zf))
        if name in ('e2e_b1n14', 'e2e_b1n4'):
            d['gt_u16'] = gt_u16
        if name == 'e2e_b1n14':
            d['pred_q'] = quantize(pred)
        out[name] = d
        print(name, 'pred mean', float(pred.mean()), 'offs absmax', float(aux['offsets'].abs().max()),
              'fused std', float(fused.std()))

    # ---------------- per-op fixtures ----------------
    g = torch.Generator().manual_seed(123)
    ops = {}
    # correlation (no reference CPU impl: fixture = K2 loop transliteration, pinned by source text)
    f1 = torch.randn(2, 40, 3, 5, generator=g)
    f2 = torch.randn(2, 40, 3, 5, generator=g)
    ops['corr_f1'], ops['corr_f2'] = f1.numpy(), f2.numpy()
    ops['corr_out'] = orc.correlation_loops(f1, f2).numpy()
    # backwarp (reference pwcnet.backwarp), flows reaching past the border, incl. w=2 level
    for tag, (P, C, h, w, s) in {'bw8': (3, 6, 8, 8, 2.5), 'bw2': (2, 5, 2, 2, 0.625)}.items():
        x = torch.randn(P, C, h, w, generator=g)
        fl = torch.randn(P, 2, h, w, generator=g) * 1.5
        fl[0, :, 0, 0] = 0.0
        fl[0, 0, 1, 1] = 0.3
        ops[f'{tag}_x'], ops[f'{tag}_flow'], ops[f'{tag}_scale'] = x.numpy(), fl.numpy(), np.float32(s)
        ops[f'{tag}_out'] = ref_pwc.backwarp(x.clone(), fl * s).numpy()
    # warp (reference models/layers/warp.py)
    x = torch.randn(3, 16, 12, 10, generator=g)
    fl = torch.randn(3, 2, 12, 10, generator=g) * 3.0
    fl[1] = 0.0
    ops['warp_x'], ops['warp_flow'] = x.numpy(), fl.numpy()
    ops['warp_out'] = ref_warp.warp(x, fl).numpy()
    # PixShuffleUpsampler (pixel shuffle + gauss blur), reference module with seeded weights
    up = ref_up.PixShuffleUpsampler(16, 4, upsample_factor=4, icnrinit=True, gauss_blur_sd=1.0)
    wgt = torch.randn(up.conv_layer[0].weight.shape, generator=g) * 0.3
    up.conv_layer[0].weight.data.copy_(wgt)
    x = torch.randn(2, 16, 6, 5, generator=g)
    with torch.no_grad():
        ops['up_w'], ops['up_x'], ops['up_out'] = wgt.numpy(), x.numpy(), up(x).numpy()
    # PWCNet alone (the alignment sub-seam), 48x48 -> offsets
    src = torch.rand(2, 3, 48, 48, generator=g)
    tgt = torch.rand(2, 3, 48, 48, generator=g)
    with torch.no_grad():
        ops['pwc_src'], ops['pwc_tgt'] = src.numpy(), tgt.numpy()
        ops['pwc_flow'] = ref_net.encoder.alignment_net(src, tgt).numpy()
    out['ops'] = ops

    for name, d in out.items():
        np.savez_compressed(os.path.join(HERE, name + '.npz'), **d)
    tot = sum(os.path.getsize(os.path.join(HERE, n + '.npz')) for n in out)
    print('wrote', list(out), 'total bytes', tot)


if __name__ == '__main__':
    main()
