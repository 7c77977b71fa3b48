"""CPU emulation of the engine's bf16 rounding points on the oracle, to rank precision upgrades.
Usage: python tools/bf16_sensitivity.py"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import dbsr_oracle as orc   # noqa: E402
import dbsr_amd                           # noqa: E402
from dbsr_amd import arch                 # noqa: E402
from dbsr_amd.weights import generate_state_dict   # noqa: E402

bf = lambda t: t.to(torch.bfloat16).float()


def run(burst, sd, fp32_layers=(), fp32_resid_prefix=()):
    orig_conv, orig_res = orc.conv, orc.res_block

    def conv(x, sd_, name, stride=1, padding=1, dilation=1):
        keep = any(name.startswith(p) for p in fp32_layers)
        w = sd_[name + '.weight'] if keep else bf(sd_[name + '.weight'])
        y = F.conv2d(x if keep else bf(x), w, sd_.get(name + '.bias'), stride=stride, padding=padding,
                     dilation=dilation)
        return y

    def res_block(x, sd_, name):
        out = F.relu(conv(x, sd_, name + '.conv1.0'))
        out = conv(bf(out), sd_, name + '.conv2.0')
        y = F.relu(out + x)
        return y if any(name.startswith(p) for p in fp32_resid_prefix) else bf(y)
    orc.conv, orc.res_block = conv, res_block
    try:
        with torch.no_grad():
            return orc.dbsr_forward(burst, sd)[0]
    finally:
        orc.conv, orc.res_block = orig_conv, orig_res


def psnr(pred, gt):
    q = (pred.clamp(0, 1) * 2 ** 14).short().float() / 2 ** 14
    return float(10 * torch.log10(1.0 / ((q - gt)[..., 40:-40, 40:-40] ** 2).mean()))


def main():
    torch.set_num_threads(os.cpu_count())
    net = dbsr_amd.dbsrnet_cvpr2021(**dbsr_amd.DBSR_SYNTHETIC_KWARGS)
    sd = orc.state_dict_to_torch(generate_state_dict(arch.state_dict_shapes(net), seed=0))
    variants = {
        'all bf16': dict(),
        'predictor fp32': dict(fp32_layers=('decoder.predictor',)),
        'pred + post resid fp32': dict(fp32_layers=('decoder.predictor',), fp32_resid_prefix=('decoder.post',)),
        'pred + upsample fp32': dict(fp32_layers=('decoder.predictor', 'decoder.upsample')),
        'decoder post convs fp32': dict(fp32_layers=('decoder.predictor', 'decoder.post')),
    }
    for name in ['e2e_b1n4', 'e2e_b1n14']:
        g = dict(np.load(f'tests/golden/{name}.npz'))
        burst = torch.from_numpy(g['burst'])
        gt = torch.from_numpy(g['gt_u16'].astype(np.float32)) / 65535
        ref = float(g['ref_psnr'][0])
        for vname, kw in variants.items():
            p = run(burst, sd, **kw)
            print(f'{name:10s} {vname:26s} dPSNR {psnr(p[0], gt[0]) - ref:+.5f} dB')


if __name__ == '__main__':
    main()
