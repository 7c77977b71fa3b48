"""CPU emulation of the engine's 16-bit storage points on the oracle: RMS / max of (pred_emulated - pred_fp32)
per storage dtype and per fp32 island, to choose the precision design (RMS <= 5.3e-4 is the
error that moves the reference's published 39.17 dB by 0.01 dB).
Usage: python tools/precision_probe.py [B]"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import dbsr_oracle as orc   # noqa: E402
import dbsr_amd                           # noqa: E402
from dbsr_amd import arch                 # noqa: E402
from dbsr_amd.weights import generate_state_dict   # noqa: E402
from dbsr_amd.burst import synthetic_bursts         # noqa: E402


def run(burst, sd, dt, fp32=(), w32=False, resid32=False):
    rnd = (lambda t: t.to(dt).float()) if dt is not None else (lambda t: t)
    keep = lambda name: any(name.startswith(p) for p in fp32)
    o_conv, o_res, o_warp, o_mer = orc.conv, orc.res_block, orc.warp, orc.merging

    def conv(x, sd_, name, stride=1, padding=1, dilation=1):
        r = (lambda t: t) if keep(name) else rnd
        return F.conv2d(r(x), (r if keep(name) else ((lambda t: t) if (w32 is True or (w32 and any(name.startswith(q) for q in w32))) else rnd))(sd_[name + '.weight']), sd_.get(name + '.bias'), stride=stride, padding=padding,
                        dilation=dilation)

    def res_block(x, sd_, name):
        out = F.relu(conv(x, sd_, name + '.conv1.0'))
        out = conv(out, sd_, name + '.conv2.0')
        y = F.relu(out + (x if keep(name) or resid32 else rnd(x)))
        return y if keep(name) or resid32 else rnd(y)

    def warp(feat, flow, **kw):
        return rnd(o_warp(rnd(feat), flow, **kw))

    def merging(x, sd_, kw, return_logits=False):
        all_feat, w = o_mer(x, sd_, kw, return_logits=True)
        wn = F.softmax(rnd(w), dim=1)
        return {'fused_enc': rnd((rnd(all_feat) * wn).sum(dim=1)), 'fusion_weights': wn}
    orc.conv, orc.res_block, orc.warp, orc.merging = conv, res_block, warp, merging
    try:
        with torch.no_grad():
            p, aux = orc.dbsr_forward(burst, sd)
            return p, aux['offsets']
    finally:
        orc.conv, orc.res_block, orc.warp, orc.merging = o_conv, o_res, o_warp, o_mer


def main():
    torch.set_num_threads(os.cpu_count())
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    net = dbsr_amd.dbsrnet_cvpr2021(**dbsr_amd.DBSR_SYNTHETIC_KWARGS)
    sd = orc.state_dict_to_torch(generate_state_dict(arch.state_dict_shapes(net), seed=0))
    burst, gt = synthetic_bursts(B, 14, 48, 48, sr_factor=8, seed=101)
    ref, roffs = run(burst, sd, None)
    print('pred mean %.4f rms %.4f max %.4f' % (ref.mean(), ref.pow(2).mean().sqrt(), ref.max()))
    variants = [
        ('bf16 all', torch.bfloat16, ()),
        ('fp16 all', torch.float16, ()),
        ('bf16, PWC fp32', torch.bfloat16, ('encoder.alignment_net',)),
        ('bf16, decoder fp32', torch.bfloat16, ('decoder',)),
        ('bf16, decoder.post fp32', torch.bfloat16, ('decoder.post', 'decoder.predictor')),
        ('fp16, PWC fp32', torch.float16, ('encoder.alignment_net',)),
        ('fp16, decoder.post fp32', torch.float16, ('decoder.post', 'decoder.predictor')),
    ]
    variants += [
        ('fp16, enc fp32', torch.float16, ('encoder.init', 'encoder.res', 'encoder.out')),
        ('fp16, merging fp32', torch.float16, ('merging',)),
        ('fp16, dec.init+pre fp32', torch.float16, ('decoder.init', 'decoder.pre')),
        ('fp16, dec.upsample fp32', torch.float16, ('decoder.upsample',)),
        ('fp16, dec.post.conv2 fp32', torch.float16, tuple('decoder.post_res_layers.%d.conv2' % i for i in range(4))),
        ('fp16, weights fp32', torch.float16, (), True),
        ('fp16, resid stream fp32', torch.float16, (), False, True),
        ('bf16, resid stream fp32', torch.bfloat16, (), False, True),
        ('bf16, weights fp32', torch.bfloat16, (), True),
        ('fp16, dec.post weights fp32', torch.float16, (), ('decoder.post',)),
        ('fp16, decoder weights fp32', torch.float16, (), ('decoder',)),
        ('fp16, dec+enc weights fp32', torch.float16, (), ('decoder', 'encoder.init', 'encoder.res', 'encoder.out')),
    ]
    for name, dt, fp32, *rest in variants:
        p, o = run(burst, sd, dt, fp32, *rest)
        d = p - ref
        dc = p.clamp(0, 1) - ref.clamp(0, 1)
        print('%-26s pred RMS %.3e max %.3e | clamped RMS %.3e | offsets max %.3e' % (
            name, d.pow(2).mean().sqrt(), d.abs().max(), dc.pow(2).mean().sqrt(), (o - roffs).abs().max()))


if __name__ == '__main__':
    main()
