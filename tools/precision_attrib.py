"""Where the fp16 forward's error comes from: a CPU emulation of the engine's 16-bit storage points on
the oracle (oracle/dbsr_oracle.py), with one stage at a time kept in fp32, at configs[1]'s parity case (B=8, N=14,
48x48, seeded weights and bursts of tests/test_gpu_parity.py::bench_case).

Storage points emulated as the engine has them (DESIGN.md "Precision"): every conv's weights and stored output
(after its activation; a ResBlock's conv2 is stored only after the residual and ReLU) rounded to fp16, fp32
accumulation and bias; PWC-Net's flows fp32; the weight predictor's logits fp32 (conv_fuse keeps them in
registers) with an fp32 softmax; the fused embedding stored fp16; the upsampler's pre-blur tensor and the blurred
image stored fp16; the last post-ResBlock's output NOT rounded and the RGB predictor in fp32 (dbsr_resblock_head).

Stages (one kept fp32 per line -- its weights and its stored tensors):
  pwc       PWC-Net (alignment_net): features, DenseNet channels, correlation volumes
  enc       the frame encoder (init, ResBlocks, out): the embeddings E
  warp      the warped embeddings Wf
  merge     projections, offset-feature extractor, weight-predictor hidden layers
  fuse      the fused embedding
  dec.lr    the decoder's init conv + pre-ResBlocks (48x48)
  dec.up    the upsampler conv's output and the blurred image (384x384)
  dec.post  the post-ResBlocks (384x384)
Error shares are the quadrature drops (rms_all^2 - rms_without^2) / rms_all^2 (independent stage errors add in
quadrature; the shares need not sum to 1).

Usage: python tools/precision_attrib.py [B] [stage,stage,... to keep fp32 together]"""
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

STAGES = ('pwc', 'enc', 'warp', 'merge', 'fuse', 'dec.lr', 'dec.up', 'dec.post')


def stage_of(name):
    if name.startswith('encoder.alignment_net'):
        return 'pwc'
    if name.startswith('encoder.'):
        return 'enc'
    if name.startswith('merging.'):
        return 'merge'
    if name.startswith(('decoder.init_layer', 'decoder.pre_res_layers')):
        return 'dec.lr'
    if name.startswith('decoder.upsample_layer'):
        return 'dec.up'
    if name.startswith(('decoder.post_res_layers', 'decoder.predictor')):
        return 'dec.post'
    raise KeyError(name)


def diffuse_round(w, dt):
    """Weight rounding to dt with the rounding error diffused along each output channel's K (taps x input channels):
    q_k = round(w_k - e_k), e_{k+1} = e_k + q_k - w_k, so every q_k is one of w_k's two nearest dt neighbours'
    neighbourhood (|q_k - w_k| <= 1 ulp) and the sum of a channel's errors stays within half an ulp -- the error
    a constant input component sees (ReLU activations have a large common mean) cancels instead of adding up."""
    co = w.shape[0]
    f = w.permute(0, 2, 3, 1).reshape(co, -1)          # [cout][tap][cin]: the packed K order
    q = torch.empty_like(f)
    e = torch.zeros(co, dtype=f.dtype)
    for k in range(f.shape[1]):
        t = (f[:, k] - e).to(dt).float()
        e = e + t - f[:, k]
        q[:, k] = t
    return q.reshape(co, w.shape[2], w.shape[3], w.shape[1]).permute(0, 3, 1, 2).contiguous()


def emulate(burst, sd, kw, fp32=(), dt=torch.float16, diffuse=()):
    """diffuse: stages whose weights take diffuse_round instead of round-to-nearest."""
    """The engine's forward with 16-bit storage except the stages in fp32 (a CPU emulation); returns pred, offsets."""
    # 'stage' keeps its weights and its stored tensors fp32; 'stage:w' only its weights, 'stage:s' only its storage;
    # 'dec.post:mid' / 'dec.post:out' only the post-ResBlocks' intermediates (conv1 outputs) / block outputs
    def R(t, st, kinds=('s',)):
        keep = st in fp32 or any(st + ':' + k in fp32 for k in kinds)
        return t if (keep or dt is None) else t.to(dt).float()
    o = {n: getattr(orc, n) for n in ('conv', 'conv_block', 'res_block', 'warp', 'merging', 'decoder',
                                      'correlation')}
    n_post = kw['dec_num_post_res_blocks']

    def conv(x, sd_, name, stride=1, padding=1, dilation=1):
        st = stage_of(name)
        w = sd_[name + '.weight']
        if name != 'decoder.predictor.0':                  # the fused RGB head runs fp32 weights
            if st in diffuse and st not in fp32 and (w.shape[-1] > 1 or '1x1' in diffuse):
                w = diffuse_round(w, dt)
            else:
                w = R(w, st, ('w',))
        y = F.conv2d(x, w, sd_.get(name + '.bias'), stride=stride, padding=padding, dilation=dilation)
        # PWC-Net's convs store their (LeakyReLU'd) outputs 16-bit, except the flow heads (fp32 flows)
        if st == 'pwc' and not name.endswith(('netSix.0', 'netMain.12')):
            y = R(y, st)
        return y

    def conv_block(x, sd_, name, ksz=3, act='relu'):
        y = o['conv_block'](x, sd_, name, ksz=ksz, act=act)
        if name == 'decoder.predictor':
            return y
        if name.startswith('merging.weight_predictor') and act == 'none':
            return y                                       # the logits: fp32 (conv_fuse)
        return R(y, stage_of(name))

    def res_block(x, sd_, name):
        st = stage_of(name)
        mid = R(F.relu(conv(x, sd_, name + '.conv1.0')), st, ('s', 'mid'))
        out = conv(mid, sd_, name + '.conv2.0')
        y = F.relu(out + x)
        if name == 'decoder.post_res_layers.%d' % (n_post - 1):
            return y                                       # dbsr_resblock_head: the block output stays fp32
        return R(y, st, ('s', 'out'))

    def correlation(first, second):
        return R(o['correlation'](first, second), 'pwc')

    def warp(feat, flow, **k):
        return R(o['warp'](feat, flow, **k), 'warp')

    def merging(x, sd_, kw_, return_logits=False):
        all_feat, w = o['merging'](x, sd_, kw_, return_logits=True)
        wn = F.softmax(w, dim=1)
        return {'fused_enc': R((all_feat * wn).sum(dim=1), 'fuse'), 'fusion_weights': wn}

    def decoder(x, sd_, kw_):
        feat = x['fused_enc']
        out = conv_block(feat, sd_, 'decoder.init_layer')
        for i in range(kw_['dec_num_pre_res_blocks']):
            out = res_block(out, sd_, f'decoder.pre_res_layers.{i}')
        out = conv_block(out, sd_, 'decoder.upsample_layer.conv_layer', ksz=1)     # stored (rounded) pre-blur
        out = F.pixel_shuffle(out, kw_['upsample_factor'])
        K = orc.gauss_kernel(kw_.get('gauss_ksz', 3), kw_['gauss_blur_sd'], out.dtype)
        shp = out.shape
        out = R(F.conv2d(out.reshape(-1, 1, *shp[-2:]), K, padding=1).view(shp), 'dec.up')
        for i in range(kw_['dec_num_post_res_blocks']):
            out = res_block(out, sd_, f'decoder.post_res_layers.{i}')
        return conv_block(out, sd_, 'decoder.predictor', ksz=1)

    orc.conv, orc.conv_block, orc.res_block, orc.correlation = conv, conv_block, res_block, correlation
    orc.warp, orc.merging, orc.decoder = warp, merging, decoder
    try:
        with torch.no_grad():
            p, aux = orc.dbsr_forward(burst, sd, kw)
            return p, aux['offsets']
    finally:
        for n, f in o.items():
            setattr(orc, n, f)


def main():
    torch.set_num_threads(os.cpu_count())
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    extra = [tuple(s.split(',')) for s in sys.argv[2:]]
    kw = dbsr_amd.DBSR_SYNTHETIC_KWARGS
    net = dbsr_amd.dbsrnet_cvpr2021(**kw)
    sd = orc.state_dict_to_torch(generate_state_dict(arch.state_dict_shapes(net), seed=0))
    burst, _ = synthetic_bursts(8, 14, 48, 48, sr_factor=8, seed=101)
    burst = burst[:B]
    with torch.no_grad():
        ref, raux = orc.dbsr_forward(burst, sd, kw)
    roffs = raux['offsets']

    def rms(p):
        return float((p.clamp(0, 1) - ref.clamp(0, 1)).pow(2).mean().sqrt())
    p_all, o_all = emulate(burst, sd, kw)
    r_all = rms(p_all)
    print('B=%d: fp16 everywhere: clamped RMS %.3e (unclamped %.3e), offsets max %.3e' % (
        B, r_all, float((p_all - ref).pow(2).mean().sqrt()), float((o_all - roffs).abs().max())), flush=True)
    print('| stage kept fp32 | clamped RMS | share of the fp16 error (quadrature) | offsets max err |')
    print('|---|---|---|---|')
    stages = [] if os.environ.get('ONLY_EXTRA') else [(s,) for s in STAGES]
    for st in stages + extra:
        if st and st[0].startswith('diffuse:'):
            p, o = emulate(burst, sd, kw, diffuse=st[0][8:].split('+'))
        else:
            p, o = emulate(burst, sd, kw, fp32=st)
        r = rms(p)
        print('| %s | %.3e | %.1f %% | %.2e |' % ('+'.join(st), r, 100 * (r_all ** 2 - r ** 2) / r_all ** 2,
                                               float((o - roffs).abs().max())), flush=True)


if __name__ == '__main__':
    main()
