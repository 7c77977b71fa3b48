"""ORACLE — test infrastructure only.  Not part of the product path.

CPU restatement (torch-CPU, fp32 or fp64) of the reference DBSR forward path, used as the parity
checker for the HIP implementation.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module.

Pinning: the restatement is checked in this container against the reference itself, imported from
/root/reference with in-process stubs (tests/golden/make_golden.py writes the fixtures under
tests/golden/ that tests/test_oracle.py compares against).  The reference's correlation layer has
no CPU implementation (external/pwcnet/correlation/correlation.py:324-325), so the one piece that is
pinned only by the CUDA source text is `correlation` below (K2, correlation.py:35-103), which is
additionally cross-checked against a literal loop transliteration of that kernel
(`correlation_loops`).

Every function cites the reference file:line it restates.  The arithmetic (conv2d, grid_sample,
interpolate, softmax, pixel_shuffle) is PyTorch's, exactly as the reference calls it.
"""
import math

import torch
import torch.nn.functional as F

DBSR_SYNTHETIC_KWARGS = dict(   # train_settings/dbsr/default_synthetic.py:73-82 (downsample_factor=4)
    enc_init_dim=64, enc_num_res_blocks=9, enc_out_dim=512,
    dec_init_conv_dim=64, dec_num_pre_res_blocks=5,
    dec_post_conv_dim=32, dec_num_post_res_blocks=4,
    upsample_factor=8, offset_feat_dim=64, weight_pred_proj_dim=64,
    num_weight_predictor_res=3, gauss_blur_sd=1.0, icnrinit=True)


# ----------------------------------------------------------------------------------------------
# models/layers
# ----------------------------------------------------------------------------------------------
def conv(x, sd, name, stride=1, padding=1, dilation=1):
    """nn.Conv2d inside conv_block (models/layers/blocks.py:46-60)."""
    return F.conv2d(x, sd[name + '.weight'], sd.get(name + '.bias'), stride=stride,
                    padding=padding, dilation=dilation)


def conv_block(x, sd, name, ksz=3, act='relu'):
    """conv_block (blocks.py:46-60): conv + optional ReLU ('none' -> no activation)."""
    pad = (ksz - 1) // 2
    y = conv(x, sd, name + '.0', padding=pad)
    return F.relu(y) if act == 'relu' else y


def res_block(x, sd, name):
    """ResBlock.forward (blocks.py:81-96): relu(conv2(relu(conv1(x))) + x)."""
    out = conv_block(x, sd, name + '.conv1', act='relu')
    out = conv_block(out, sd, name + '.conv2', act='none')
    return F.relu(out + x)


def warp(feat, flow, mode='bilinear', padding_mode='zeros'):
    """models/layers/warp.py:19-46 (verbatim arithmetic order)."""
    B, C, H, W = feat.size()
    rowv, colv = torch.meshgrid([torch.arange(0.5, H + 0.5, dtype=feat.dtype),
                                 torch.arange(0.5, W + 0.5, dtype=feat.dtype)], indexing='ij')
    grid = torch.stack((colv, rowv), dim=0).unsqueeze(0).to(feat.dtype)
    grid = grid + flow
    grid_norm_c = 2.0 * grid[:, 0] / W - 1.0
    grid_norm_r = 2.0 * grid[:, 1] / H - 1.0
    grid_norm = torch.stack((grid_norm_c, grid_norm_r), dim=1).permute(0, 2, 3, 1)
    return F.grid_sample(feat, grid_norm, mode=mode, padding_mode=padding_mode, align_corners=False)


def gauss_kernel(ksz, sd, dtype=torch.float32):
    """PixShuffleUpsampler._get_gaussian_kernel (upsampling.py:24-29) via gauss_2d/gauss_1d
    (filtering.py:20-40), density=True then normalised to sum 1."""
    k = torch.arange(-(ksz - 1) / 2, (ksz + 1) / 2).reshape(1, -1)
    g1 = torch.exp(-1.0 / (2 * sd ** 2) * (k - 0.0) ** 2) / (math.sqrt(2 * math.pi) * sd)
    K = g1.reshape(1, 1, -1) * g1.reshape(1, -1, 1)
    K = K / K.sum()
    return K.unsqueeze(0).to(dtype)       # [1,1,ksz,ksz]


# ----------------------------------------------------------------------------------------------
# external/pwcnet/correlation (K2)
# ----------------------------------------------------------------------------------------------
def correlation(first, second):
    """Cost volume of kernel_Correlation_updateOutput (correlation.py:35-103) with the zero padding
    of kernel_Correlation_rearrange (:8-33, rbot buffers padded by 4, :281-282):
    out[n, (dy+4)*9 + (dx+4), y, x] = sum_c first[n,c,y,x] * second[n,c,y+dy,x+dx] / C."""
    N, C, H, W = first.shape
    sp = F.pad(second, (4, 4, 4, 4))
    outs = []
    for top in range(81):
        dx = top % 9 - 4          # s2o, correlation.py:72
        dy = top // 9 - 4         # s2p, correlation.py:73
        sh = sp[:, :, 4 + dy:4 + dy + H, 4 + dx:4 + dx + W]
        outs.append((first * sh).sum(1) / float(C))
    return torch.stack(outs, 1)


def correlation_loops(first, second):
    """Literal transliteration of K2's indexing (correlation.py:47-100) with python loops, for small
    cross-checks of `correlation`.  Sums channels in K2's order: 32 strided partial sums, then a
    serial sum of the partials (:78-96)."""
    N, C, H, W = first.shape
    rb0 = torch.zeros(N, H + 8, W + 8, C, dtype=first.dtype)
    rb1 = torch.zeros(N, H + 8, W + 8, C, dtype=first.dtype)
    rb0[:, 4:4 + H, 4:4 + W, :] = first.permute(0, 2, 3, 1)
    rb1[:, 4:4 + H, 4:4 + W, :] = second.permute(0, 2, 3, 1)
    out = torch.zeros(N, 81, H, W, dtype=first.dtype)
    for item in range(N):
        for by in range(H):
            for bx in range(W):
                x1, y1 = bx + 4, by + 4
                for top in range(81):
                    s2o, s2p = top % 9 - 4, top // 9 - 4
                    x2, y2 = x1 + s2o, y1 + s2p
                    partial = [0.0] * 32
                    for lane in range(32):
                        for ch in range(lane, C, 32):
                            partial[lane] += float(rb0[item, y1, x1, ch]) * float(rb1[item, y2, x2, ch])
                    out[item, top, by, bx] = sum(partial) / float(C)
    return out


# ----------------------------------------------------------------------------------------------
# models/alignment/pwcnet.py
# ----------------------------------------------------------------------------------------------
def backwarp(tenInput, tenFlow):
    """pwcnet.py:16-38 (the module-level grid caches are a pure memo, not restated)."""
    dt = tenFlow.dtype
    tenHor = torch.linspace(-1.0 + (1.0 / tenFlow.shape[3]), 1.0 - (1.0 / tenFlow.shape[3]),
                            tenFlow.shape[3], dtype=dt).view(1, 1, 1, -1).expand(-1, -1, tenFlow.shape[2], -1)
    tenVer = torch.linspace(-1.0 + (1.0 / tenFlow.shape[2]), 1.0 - (1.0 / tenFlow.shape[2]),
                            tenFlow.shape[2], dtype=dt).view(1, 1, -1, 1).expand(-1, -1, -1, tenFlow.shape[3])
    grid = torch.cat([tenHor, tenVer], 1)
    partial = tenFlow.new_ones([tenFlow.shape[0], 1, tenFlow.shape[2], tenFlow.shape[3]])
    tenFlow = torch.cat([tenFlow[:, 0:1] / ((tenInput.shape[3] - 1.0) / 2.0),
                         tenFlow[:, 1:2] / ((tenInput.shape[2] - 1.0) / 2.0)], 1)
    tenInput = torch.cat([tenInput, partial], 1)
    out = F.grid_sample(tenInput, (grid + tenFlow).permute(0, 2, 3, 1), mode='bilinear',
                        padding_mode='zeros', align_corners=False)
    mask = out[:, -1:]
    mask[mask > 0.999] = 1.0
    mask[mask < 1.0] = 0.0
    return out[:, :-1].contiguous() * mask.contiguous()


def _lrelu(x):
    return F.leaky_relu(x, negative_slope=0.1)


def pwc_extractor(x, sd, p):
    """Extractor.forward (pwcnet.py:103-111): 6 levels of (3x3 s2, 3x3, 3x3) + LeakyReLU(0.1)."""
    feats = []
    for lvl in ['netOne', 'netTwo', 'netThr', 'netFou', 'netFiv', 'netSix']:
        x = _lrelu(conv(x, sd, f'{p}.netExtractor.{lvl}.0', stride=2))
        x = _lrelu(conv(x, sd, f'{p}.netExtractor.{lvl}.2'))
        x = _lrelu(conv(x, sd, f'{p}.netExtractor.{lvl}.4'))
        feats.append(x)
    return feats


_BACKWARP = {5: 0.625, 4: 1.25, 3: 2.5, 2: 5.0}   # fltBackwarp, pwcnet.py:121


def pwc_decoder(level, first, second, prev, sd, p):
    """Decoder.forward (pwcnet.py:153-184)."""
    name = {2: 'netTwo', 3: 'netThr', 4: 'netFou', 5: 'netFiv', 6: 'netSix'}[level]
    d = f'{p}.{name}'
    if prev is None:
        vol = _lrelu(correlation(first, second))
        feat = vol
    else:
        flow = F.conv_transpose2d(prev['tenFlow'], sd[d + '.netUpflow.weight'], sd[d + '.netUpflow.bias'],
                                  stride=2, padding=1)
        upfeat = F.conv_transpose2d(prev['tenFeat'], sd[d + '.netUpfeat.weight'], sd[d + '.netUpfeat.bias'],
                                    stride=2, padding=1)
        vol = _lrelu(correlation(first, backwarp(second, flow * _BACKWARP[level])))
        feat = torch.cat([vol, first, flow, upfeat], 1)
    for sub in ['netOne', 'netTwo', 'netThr', 'netFou', 'netFiv']:
        feat = torch.cat([_lrelu(conv(feat, sd, f'{d}.{sub}.0')), feat], 1)
    flow = conv(feat, sd, f'{d}.netSix.0')
    return {'tenFlow': flow, 'tenFeat': feat}


def pwc_refiner(x, sd, p):
    """Refiner (pwcnet.py:186-207): dilations 1,2,4,8,16,1,1; LeakyReLU after all but the last."""
    dil = [1, 2, 4, 8, 16, 1, 1]
    for i, d in enumerate(dil):
        x = conv(x, sd, f'{p}.netRefiner.netMain.{2 * i}', padding=d, dilation=d)
        if i < 6:
            x = _lrelu(x)
    return x


def pwc_network(tenFirst, tenSecond, sd, p):
    """Network.forward (pwcnet.py:221-231)."""
    f1 = pwc_extractor(tenFirst, sd, p)
    f2 = pwc_extractor(tenSecond, sd, p)
    est = pwc_decoder(6, f1[-1], f2[-1], None, sd, p)
    est = pwc_decoder(5, f1[-2], f2[-2], est, sd, p)
    est = pwc_decoder(4, f1[-3], f2[-3], est, sd, p)
    est = pwc_decoder(3, f1[-4], f2[-4], est, sd, p)
    est = pwc_decoder(2, f1[-5], f2[-5], est, sd, p)
    return est['tenFlow'] + pwc_refiner(est['tenFeat'], sd, p)


def pwcnet(source_img, target_img, sd, p='encoder.alignment_net.net'):
    """PWCNet.forward (pwcnet.py:248-281), rgb2bgr=False."""
    W, H = source_img.shape[-1], source_img.shape[-2]
    source_img = source_img.view(-1, 3, H, W)
    target_img = target_img.view(-1, 3, H, W)
    Wp = int(math.floor(math.ceil(W / 64.0) * 64.0))
    Hp = int(math.floor(math.ceil(H / 64.0) * 64.0))
    s_re = F.interpolate(source_img, size=(Hp, Wp), mode='bilinear', align_corners=False)
    t_re = F.interpolate(target_img, size=(Hp, Wp), mode='bilinear', align_corners=False)
    flow = pwc_network(t_re, s_re, sd, p)
    flow = 20.0 * F.interpolate(flow, size=(H, W), mode='bilinear', align_corners=False)
    sx, sy = float(W) / float(Wp), float(H) / float(Hp)
    return torch.stack((flow[:, 0] * sx, flow[:, 1] * sy), dim=1)


# ----------------------------------------------------------------------------------------------
# models/dbsr
# ----------------------------------------------------------------------------------------------
def encoder(x, sd, kw, zero_flow=False):
    """ResEncoderWarpAlignnet.forward (encoders.py:48-86)."""
    B, N = x.shape[:2]
    x_rgb = torch.stack((x[:, :, 0], x[:, :, 1:3].mean(dim=2), x[:, :, 3]), dim=2)
    x_ref = x_rgb[:, :1].repeat(1, N - 1, 1, 1, 1).contiguous()
    x_oth = x_rgb[:, 1:].contiguous()
    if zero_flow:   # config 1's identity-flow alignment stub (BASELINE.json configs[0])
        offsets = x.new_zeros(B * (N - 1), 2, x.shape[-2], x.shape[-1])
    else:
        offsets = pwcnet(x_oth.view(-1, *x_oth.shape[-3:]), x_ref.view(-1, *x_ref.shape[-3:]), sd)
    shape = x.shape
    x = x.reshape(-1, *x.shape[-3:])
    out = conv_block(x, sd, 'encoder.init_layer')
    for i in range(kw['enc_num_res_blocks']):
        out = res_block(out, sd, f'encoder.res_layers.{i}')
    feat = conv_block(out, sd, 'encoder.out_layer')
    feat = feat.view(shape[0], shape[1], *feat.shape[-3:])
    ref_feat = feat[:, :1].contiguous()
    oth_feat = feat[:, 1:].contiguous().view(-1, *feat.shape[-3:])
    oth_feat = warp(oth_feat, offsets)
    oth_feat = oth_feat.view(shape[0], shape[1] - 1, *oth_feat.shape[-3:])
    offsets = offsets.view(shape[0], shape[1] - 1, 2, shape[-2], shape[-1])
    return {'ref_feat': ref_feat.expand(-1, shape[1] - 1, -1, -1, -1), 'oth_feat': oth_feat,
            'offsets': offsets}


def merging(x, sd, kw, return_logits=False):
    """WeightedSum.forward (merging.py:61-127) with use_offset=True and ref_offset_noise=0; offset_modulo (default 1.0,
    None: no remainder, merging.py:101-102), softmax (default True; False: ReLU-normalised weights, :117-121) and
    use_base_frame (default True; False: the mean projected embedding as the base, :79-82) from kw."""
    ref_feat = x['ref_feat'][:, :1].contiguous()
    oth_feat, offsets = x['oth_feat'], x['offsets']
    shape = ref_feat.shape
    all_feat = torch.cat((ref_feat, oth_feat), dim=1)
    proj = conv_block(all_feat.view(-1, *all_feat.shape[-3:]), sd, 'merging.feat_project_layer', ksz=1)
    proj = proj.view(*all_feat.shape[:2], -1, *all_feat.shape[-2:])
    base = proj[:, :1].contiguous() if kw.get('use_base_frame', True) else proj.mean(dim=1, keepdim=True)
    diff = (proj - base).view(-1, *proj.shape[-3:])
    base = base.expand(-1, all_feat.shape[1], -1, -1, -1).contiguous().view(-1, *base.shape[-3:])
    offsets_base = offsets.new_zeros((shape[0], 1, 2, *shape[-2:]))
    offsets_all = torch.cat((offsets_base, offsets), dim=1).view(-1, 2, *shape[-2:])
    if kw.get('offset_modulo', 1.0) is not None:
        offsets_all = offsets_all % kw.get('offset_modulo', 1.0)
    of = conv_block(offsets_all, sd, 'merging.offset_feat_extractor.0')
    for i in range(1, 1 + kw.get('num_offset_feat_extractor_res', 1)):
        of = res_block(of, sd, f'merging.offset_feat_extractor.{i}')
    w = torch.cat([base, diff, of], dim=1)
    nres = kw['num_weight_predictor_res']
    w = conv_block(w, sd, 'merging.weight_predictor.0')
    for i in range(1, 1 + nres):
        w = res_block(w, sd, f'merging.weight_predictor.{i}')
    w = conv_block(w, sd, f'merging.weight_predictor.{nres + 1}', act='none')
    w = w.view(shape[0], -1, *w.shape[-3:])
    if return_logits:
        return all_feat, w
    if kw.get('softmax', True):
        wn = F.softmax(w, dim=1)
    else:
        wn = F.relu(w)
        wn = wn / (wn.sum(dim=1, keepdim=True) + 1e-12)
    fused = (all_feat * wn).sum(dim=1)
    return {'fused_enc': fused, 'fusion_weights': wn}


def fuse_partial_stats(all_feat, logits, first):
    """Frame-sharded fusion, rank-local half (splits merging.py:116-124): over frames
    n >= first of this shard, m = max l, s = sum e^(l-m), a = sum e^(l-m) f.  Layout [B,H,W,3C]
    (m | s | a), the one dbsr_fuse_partial writes."""
    lg, f = logits[:, first:], all_feat[:, first:]
    B, _, C, H, W = all_feat.shape
    if lg.shape[1] == 0:
        m = torch.full((B, C, H, W), float('-inf'), dtype=logits.dtype)
        s = torch.zeros(B, C, H, W, dtype=logits.dtype)
        a = torch.zeros(B, C, H, W, dtype=logits.dtype)
    else:
        m = lg.max(dim=1).values
        e = torch.exp(lg - m.unsqueeze(1))
        s, a = e.sum(dim=1), (e * f).sum(dim=1)
    return torch.cat([m, s, a], dim=1).permute(0, 2, 3, 1).contiguous()


def fuse_combine(gathered):
    """Log-sum-exp combine of gathered [R,B,H,W,3C] statistics -> fused [B,C,H,W] (dbsr_fuse_combine)."""
    C = gathered.shape[-1] // 3
    m, s, a = gathered[..., :C], gathered[..., C:2 * C], gathered[..., 2 * C:]
    M = m.max(dim=0).values
    k = torch.where(torch.isinf(m), torch.zeros_like(m), torch.exp(m - M.unsqueeze(0)))
    return ((a * k).sum(0) / (s * k).sum(0)).permute(0, 3, 1, 2).contiguous()


def decoder(x, sd, kw):
    """ResPixShuffleConv.forward (decoders.py:54-62) with PixShuffleUpsampler (upsampling.py:51-66)."""
    feat = x['fused_enc']
    out = conv_block(feat, sd, 'decoder.init_layer')
    for i in range(kw['dec_num_pre_res_blocks']):
        out = res_block(out, sd, f'decoder.pre_res_layers.{i}')
    out = conv_block(out, sd, 'decoder.upsample_layer.conv_layer', ksz=1)
    out = F.pixel_shuffle(out, kw['upsample_factor'])
    if kw.get('gauss_blur_sd') is not None:
        ksz = kw.get('gauss_ksz', 3)
        K = gauss_kernel(ksz, kw['gauss_blur_sd'], out.dtype)
        shp = out.shape
        out = F.conv2d(out.reshape(-1, 1, *shp[-2:]), K, padding=(ksz - 1) // 2).view(shp)
    for i in range(kw['dec_num_post_res_blocks']):
        out = res_block(out, sd, f'decoder.post_res_layers.{i}')
    return conv_block(out, sd, 'decoder.predictor', ksz=1)     # conv_block default act='relu'


def dbsr_forward(burst, sd, kw=DBSR_SYNTHETIC_KWARGS, zero_flow=False, return_intermediates=False):
    """DBSRNet.forward (dbsrnet.py:33-38)."""
    enc = encoder(burst, sd, kw, zero_flow=zero_flow)
    mer = merging(enc, sd, kw)
    pred = decoder(mer, sd, kw)
    aux = {'offsets': enc['offsets'], 'fusion_weights': mer['fusion_weights']}
    if return_intermediates:
        aux['fused_enc'] = mer['fused_enc']
    return pred, aux


def state_dict_to_torch(sd_np, dtype=torch.float32):
    return {k: torch.from_numpy(v).to(dtype) for k, v in sd_np.items()}


# ----------------------------------------------------------------------------------------------
# BurstSR scoring: SpatialColorAlignment (models/loss/spatial_color_alignment.py:23-108)
# ----------------------------------------------------------------------------------------------
def gaussian_kernel_2d(sd, ksz=None):
    """get_gaussian_kernel (filtering.py:20-51): normalised density on an odd ksz grid."""
    if ksz is None:
        ksz = int(4 * sd + 1)
    k = torch.arange(-(ksz - 1) / 2, (ksz + 1) / 2).reshape(1, -1)
    g = torch.exp(-1.0 / (2 * sd ** 2) * (k - torch.zeros(1, 1)) ** 2) / (math.sqrt(2 * math.pi) * sd)
    K = g.reshape(1, 1, -1) * g.reshape(1, -1, 1)
    return (K / K.sum()), ksz


def apply_kernel(im, ksz, kernel):
    """filtering.py:54-63."""
    shape = im.shape
    im = im.reshape(-1, 1, *im.shape[-2:])
    im = F.pad(im, [ksz // 2] * 4, mode='reflect')
    return F.conv2d(im, kernel.unsqueeze(0).to(im.dtype)).view(shape)


def match_colors(im_ref, im_q, im_test, ksz, gauss_kernel, bi=5, thresh=20):
    """spatial_color_alignment.py:23-67; torch.lstsq(B, A) (removed in torch 2.x) is its least-squares
    solution of A X = B, torch.linalg.lstsq here.  Returns (im_test^T C, valid, C)."""
    ref_m = apply_kernel(im_ref, ksz, gauss_kernel)[:, :, bi:-bi, bi:-bi].contiguous()
    q_m = apply_kernel(im_q, ksz, gauss_kernel)[:, :, bi:-bi, bi:-bi].contiguous()
    ref_re = ref_m.view(*ref_m.shape[:2], -1)
    q_re = q_m.view(*q_m.shape[:2], -1)
    c_mat = torch.stack([torch.linalg.lstsq(iq.t(), ir.t()).solution[:3] for ir, iq in zip(ref_re, q_re)], 0)
    q_conv = torch.matmul(q_re.permute(0, 2, 1), c_mat).permute(0, 2, 1).view(q_m.shape)
    err = ((q_conv - ref_m) * 255.0).norm(dim=1)
    valid = err < thresh
    pad = (im_q.shape[-1] - valid.shape[-1]) // 2
    valid = F.pad(valid, [pad] * 4)
    f = im_test.shape[-1] / valid.shape[-1]
    valid = F.interpolate(valid.unsqueeze(1).float(), scale_factor=f, mode='bilinear') > 0.9
    t_re = im_test.view(*im_test.shape[:2], -1)
    out = torch.matmul(t_re.permute(0, 2, 1), c_mat).permute(0, 2, 1).view(im_test.shape)
    return out, valid, c_mat


def spatial_color_alignment(pred, gt, burst_input, sd, sr_factor=4, p='encoder.alignment_net.net'):
    """SpatialColorAlignment.forward (spatial_color_alignment.py:87-108) with the oracle PWC-Net.
    Returns (pred_warped_m, valid, flow, c_mat)."""
    flow = pwcnet(pred / (pred.max() + 1e-6), gt / (gt.max() + 1e-6), sd, p)
    pred_warped = warp(pred, flow)
    ds = 1.0 / float(2.0 * sr_factor)
    flow_ds = F.interpolate(flow, scale_factor=ds, mode='bilinear') * ds
    burst_0 = burst_input[:, 0, [0, 1, 3]].contiguous()
    burst_0_warped = warp(burst_0, flow_ds)
    gt_ds = F.interpolate(gt, scale_factor=ds, mode='bilinear')
    K, ksz = gaussian_kernel_2d(1.5)
    out, valid, c_mat = match_colors(gt_ds, burst_0_warped, pred_warped, ksz, K)
    return out, valid, flow, c_mat
