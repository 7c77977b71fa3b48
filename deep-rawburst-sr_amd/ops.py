"""Op-level mirror of the reference's functional sub-seams, NCHW in / NCHW out like the reference:

  FunctionCorrelation(tenFirst, tenSecond)      external/pwcnet/correlation/correlation.py:385-387
  backwarp(tenInput, tenFlow)                   models/alignment/pwcnet.py:16-38
  warp(feat, flow, mode, padding_mode)          models/layers/warp.py:19-46
  conv2d(...)                                   nn.Conv2d (+ fused activation / residual) via dbsr_conv2d

Each runs the HIP kernel of libdbsr_hip.so; the NCHW<->NHWC permutes around the call are torch
device copies (layout plumbing for callers that hold NCHW tensors; the engine never uses them).
Errors mirror the reference: non-contiguous input to the correlation raises (correlation.py:286-287),
a CPU tensor raises (correlation.py:324-325 raises NotImplementedError on CPU).
"""
import collections

import torch

from . import _lib as L


def _nhwc(x, dtype=None):
    t = x.permute(0, 2, 3, 1)
    if dtype is not None:
        t = t.to(dtype)
    c = t.shape[-1]
    ld = (c + 7) // 8 * 8 if c <= 16 else (c + 31) // 32 * 32     # dbsr_conv2d channel padding
    out = torch.zeros(*t.shape[:-1], ld, dtype=t.dtype, device=t.device)
    out[..., :c] = t
    return out, ld


def _need_cuda(*ts):
    for t in ts:
        if not t.is_cuda:
            raise NotImplementedError('dbsr_amd ops run on the HIP device only (no CPU implementation, as '
                                      'correlation.py:324-325)')


def FunctionCorrelation(tenFirst, tenSecond, leaky=False):
    """81-channel cost volume / C (K2).  leaky=True fuses the callers' leaky_relu(0.1)."""
    _need_cuda(tenFirst, tenSecond)
    if not (tenFirst.is_contiguous() and tenSecond.is_contiguous()):
        raise AssertionError('correlation inputs must be contiguous (correlation.py:286-287)')
    N, C, H, W = tenFirst.shape
    dt = tenFirst.dtype
    a, lda = _nhwc(tenFirst)
    b, ldb = _nhwc(tenSecond)
    out = torch.zeros(N, H, W, 88, dtype=dt, device=tenFirst.device)
    L.check(L.lib().dbsr_correlation(N, H, W, C, L.tensor_desc(a, lda), L.tensor_desc(b, ldb),
                                     L.tensor_desc(out, 88), 1 if leaky else 0, L.stream_ptr(tenFirst.device)),
            'dbsr_correlation')
    return out[..., :81].permute(0, 3, 1, 2).contiguous()


class ModuleCorrelation(torch.nn.Module):
    def forward(self, tenFirst, tenSecond):
        return FunctionCorrelation(tenFirst, tenSecond)


def backwarp(tenInput, tenFlow):
    _need_cuda(tenInput, tenFlow)
    N, C, H, W = tenInput.shape
    x, ldx = _nhwc(tenInput)
    fl = tenFlow.permute(0, 2, 3, 1).to(torch.float32).contiguous()
    out = torch.zeros_like(x)
    L.check(L.lib().dbsr_backwarp(N, H, W, C, L.tensor_desc(x, ldx), L.tensor_desc(fl, 2), 1.0,
                                  L.tensor_desc(out, ldx), L.stream_ptr(tenInput.device)), 'dbsr_backwarp')
    return out[..., :C].permute(0, 3, 1, 2).contiguous()


def warp(feat, flow, mode='bilinear', padding_mode='zeros'):
    if mode != 'bilinear' or padding_mode != 'zeros':
        raise NotImplementedError('only bilinear / zeros is on the hot path (encoders.py:80)')
    _need_cuda(feat, flow)
    N, C, H, W = feat.shape
    x, ld = _nhwc(feat)
    fl = flow.to(torch.float32).contiguous()
    out = torch.zeros_like(x)
    L.check(L.lib().dbsr_warp_bilinear(N, H, W, ld, L.tensor_desc(x, ld), fl.data_ptr(), 2 * H * W,
                                       L.tensor_desc(out, ld), L.stream_ptr(feat.device)), 'dbsr_warp_bilinear')
    return out[..., :C].permute(0, 3, 1, 2).contiguous()


_PACKED = collections.OrderedDict()    # (weight, bias, version, dtype, shuffle) -> packed MFMA weights
_PACKED_MAX = 64


def _packed(weight, bias, compute_dtype, shuffle, stream):
    """Packed weights (dbsr_conv_pack_weights) of a parameter, cached while the tensor is unchanged (same
    storage and autograd version counter), so a repeated op-level call does not repack."""
    key = (weight.data_ptr(), weight._version, tuple(weight.shape),
           bias.data_ptr() if bias is not None else 0, bias._version if bias is not None else 0,
           compute_dtype, shuffle, weight.device)
    hit = _PACKED.get(key)
    if hit is not None:
        _PACKED.move_to_end(key)
        return hit[0], hit[1]
    Cout, Cin, kh, kw = weight.shape
    dev = weight.device
    n = L.lib().dbsr_conv_packed_elems(Cout, Cin, kh, kw)
    wp = torch.empty(n, dtype=compute_dtype, device=dev)
    bp = torch.empty(Cout, dtype=torch.float32, device=dev) if bias is not None else None
    w32 = weight.detach().to(torch.float32).contiguous()
    b32 = bias.detach().to(torch.float32).contiguous() if bias is not None else None
    L.check(L.lib().dbsr_conv_pack_weights(w32.data_ptr(), b32.data_ptr() if b32 is not None else None, Cout, Cin,
                                           kh, kw, L.dtype_code(compute_dtype), shuffle, wp.data_ptr(),
                                           bp.data_ptr() if bp is not None else None, stream), 'pack')
    # the cache keeps the source tensors alive so their storage (the key) cannot be reused meanwhile
    _PACKED[key] = (wp, bp, weight, bias, w32, b32)
    while len(_PACKED) > _PACKED_MAX:
        _PACKED.popitem(last=False)
    return wp, bp


def conv2d(x, weight, bias=None, stride=1, padding=0, dilation=1, act=L.ACT_NONE, residual=None,
           post_act=L.ACT_NONE, compute_dtype=torch.float32, out_f32=False, head=None, shuffle=1):
    """act(conv2d(x) + bias) (+ residual, then post_act); NCHW in/out, computed by dbsr_conv2d.
    head = (w [hc, Cout, 1, 1], b [hc] | None): return ReLU(conv1x1(result, w, b)) as fp32 NCHW instead,
    computed by dbsr_conv2d_head (the conv's own result is not stored).
    shuffle = s > 1: return PixelShuffle(s) of the result (upsampling.py:51-66's conv + shuffle)."""
    _need_cuda(x, weight)
    N, Cin, H, W = x.shape
    Cout, _, kh, kw = weight.shape
    dev = x.device
    xs, ldx = _nhwc(x, compute_dtype)
    s = L.stream_ptr(dev)
    wp, bp = _packed(weight, bias, compute_dtype, shuffle, s)
    oh = (H + 2 * padding - dilation * (kh - 1) - 1) // stride + 1
    ow = (W + 2 * padding - dilation * (kw - 1) - 1) // stride + 1
    ody = torch.float32 if out_f32 else compute_dtype
    pc = Cout // (shuffle * shuffle)
    ldy = (pc + 7) // 8 * 8
    y = torch.zeros(N, oh * shuffle, ow * shuffle, ldy, dtype=ody, device=dev)
    d = L.ConvDesc()
    d.n_frames = N
    d.x = L.tensor_desc(xs, ldx)
    d.in_h, d.in_w, d.cin = H, W, Cin
    d.w = wp.data_ptr()
    d.bias = bp.data_ptr() if bp is not None else None
    d.cout, d.kh, d.kw, d.stride, d.pad, d.dil = Cout, kh, kw, stride, padding, dilation
    d.y = L.tensor_desc(y, ldy)
    d.out_h, d.out_w = oh, ow
    d.act = act
    if residual is not None:
        rr, ldr = _nhwc(residual, ody)
        d.res = L.tensor_desc(rr, ldr)
    else:
        d.res = L.NULL_TENSOR
    d.post_act = post_act
    d.out_mode, d.shuffle = (L.OUT_SHUFFLE, shuffle) if shuffle > 1 else (L.OUT_NHWC, 0)
    need = L.lib().dbsr_conv_workspace_bytes(d)
    ws = torch.zeros(max(need // 4, 1), dtype=torch.float32, device=dev)
    d.workspace, d.workspace_bytes = ws.data_ptr(), need
    if head is not None:
        hw, hb = head
        hc = hw.shape[0]
        hw32 = hw.reshape(hc, -1).to(device=dev, dtype=torch.float32).contiguous()
        hb32 = hb.to(device=dev, dtype=torch.float32).contiguous() if hb is not None else None
        out = torch.zeros(N, hc, oh, ow, dtype=torch.float32, device=dev)
        L.check(L.lib().dbsr_conv2d_head(d, hw32.data_ptr(), hb32.data_ptr() if hb32 is not None else None, hc,
                                         L.tensor_desc(out, 1, 0, img_stride=hc * oh * ow, dtype=torch.float32),
                                         s), 'dbsr_conv2d_head')
        return out
    conv2d.last_kernel = L.lib().dbsr_conv_kernel_for(d)     # which kernel family ran (tests)
    conv2d.last_variant = L.lib().dbsr_conv_dispatch_variant(d)
    L.check(L.lib().dbsr_conv2d(d, s), 'dbsr_conv2d')
    return y[..., :pc].permute(0, 3, 1, 2).contiguous()


# ---------------------------------------------------------------------------------------------------
# training-step kernels (backward of the ops above; dbsr_hip.h 'training step')
# ---------------------------------------------------------------------------------------------------
def conv2d_wgrad(x, dy, k, compute_dtype=torch.float32, with_bias=False):
    """dL/dW of nn.Conv2d(k x k, stride 1, pad k//2) for input x [N,Cin,H,W] and output gradient dy
    [N,Cout,H,W] (dbsr_conv_wgrad): fp32 [Cout,Cin,k,k].  with_bias: also dL/db = dy.sum((0, 2, 3)) from the
    same pass (dbsr_conv_wgrad_bias), returned as (dw, db)."""
    _need_cuda(x, dy)
    N, Cin, H, W = x.shape
    Cout = dy.shape[1]
    xs, ldx = _nhwc(x, compute_dtype)
    ds, ldd = _nhwc(dy, compute_dtype)
    dw = torch.zeros(Cout, Cin, k, k, dtype=torch.float32, device=x.device)
    need = L.lib().dbsr_conv_wgrad_workspace_bytes(N, H, W, Cin, Cout, k)
    ws = torch.empty(max(need // 4, 1), dtype=torch.float32, device=x.device)
    if not with_bias:
        L.check(L.lib().dbsr_conv_wgrad(N, H, W, L.tensor_desc(xs, ldx), Cin, L.tensor_desc(ds, ldd), Cout, k,
                                        dw.data_ptr(), 0, ws.data_ptr(), need, L.stream_ptr(x.device)),
                'dbsr_conv_wgrad')
        return dw
    db = torch.zeros(Cout, dtype=torch.float32, device=x.device)
    L.check(L.lib().dbsr_conv_wgrad_bias(N, H, W, L.tensor_desc(xs, ldx), Cin, L.tensor_desc(ds, ldd), Cout, k,
                                         dw.data_ptr(), db.data_ptr(), 0, ws.data_ptr(), need,
                                         L.stream_ptr(x.device)), 'dbsr_conv_wgrad_bias')
    return dw, db


def conv2d_dgrad(dy, weight, residual=None, gate=None, compute_dtype=torch.float32):
    """dL/dX of nn.Conv2d(weight, stride 1, pad k//2) for output gradient dy [N,Cout,H,W]: the forward conv
    kernel on dgrad-packed weights (dbsr_dgrad_weights + dbsr_conv_pack_weights), then + residual and
    * (gate > 0) in its epilogue (the ResBlock / ReLU backward).  NCHW fp32/bf16 out."""
    _need_cuda(dy, weight)
    Cout, Cin, kh, kw = weight.shape
    w32 = weight.to(torch.float32).contiguous()
    wt = torch.empty(Cin, Cout, kh, kw, dtype=torch.float32, device=dy.device)
    s = L.stream_ptr(dy.device)
    L.check(L.lib().dbsr_dgrad_weights(w32.data_ptr(), Cout, Cin, kh, kw, wt.data_ptr(), s), 'dbsr_dgrad_weights')
    N, _, H, W = dy.shape
    ds, ldd = _nhwc(dy, compute_dtype)
    n = L.lib().dbsr_conv_packed_elems(Cin, Cout, kh, kw)
    wp = torch.empty(n, dtype=compute_dtype, device=dy.device)
    L.check(L.lib().dbsr_conv_pack_weights(wt.data_ptr(), None, Cin, Cout, kh, kw, L.dtype_code(compute_dtype), 1,
                                           wp.data_ptr(), None, s), 'pack')
    ldy = (Cin + 7) // 8 * 8
    y = torch.zeros(N, H, W, ldy, dtype=compute_dtype, device=dy.device)
    d = L.ConvDesc()
    d.n_frames = N
    d.x = L.tensor_desc(ds, ldd)
    d.in_h, d.in_w, d.cin = H, W, Cout
    d.w, d.bias = wp.data_ptr(), None
    d.cout, d.kh, d.kw, d.stride, d.pad, d.dil = Cin, kh, kw, 1, kh // 2, 1
    d.y = L.tensor_desc(y, ldy)
    d.out_h, d.out_w = H, W
    d.act, d.post_act = L.ACT_NONE, L.ACT_NONE
    keep = []
    if residual is not None:
        rr, ldr = _nhwc(residual, compute_dtype)
        if ldr != ldy:
            rr = torch.nn.functional.pad(rr, (0, ldy - ldr)) if ldr < ldy else rr[..., :ldy].contiguous()
        d.res = L.tensor_desc(rr, ldy)
        keep.append(rr)
    if gate is not None:
        gg, ldg = _nhwc(gate, compute_dtype)
        if ldg != ldy:
            gg = torch.nn.functional.pad(gg, (0, ldy - ldg)) if ldg < ldy else gg[..., :ldy].contiguous()
        d.gate = L.tensor_desc(gg, ldy)
        keep.append(gg)
    d.out_mode, d.shuffle = L.OUT_NHWC, 0
    need = L.lib().dbsr_conv_workspace_bytes(d)
    ws = torch.zeros(max(need // 4, 1), dtype=torch.float32, device=dy.device)
    d.workspace, d.workspace_bytes = ws.data_ptr(), need
    conv2d_dgrad.last_kernel = L.lib().dbsr_conv_kernel_for(d)     # which kernel family ran (tests)
    L.check(L.lib().dbsr_conv2d(d, s), 'dbsr_conv2d (dgrad)')
    return y[..., :Cin].permute(0, 3, 1, 2).contiguous()


def fuse_backward(weights, all_feat, fused, dfused):
    """Softmax-fusion backward (merging.py:116-124): weights / all_feat [B,N,C,H,W], fused / dfused [B,C,H,W]
    -> (dlogits [B,N,C,H,W], dfeat [B,N,C,H,W])."""
    _need_cuda(weights, all_feat, fused, dfused)
    B, N, C, H, W = all_feat.shape
    dt = all_feat.dtype
    nh = lambda t: t.reshape(-1, C, H, W).permute(0, 2, 3, 1).contiguous()          # noqa: E731
    w, f = nh(weights.to(dt)), nh(all_feat)
    fu, dfu = nh(fused.to(dt)), nh(dfused.to(dt))
    dl = torch.empty_like(w)
    df = torch.empty_like(f)
    img = H * W * C
    L.check(L.lib().dbsr_fuse_backward(B, N, H * W, C, L.tensor_desc(w, C, img_stride=img),
                                       L.tensor_desc(f, C, img_stride=img, fmap=(1, N, 0, 1)),
                                       L.tensor_desc(f, C, img_stride=img, fmap=(N - 1, N, 1, 1)),
                                       L.tensor_desc(fu, C, img_stride=img), L.tensor_desc(dfu, C, img_stride=img),
                                       L.tensor_desc(dl, C, img_stride=img),
                                       L.tensor_desc(df, C, img_stride=img, fmap=(1, N, 0, 1)),
                                       L.tensor_desc(df, C, img_stride=img, fmap=(N - 1, N, 1, 1)),
                                       L.stream_ptr(all_feat.device)), 'dbsr_fuse_backward')
    back = lambda t: t.view(B, N, H, W, C).permute(0, 1, 4, 2, 3).contiguous()        # noqa: E731
    return back(dl), back(df)


def warp_backward(dout, flow):
    """dL/dfeat of warp(feat, flow) (warp.py:19-46): dout [N,C,H,W], flow [N,2,H,W] -> fp32 [N,C,H,W]."""
    _need_cuda(dout, flow)
    N, C, H, W = dout.shape
    d = dout.permute(0, 2, 3, 1).contiguous()
    fl = flow.to(torch.float32).contiguous()
    out = torch.zeros(N, H, W, C, dtype=torch.float32, device=dout.device)
    L.check(L.lib().dbsr_warp_backward(N, H, W, C, L.tensor_desc(d, C), fl.data_ptr(), 2 * H * W, out.data_ptr(),
                                       L.FrameMap(1, 1, 0, 1), H * W * C, L.stream_ptr(dout.device)),
            'dbsr_warp_backward')
    return out.permute(0, 3, 1, 2).contiguous()


def warp_backward_gather(dout, flow, gate=None):
    """dL/dfeat of warp(feat, flow) (warp.py:19-46) by the owner-computes gather kernel, optionally times
    [gate > 0] (the encoder's ReLU): dout [N,C,H,W] (fp32 / bf16 / fp16), flow [N,2,H,W], gate like dout ->
    [N,C,H,W] in dout's dtype."""
    _need_cuda(dout, flow)
    N, C, H, W = dout.shape
    dev = dout.device
    d = dout.permute(0, 2, 3, 1).contiguous()
    fl = flow.to(torch.float32).contiguous()
    out = torch.empty_like(d)
    g = gate.to(dout.dtype).permute(0, 2, 3, 1).contiguous() if gate is not None else None
    need = L.lib().dbsr_warp_backward_gather_workspace_bytes(N, H, W)
    ws = torch.empty(need, dtype=torch.uint8, device=dev)
    L.check(L.lib().dbsr_warp_backward_gather(N, H, W, C, L.tensor_desc(d, C), fl.data_ptr(), 2 * H * W,
                                              L.tensor_desc(g, C) if g is not None else L.NULL_TENSOR,
                                              L.tensor_desc(out, C), ws.data_ptr(), need, L.stream_ptr(dev)),
            'dbsr_warp_backward_gather')
    return out.permute(0, 3, 1, 2).contiguous()


def chan_sum(t):
    """Per-channel sum over batch and pixels (the conv bias gradient) of t [N,C,H,W] -> fp32 [C]."""
    _need_cuda(t)
    N, C, H, W = t.shape
    ld = (C + 7) // 8 * 8
    x = torch.zeros(N, H, W, ld, dtype=t.dtype, device=t.device)
    x[..., :C] = t.permute(0, 2, 3, 1)
    out = torch.empty(C, dtype=torch.float32, device=t.device)
    need = L.lib().dbsr_chan_sum_workspace_bytes(N, H * W, C)
    ws = torch.empty(max(need // 4, 1), dtype=torch.float32, device=t.device)
    L.check(L.lib().dbsr_chan_sum(N, H * W, C, L.tensor_desc(x, ld), out.data_ptr(), 0, ws.data_ptr(), need,
                                  L.stream_ptr(t.device)), 'dbsr_chan_sum')
    return out
