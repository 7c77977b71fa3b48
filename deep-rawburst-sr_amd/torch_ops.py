"""torch.ops.dbsr.* -- the HIP kernels as PyTorch operators.

Loading this module loads libdbsr_torch.so (TORCH_LIBRARY(dbsr, m) over the C ABI of libdbsr_hip.so,
csrc/torch/torch_ops.cpp) and registers autograd formulas, so the ops compose with torch autograd the
way the reference's _FunctionCorrelation does (external/pwcnet/correlation/correlation.py:278-383):

    torch.ops.dbsr.correlation(first, second, leaky=False)      FunctionCorrelation (+ the callers'
                                                                leaky_relu with leaky=True)
    torch.ops.dbsr.backwarp(input, flow)                        pwcnet.py:16-38
    torch.ops.dbsr.warp_bilinear(feat, flow)                    warp.py:19-46
    torch.ops.dbsr.fuse_softmax(logits, feats, want_weights)    merging.py:116-126 -> (fused, weights)
    torch.ops.dbsr.conv2d_fused(x, w, b, stride, padding, dilation, act, residual, post_act)

Gradients: correlation w.r.t. both inputs (K3/K4), warp and fusion w.r.t. the features / logits (the
flow is the frozen PWC-Net's output and takes none, encoders.py:56-61).  No CPU kernels: like the
reference's correlation (correlation.py:324-325) the ops raise on CPU tensors.
"""
import os

import torch

from . import _lib

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, 'libdbsr_torch.so')
_loaded = False


def load():
    """Load the operator library once (raises if it is missing: build with `make`)."""
    global _loaded
    if _loaded:
        return torch.ops.dbsr
    _lib.lib()                               # the C-ABI library it links against (ABI version check)
    if not os.path.exists(LIB_PATH):
        raise _lib.DBSRLibError('libdbsr_torch.so not found at %s: build it with `make`' % LIB_PATH)
    torch.ops.load_library(LIB_PATH)
    _register_autograd()
    _loaded = True
    return torch.ops.dbsr


def _register_autograd():
    lib = torch.library

    def corr_setup(ctx, inputs, output):
        first, second, leaky = inputs
        ctx.save_for_backward(first, second, output)
        ctx.leaky = leaky

    def corr_bwd(ctx, grad):
        first, second, out = ctx.saved_tensors
        d1, d2 = torch.ops.dbsr.correlation_backward(grad.contiguous(), first, second, out, ctx.leaky)
        return d1, d2, None

    lib.register_autograd('dbsr::correlation', corr_bwd, setup_context=corr_setup)

    def warp_setup(ctx, inputs, output):
        ctx.save_for_backward(inputs[1])

    def warp_bwd(ctx, grad):
        (flow,) = ctx.saved_tensors
        return torch.ops.dbsr.warp_bilinear_backward(grad.contiguous(), flow), None

    lib.register_autograd('dbsr::warp_bilinear', warp_bwd, setup_context=warp_setup)

    def fuse_setup(ctx, inputs, output):
        logits, feats, want = inputs
        if feats.shape[2] % 8:
            # the forward kernel takes C % 4, the backward C % 8: fail while recording, not in backward()
            raise RuntimeError('dbsr::fuse_softmax: autograd needs C % 8 == 0 (got C = %d)' % feats.shape[2])
        fused, weights = output
        if weights.numel() == 0:           # weights are needed for the backward: recompute them
            _, weights = torch.ops.dbsr.fuse_softmax(logits, feats, True)
        ctx.save_for_backward(weights, feats, fused)

    def fuse_bwd(ctx, dfused, dweights):
        weights, feats, fused = ctx.saved_tensors
        if dweights is not None and dweights.numel() and bool(dweights.abs().sum() != 0):
            raise NotImplementedError('dbsr::fuse_softmax: gradient through the returned weights is not '
                                      'supported (the reference discards them, dbsrnet.py:38)')
        dl, df = torch.ops.dbsr.fuse_backward(weights, feats, fused, dfused.contiguous())
        return dl, df, None

    lib.register_autograd('dbsr::fuse_softmax', fuse_bwd, setup_context=fuse_setup)


def FunctionCorrelation(tenFirst, tenSecond):
    """Drop-in for external/pwcnet/correlation/correlation.py:385-387 (differentiable)."""
    return load().correlation(tenFirst, tenSecond, False)


class ModuleCorrelation(torch.nn.Module):
    """correlation.py:391-396."""
    def forward(self, tenFirst, tenSecond):
        return FunctionCorrelation(tenFirst, tenSecond)
