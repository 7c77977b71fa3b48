"""ctypes binding of libdbsr_hip.so (C ABI: include/dbsr_hip.h).

torch is imported first so that the library's libamdhip64.so.7 dependency resolves to the HIP
runtime torch already loaded (same SONAME) and kernels share torch's streams and allocations.
There is no fallback: if the library is missing or fails to load, every op raises.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('DBSR_HIP_LIB', os.path.join(_HERE, 'libdbsr_hip.so'))

DBSR_F32, DBSR_BF16, DBSR_F16 = 0, 1, 2
ACT_NONE, ACT_RELU, ACT_LRELU = 0, 1, 2
OUT_NHWC, OUT_SHUFFLE, OUT_NCHW_F32 = 0, 1, 2
ABI_VERSION = 22


class FrameMap(ctypes.Structure):
    _fields_ = [('fpg', ctypes.c_int), ('group_stride', ctypes.c_int), ('group_offset', ctypes.c_int),
                ('inner_stride', ctypes.c_int)]


IDENTITY = (1, 1, 0, 1)


class Tensor(ctypes.Structure):
    _fields_ = [('ptr', ctypes.c_void_p), ('dtype', ctypes.c_int), ('img_stride', ctypes.c_longlong),
                ('ld', ctypes.c_int), ('c0', ctypes.c_int), ('map', FrameMap)]


class PwcDenseConv(ctypes.Structure):
    """dbsr_pwc_dense_conv (include/dbsr_hip.h)."""
    _fields_ = [('w', ctypes.c_void_p), ('bias', ctypes.c_void_p), ('kp', ctypes.c_int), ('cg', ctypes.c_int),
                ('start', ctypes.c_int), ('cout', ctypes.c_int), ('out_off', ctypes.c_int)]


class PwcExtConv(ctypes.Structure):
    """dbsr_pwc_ext_conv (include/dbsr_hip.h)."""
    _fields_ = [('w', ctypes.c_void_p), ('bias', ctypes.c_void_p), ('cin', ctypes.c_int), ('cout', ctypes.c_int),
                ('stride', ctypes.c_int)]


class PackJob(ctypes.Structure):
    """dbsr_pack_job (include/dbsr_hip.h): one conv of a batched repack."""
    _fields_ = [('w', ctypes.c_void_p), ('bias', ctypes.c_void_p), ('w_packed', ctypes.c_void_p),
                ('bias_out', ctypes.c_void_p), ('cout', ctypes.c_int), ('cin', ctypes.c_int), ('kh', ctypes.c_int),
                ('kw', ctypes.c_int), ('dtype', ctypes.c_int), ('shuffle', ctypes.c_int), ('transposed', ctypes.c_int),
                ('lo', ctypes.c_int), ('src_cin', ctypes.c_int), ('pad_', ctypes.c_int), ('blk0', ctypes.c_longlong)]


class ConvDesc(ctypes.Structure):
    _fields_ = [('n_frames', ctypes.c_int),
                ('x', Tensor), ('in_h', ctypes.c_int), ('in_w', ctypes.c_int), ('cin', ctypes.c_int),
                ('w', ctypes.c_void_p), ('bias', ctypes.c_void_p), ('cout', ctypes.c_int), ('kh', ctypes.c_int),
                ('kw', ctypes.c_int), ('stride', ctypes.c_int), ('pad', ctypes.c_int), ('dil', ctypes.c_int),
                ('y', Tensor), ('out_h', ctypes.c_int), ('out_w', ctypes.c_int),
                ('act', ctypes.c_int),
                ('res', Tensor), ('post_act', ctypes.c_int),
                ('out_mode', ctypes.c_int), ('shuffle', ctypes.c_int),
                ('workspace', ctypes.c_void_p), ('workspace_bytes', ctypes.c_size_t), ('precise', ctypes.c_int),
                ('max_blocks', ctypes.c_int), ('gate', Tensor), ('plan_h', ctypes.c_int)]


_lib = None


class DBSRLibError(RuntimeError):
    pass


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise DBSRLibError('libdbsr_hip.so not found at %s: build it with `make` (or __graft_entry__.build())'
                               % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        c_int, c_void_p, c_float, c_ll, c_size_t = (ctypes.c_int, ctypes.c_void_p, ctypes.c_float,
                                                    ctypes.c_longlong, ctypes.c_size_t)
        sigs = {
            'dbsr_abi_version': ([], c_int),
            'dbsr_last_error': ([], ctypes.c_char_p),
            'dbsr_conv_packed_elems': ([c_int, c_int, c_int, c_int], c_size_t),
            'dbsr_weights_round_diffuse': ([c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p], c_int),
            'dbsr_conv_pack_weights': ([c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p,
                                        c_void_p, c_void_p], c_int),
            'dbsr_pack_batch_prepare': ([ctypes.POINTER(PackJob), c_int], c_ll),
            'dbsr_conv_pack_weights_batch': ([c_void_p, c_int, c_ll, c_void_p], c_int),
            'dbsr_conv2d': ([ctypes.POINTER(ConvDesc), c_void_p], c_int),
            'dbsr_set_conv_algo': ([c_int], c_int),
            'dbsr_conv_kernel_for': ([ctypes.POINTER(ConvDesc)], c_int),
            'dbsr_conv_dispatch_variant': ([ctypes.POINTER(ConvDesc)], c_int),
            'dbsr_conv_lane_reach': ([ctypes.POINTER(ConvDesc), c_int], c_int),
            'dbsr_conv_workspace_bytes': ([ctypes.POINTER(ConvDesc)], c_size_t),
            'dbsr_conv2d_head': ([ctypes.POINTER(ConvDesc), c_void_p, c_void_p, c_int, Tensor, c_void_p], c_int),
            'dbsr_conv_head_ok': ([ctypes.POINTER(ConvDesc)], c_int),
            'dbsr_conv_shuffle_blur': ([ctypes.POINTER(ConvDesc), c_void_p, c_void_p], c_int),
            'dbsr_conv_shuffle_blur_ok': ([ctypes.POINTER(ConvDesc)], c_int),
            'dbsr_resblock': ([ctypes.POINTER(ConvDesc), ctypes.POINTER(ConvDesc), c_void_p], c_int),
            'dbsr_resblock_ok': ([ctypes.POINTER(ConvDesc), ctypes.POINTER(ConvDesc)], c_int),
            'dbsr_resblock_head': ([ctypes.POINTER(ConvDesc), ctypes.POINTER(ConvDesc), c_void_p, c_void_p, c_int, Tensor,
                                    c_void_p], c_int),
            'dbsr_correlation': ([c_int, c_int, c_int, c_int, Tensor, Tensor, Tensor, c_int, c_void_p], c_int),
            'dbsr_correlation_backward': ([c_int, c_int, c_int, c_int, Tensor, Tensor, Tensor, Tensor, c_int, Tensor,
                                           Tensor, c_void_p], c_int),
            'dbsr_backwarp': ([c_int, c_int, c_int, c_int, Tensor, Tensor, c_float, Tensor, c_void_p], c_int),
            'dbsr_warp_bilinear': ([c_int, c_int, c_int, c_int, Tensor, c_void_p, c_ll, Tensor, c_void_p], c_int),
            'dbsr_warp_project': ([c_int, c_int, c_int, c_int, Tensor, c_void_p, c_ll, Tensor, c_void_p, c_void_p, c_int,
                                   Tensor, c_void_p], c_int),
            'dbsr_fuse_relu_norm': ([c_int, c_int, c_int, c_int, Tensor, Tensor, Tensor, Tensor, Tensor, c_void_p], c_int),
            'dbsr_burst_mean': ([c_int, c_int, c_int, c_int, Tensor, Tensor, c_void_p], c_int),
            'dbsr_fuse_softmax': ([c_int, c_int, c_int, c_int, Tensor, Tensor, Tensor, Tensor, Tensor, c_void_p],
                                  c_int),
            'dbsr_conv_fuse_softmax': ([ctypes.POINTER(ConvDesc), c_int, c_int, Tensor, Tensor, Tensor, Tensor,
                                        c_void_p], c_int),
            'dbsr_conv_fuse_relu_norm': ([ctypes.POINTER(ConvDesc), c_int, c_int, Tensor, Tensor, Tensor, Tensor,
                                          c_void_p], c_int),
            'dbsr_conv_fuse_ok': ([ctypes.POINTER(ConvDesc), c_int, c_int], c_int),
            'dbsr_fuse_partial': ([c_int, c_int, c_int, c_int, c_int, Tensor, Tensor, Tensor, c_void_p, c_void_p], c_int),
            'dbsr_fuse_combine': ([c_int, c_int, c_int, c_int, c_void_p, Tensor, c_void_p], c_int),
            'dbsr_conv_transpose_k4s2': ([c_int, c_int, c_int, c_int, c_int, Tensor, c_void_p, c_void_p, Tensor,
                                          c_void_p], c_int),
            'dbsr_pack_burst': ([c_int, c_int, c_int, c_int, c_void_p, Tensor, c_int, c_int, Tensor, c_void_p], c_int),
            'dbsr_flow_finalize': ([c_int, c_int, c_int, c_int, Tensor, c_int, c_int, c_int, c_int, c_void_p, c_float,
                                    Tensor, c_void_p], c_int),
            'dbsr_gauss_blur3': ([c_int, c_int, c_int, c_int, Tensor, c_void_p, Tensor, c_void_p], c_int),
            'dbsr_merge_prep': ([c_int, c_int, c_int, c_int, Tensor, Tensor, c_void_p], c_int),
            'dbsr_pwc_assemble': ([c_int, c_int, c_int, c_int, Tensor, Tensor, Tensor, Tensor, c_void_p], c_int),
            'dbsr_zero': ([c_void_p, c_size_t, c_void_p], c_int),
            'dbsr_nhwc_to_nchw_f32': ([c_int, c_int, c_int, Tensor, c_void_p, c_void_p], c_int),
            'dbsr_conv_wgrad_workspace_bytes': ([c_int, c_int, c_int, c_int, c_int, c_int], c_size_t),
            'dbsr_conv_wgrad': ([c_int, c_int, c_int, Tensor, c_int, Tensor, c_int, c_int, c_void_p, c_int, c_void_p,
                                 c_size_t, c_void_p], c_int),
            'dbsr_set_wgrad_algo': ([c_int], c_int),
            'dbsr_conv_wgrad_bias': ([c_int, c_int, c_int, Tensor, c_int, Tensor, c_int, c_int, c_void_p, c_void_p,
                                      c_int, c_void_p, c_size_t, c_void_p], c_int),
            'dbsr_head_forward': ([c_int, c_int, Tensor, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p], c_int),
            'dbsr_head_backward_workspace_bytes': ([c_int, c_int, c_int, c_int], c_size_t),
            'dbsr_head_backward': ([c_int, c_int, Tensor, c_int, Tensor, c_void_p, c_int, Tensor, c_void_p, c_void_p,
                                    c_int, c_void_p, c_size_t, c_void_p], c_int),
            'dbsr_chan_sum_workspace_bytes': ([c_int, c_int, c_int], c_size_t),
            'dbsr_chan_sum': ([c_int, c_int, c_int, Tensor, c_void_p, c_int, c_void_p, c_size_t, c_void_p], c_int),
            'dbsr_l1_loss_backward': ([c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, Tensor, c_void_p,
                                       c_void_p, c_size_t, c_void_p], c_int),
            'dbsr_relu_grad': ([c_int, c_int, c_int, c_int, c_void_p, c_void_p, Tensor, c_void_p], c_int),
            'dbsr_unshuffle_gate': ([c_int, c_int, c_int, c_int, c_int, Tensor, Tensor, Tensor, c_void_p], c_int),
            'dbsr_fuse_backward': ([c_int, c_int, c_int, c_int, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor,
                                    Tensor, c_void_p], c_int),
            'dbsr_merge_prep_backward': ([c_int, c_int, c_int, c_int, Tensor, Tensor, Tensor, c_void_p], c_int),
            'dbsr_warp_backward': ([c_int, c_int, c_int, c_int, Tensor, c_void_p, c_ll, c_void_p, FrameMap, c_ll,
                                    c_void_p], c_int),
            'dbsr_enc_grad_gate': ([c_int, c_int, c_int, c_int, Tensor, c_void_p, Tensor, Tensor, c_void_p], c_int),
            'dbsr_warp_backward_gather_workspace_bytes': ([c_int, c_int, c_int], c_size_t),
            'dbsr_warp_backward_gather': ([c_int, c_int, c_int, c_int, Tensor, c_void_p, c_ll, Tensor, Tensor, c_void_p,
                                           c_size_t, c_void_p], c_int),
            'dbsr_gate_copy': ([c_int, c_int, c_int, Tensor, Tensor, Tensor, c_void_p], c_int),
            'dbsr_adam_step': ([c_ll, c_void_p, c_void_p, c_void_p, c_void_p, c_float, c_float, c_float, c_float, c_int,
                                c_float, c_void_p], c_int),
            'dbsr_dgrad_weights': ([c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p], c_int),
            'dbsr_pwc_dense': ([c_int, c_int, c_int, Tensor, c_int, c_void_p, Tensor, c_void_p], c_int),
            'dbsr_pwc_dense_supported': ([c_int, c_int, c_int], c_int),
            'dbsr_pwc_extract': ([c_int, c_int, c_int, Tensor, c_void_p, c_void_p, c_void_p], c_int),
            'dbsr_pwc_extract_supported': ([c_int, c_int], c_int),
            'dbsr_pwc_level_prep': ([c_int, c_int, c_int, c_int, c_float, Tensor, Tensor, Tensor, Tensor, c_int, Tensor,
                                     c_void_p, c_void_p, c_void_p, c_void_p, c_void_p], c_int),
            'dbsr_pwc_level_prep_supported': ([c_int, c_int, c_int], c_int),
            'dbsr_resize_bilinear': ([c_int, c_int, c_int, c_void_p, c_int, c_int, c_float, c_float, c_float, c_void_p,
                                      c_void_p], c_int),
            'dbsr_gauss_reflect': ([c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p], c_int),
            'dbsr_color_fit': ([c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p], c_int),
            'dbsr_color_apply': ([c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_float, c_void_p, c_int,
                                  c_int, c_float, c_float, c_void_p, c_void_p, c_void_p], c_int),
        }
        for name, (args, res) in sigs.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        if L.dbsr_abi_version() != ABI_VERSION:
            raise DBSRLibError('libdbsr_hip.so ABI %d != expected %d' % (L.dbsr_abi_version(), ABI_VERSION))
        _lib = L
    return _lib


EXPORTED = ['dbsr_abi_version', 'dbsr_last_error', 'dbsr_conv_packed_elems', 'dbsr_conv_pack_weights',
            'dbsr_pack_batch_prepare', 'dbsr_conv_pack_weights_batch',
            'dbsr_weights_round_diffuse', 'dbsr_fuse_relu_norm', 'dbsr_burst_mean', 'dbsr_conv2d',
            'dbsr_set_conv_algo', 'dbsr_conv_kernel_for', 'dbsr_conv_dispatch_variant', 'dbsr_conv_lane_reach', 'dbsr_conv_workspace_bytes', 'dbsr_conv2d_head',
            'dbsr_conv_head_ok', 'dbsr_conv_shuffle_blur', 'dbsr_conv_shuffle_blur_ok', 'dbsr_resblock', 'dbsr_resblock_ok', 'dbsr_resblock_head',
            'dbsr_correlation', 'dbsr_correlation_backward', 'dbsr_backwarp', 'dbsr_warp_bilinear', 'dbsr_warp_project', 'dbsr_fuse_softmax',
            'dbsr_fuse_partial', 'dbsr_fuse_combine', 'dbsr_conv_fuse_softmax', 'dbsr_conv_fuse_relu_norm', 'dbsr_conv_fuse_ok',
            'dbsr_conv_transpose_k4s2', 'dbsr_pack_burst', 'dbsr_flow_finalize', 'dbsr_gauss_blur3',
            'dbsr_merge_prep', 'dbsr_pwc_assemble', 'dbsr_zero', 'dbsr_nhwc_to_nchw_f32', 'dbsr_conv_wgrad_workspace_bytes', 'dbsr_conv_wgrad', 'dbsr_conv_wgrad_bias', 'dbsr_set_wgrad_algo', 'dbsr_head_forward', 'dbsr_head_backward_workspace_bytes', 'dbsr_head_backward',
            'dbsr_chan_sum_workspace_bytes', 'dbsr_chan_sum', 'dbsr_l1_loss_backward', 'dbsr_relu_grad', 'dbsr_unshuffle_gate',
            'dbsr_fuse_backward', 'dbsr_merge_prep_backward', 'dbsr_warp_backward', 'dbsr_enc_grad_gate',
            'dbsr_warp_backward_gather_workspace_bytes', 'dbsr_warp_backward_gather', 'dbsr_gate_copy',
            'dbsr_adam_step', 'dbsr_dgrad_weights',
            'dbsr_resize_bilinear', 'dbsr_gauss_reflect', 'dbsr_color_fit', 'dbsr_color_apply', 'dbsr_pwc_dense',
            'dbsr_pwc_dense_supported', 'dbsr_pwc_extract', 'dbsr_pwc_extract_supported',
            'dbsr_pwc_level_prep', 'dbsr_pwc_level_prep_supported']


def check(rc, what):
    if rc != 0:
        msg = lib().dbsr_last_error().decode(errors='replace')
        raise DBSRLibError('%s failed (rc=%d): %s' % (what, rc, msg))


def dtype_code(dt):
    if dt == torch.float32:
        return DBSR_F32
    if dt == torch.bfloat16:
        return DBSR_BF16
    if dt == torch.float16:
        return DBSR_F16
    raise ValueError('unsupported dtype %s' % dt)


def tensor_desc(t, ld, c0=0, img_stride=None, fmap=IDENTITY, dtype=None):
    """Describe a channel slice [c0, ...) of NHWC images stored in torch tensor `t` (any shape whose
    memory is [images][pixels][ld])."""
    if t is None:
        return Tensor(None, 0, 0, 0, 0, FrameMap(1, 1, 0, 1))
    if img_stride is None:
        img_stride = t[0].numel() if t.dim() > 1 else t.numel()
    return Tensor(t.data_ptr(), dtype_code(t.dtype if dtype is None else dtype), int(img_stride), int(ld), int(c0),
                  FrameMap(*fmap))


NULL_TENSOR = Tensor(None, 0, 0, 0, 0, FrameMap(1, 1, 0, 1))


def stream_ptr(device=None):
    return torch.cuda.current_stream(device).cuda_stream
