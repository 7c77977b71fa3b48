"""CPU-only checks of the C ABI: the library loads, exports every function include/dbsr_hip.h
declares, and rejects bad arguments with an error code + message (no GPU work is launched)."""
import ctypes
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, 'include', 'dbsr_hip.h')


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return sorted(set(re.findall(r'\b(dbsr_[a-z0-9_]+)\s*\(', src)))


@pytest.fixture(scope='module')
def L():
    from dbsr_amd import _lib
    _lib.lib()
    return _lib


def test_header_declares_expected(L):
    assert declared_functions() == sorted(L.EXPORTED)


def test_library_exports_all_declared(L):
    raw = ctypes.CDLL(L.LIB_PATH)
    for name in declared_functions():
        assert hasattr(raw, name), name
    assert L.lib().dbsr_abi_version() == L.ABI_VERSION


def test_struct_layout_matches_c():
    from dbsr_amd import _lib
    # dbsr_frame_map 16 B; dbsr_tensor: ptr 8, dtype 4 (+4 pad), img_stride 8, ld 4, c0 4, map 16 -> 48
    assert ctypes.sizeof(_lib.FrameMap) == 16
    assert ctypes.sizeof(_lib.Tensor) == 48
    # conv desc: the C compiler's layout, probed through offsetof-equivalent arithmetic on the fields
    assert _lib.ConvDesc.precise.offset == _lib.ConvDesc.workspace_bytes.offset + 8


def test_splitk_workspace_query(L):
    # a PWC level-6 dense conv (104 pixels, cin 529, cout 32) cannot fill the chip -> split-K
    d = L.ConvDesc()
    d.n_frames = 104
    d.x = L.Tensor(1, L.DBSR_BF16, 544, 544, 0, L.FrameMap(1, 1, 0, 1))
    d.in_h = d.in_w = 1
    d.cin, d.cout, d.kh, d.kw, d.stride, d.pad, d.dil = 529, 32, 3, 3, 1, 1, 1
    d.w = 1
    d.y = L.Tensor(1, L.DBSR_BF16, 544, 544, 0, L.FrameMap(1, 1, 0, 1))
    d.out_h = d.out_w = 1
    assert L.lib().dbsr_conv_workspace_bytes(d) > 0
    d.n_frames, d.in_h, d.in_w, d.out_h, d.out_w = 112, 48, 48, 48, 48      # big conv: no split
    d.cin, d.cout = 4, 64
    d.x.ld = 8
    d.y.ld = 64
    assert L.lib().dbsr_conv_workspace_bytes(d) == 0


def test_pointwise_dispatch(L):
    """dbsr_conv_kernel_for (host logic only): the merge's 1x1 512->64 projection over 104 frames takes the
    pointwise kernel (5), and so does the training dgrad of it (64 -> 512 + residual); fp32, a gate, a
    misaligned residual, a non-power-of-two cin or a tiny pixel count do not."""
    lib = L.lib()
    d = L.ConvDesc()
    d.n_frames = 104
    d.x = L.Tensor(1, L.DBSR_BF16, 48 * 48 * 512, 512, 0, L.FrameMap(1, 1, 0, 1))
    d.in_h = d.in_w = d.out_h = d.out_w = 48
    d.cin, d.cout, d.kh, d.kw, d.stride, d.pad, d.dil = 512, 64, 1, 1, 1, 0, 1
    d.w = 1
    d.y = L.Tensor(1, L.DBSR_BF16, 48 * 48 * 192, 192, 0, L.FrameMap(13, 14, 1, 1))
    d.res = L.NULL_TENSOR
    assert lib.dbsr_conv_kernel_for(d) == 5
    assert lib.dbsr_conv_workspace_bytes(d) == 0
    d.cout = 32
    assert lib.dbsr_conv_kernel_for(d) == 5
    d.cin = 96
    assert lib.dbsr_conv_kernel_for(d) != 5
    d.cin = 512
    d.n_frames, d.in_h, d.in_w, d.out_h, d.out_w = 1, 8, 8, 8, 8          # 64 pixels: generic kernel
    assert lib.dbsr_conv_kernel_for(d) != 5
    d.n_frames, d.in_h, d.in_w, d.out_h, d.out_w = 104, 48, 48, 48, 48
    d.res = L.Tensor(1, L.DBSR_BF16, 48 * 48 * 32, 32, 0, L.FrameMap(1, 1, 0, 1))
    assert lib.dbsr_conv_kernel_for(d) == 5
    d.res = L.Tensor(1, L.DBSR_BF16, 48 * 48 * 36, 36, 0, L.FrameMap(1, 1, 0, 1))   # ld not 16-B aligned
    assert lib.dbsr_conv_kernel_for(d) != 5
    d.res = L.NULL_TENSOR
    d.gate = L.Tensor(1, L.DBSR_BF16, 48 * 48 * 32, 32, 0, L.FrameMap(1, 1, 0, 1))
    assert lib.dbsr_conv_kernel_for(d) != 5
    d.gate = L.NULL_TENSOR
    d.cin, d.cout = 64, 512                                                   # dgrad of the projection
    d.y = L.Tensor(1, L.DBSR_BF16, 48 * 48 * 512, 512, 0, L.FrameMap(1, 1, 0, 1))
    assert lib.dbsr_conv_kernel_for(d) == 5
    d.cin, d.cout = 512, 32
    d.x.dtype = d.y.dtype = L.DBSR_F32
    assert lib.dbsr_conv_kernel_for(d) != 5


def test_packed_size(L):
    # cin 117 -> 128 (cin > 16 pads to 32: 16 groups of 8) * 9 taps = 144 k-groups; cout 128 -> 128 rows;
    # 3x3 with cin > 16: followed by the chunk-major copy of the pipelined kernel (same size)
    assert L.lib().dbsr_conv_packed_elems(128, 117, 3, 3) == 2 * 128 * 144 * 8
    # cin 4 -> 8 (1 group) * 9 taps = 9 -> 12 k-groups; cout 64
    assert L.lib().dbsr_conv_packed_elems(64, 4, 3, 3) == 64 * 12 * 8
    assert L.lib().dbsr_conv_packed_elems(3, 32, 1, 1) == 64 * 4 * 8


def test_conv_rejects_bad_desc(L):
    lib = L.lib()
    assert lib.dbsr_conv2d(None, None) == -1
    assert b'null desc' in lib.dbsr_last_error()
    d = L.ConvDesc()
    d.n_frames = 1
    d.x = L.Tensor(1234, L.DBSR_F32, 100, 12, 0, L.FrameMap(1, 1, 0, 1))     # ld not a multiple of 8
    d.in_h = d.in_w = 4
    d.cin, d.cout, d.kh, d.kw, d.stride, d.pad, d.dil = 4, 8, 3, 3, 1, 1, 1
    d.w = 5678
    d.y = L.Tensor(4321, L.DBSR_F32, 100, 8, 0, L.FrameMap(1, 1, 0, 1))
    d.out_h = d.out_w = 4
    assert lib.dbsr_conv2d(d, None) == -1
    assert b'multiples of 8' in lib.dbsr_last_error()
    d.x.ld = 8
    d.out_h = 5                                                            # inconsistent geometry
    assert lib.dbsr_conv2d(d, None) == -1
    assert b'inconsistent' in lib.dbsr_last_error()


def test_other_ops_reject_null(L):
    lib = L.lib()
    nt = L.NULL_TENSOR
    assert lib.dbsr_correlation(1, 2, 2, 4, nt, nt, nt, 1, None) == -1
    assert lib.dbsr_warp_bilinear(1, 2, 2, 8, nt, None, 0, nt, None) == -1
    assert lib.dbsr_fuse_softmax(1, 2, 4, 8, nt, nt, nt, nt, nt, None) == -1
    assert lib.dbsr_backwarp(1, 2, 2, 4, nt, nt, 1.0, nt, None) == -1


def test_product_refuses_cpu_tensors():
    import torch
    import dbsr_amd
    from dbsr_amd import ops
    net = dbsr_amd.dbsrnet_cvpr2021(**dbsr_amd.DBSR_SYNTHETIC_KWARGS)
    with pytest.raises(RuntimeError):
        net(torch.zeros(1, 3, 4, 48, 48))
    with pytest.raises(NotImplementedError):
        ops.FunctionCorrelation(torch.zeros(1, 8, 4, 4), torch.zeros(1, 8, 4, 4))


def test_torch_ops_registered():
    """libdbsr_torch.so registers the TORCH_LIBRARY(dbsr) schemas with autograd formulas."""
    import torch
    from dbsr_amd import torch_ops
    torch_ops.load()
    names = ['correlation', 'correlation_backward', 'backwarp', 'warp_bilinear', 'warp_bilinear_backward',
             'fuse_softmax', 'fuse_backward', 'conv2d_fused']
    for n in names:
        assert hasattr(torch.ops.dbsr, n), n
    assert 'bool leaky=False' in str(torch.ops.dbsr.correlation.default._schema)
    # HIP implementations only (no CPU kernel, like correlation.py:324-325): CPU tensors fail loudly
    with pytest.raises(NotImplementedError, match="dbsr::correlation.*CPU"):
        torch.ops.dbsr.correlation(torch.zeros(1, 4, 3, 3), torch.zeros(1, 4, 3, 3))


def test_lds_dma_kernels_own_their_simds():
    """Static ISA audit of the shipped code objects (tools/isa_audit.py): every
    kernel issuing LDS-DMA declares the registers its code uses, sets M0 in the same basic block before each
    LDS-DMA instruction, fits its declared LDS, and (DBSR_OWN_SIMDS) claims the whole register file of its
    SIMDs, so a future LDS-DMA kernel without the marker fails here instead of silently racing."""
    import importlib.util
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location('isa_audit', os.path.join(repo, 'tools', 'isa_audit.py'))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    rows, bad = mod.audit(os.path.join(repo, 'deep-rawburst-sr_amd', 'libdbsr_hip.so'))
    assert len(rows) >= 40, 'expected the pipelined / weight-stationary / tiled LDS-DMA kernels'
    assert not bad, bad
