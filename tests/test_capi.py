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


def test_pack_batch_prepare(L):
    """dbsr_pack_batch_prepare (host only, ABI 22): 80-byte jobs; blk0 = the running sum of each job's 256-element
    blocks (the row layout, doubled by the pipe copy for 16-bit 3x3 convs with cin > 16); bad jobs refused."""
    lib = L.lib()
    assert ctypes.sizeof(L.PackJob) == 80 and L.PackJob.blk0.offset == 72
    dummy = 256
    shapes = [(64, 64, 3, 3, L.DBSR_BF16, 1, 0, 0, 0), (64, 4, 3, 3, L.DBSR_BF16, 1, 0, 0, 0),
              (2048, 64, 1, 1, L.DBSR_F16, 8, 0, 0, 0), (128, 128, 3, 3, L.DBSR_F32, 1, 0, 0, 0),
              (64, 128, 3, 3, L.DBSR_BF16, 1, 1, 128, 192)]      # rows [128, 192) of a 192 -> 128 conv's dgrad
    jobs = (L.PackJob * len(shapes))(*[L.PackJob(w=dummy, w_packed=dummy, cout=co, cin=ci, kh=kh, kw=kw, dtype=dt,
                                                 shuffle=sh, transposed=tr, lo=lo, src_cin=sc)
                                       for co, ci, kh, kw, dt, sh, tr, lo, sc in shapes])
    n = lib.dbsr_pack_batch_prepare(jobs, len(shapes))
    blk = 0
    for j, (co, ci, kh, kw, dt, *_rest) in zip(jobs, shapes):
        assert j.blk0 == blk
        rows = lib.dbsr_conv_packed_elems(co, ci, kh, kw)
        if dt == L.DBSR_F32 and kh == 3 and ci > 16:
            rows //= 2                  # (fp32 packs carry no pipe copy; the buffer keeps its room)
        blk += (rows + 255) // 256
    assert n == blk
    bad = [L.PackJob(w=None, w_packed=dummy, cout=64, cin=64, kh=3, kw=3, dtype=L.DBSR_BF16, shuffle=1),
           L.PackJob(w=dummy, w_packed=dummy, cout=60, cin=64, kh=1, kw=1, dtype=L.DBSR_BF16, shuffle=8),
           L.PackJob(w=dummy, w_packed=dummy, cout=64, cin=128, kh=3, kw=3, dtype=L.DBSR_BF16, shuffle=1,
                     transposed=1, lo=160, src_cin=192),
           L.PackJob(w=dummy, w_packed=dummy, cout=64, cin=64, kh=3, kw=3, dtype=7, shuffle=1)]
    for b in bad:
        one = (L.PackJob * 1)(b)
        assert lib.dbsr_pack_batch_prepare(one, 1) == -1
        assert b'pack_batch_prepare' in lib.dbsr_last_error()
    assert lib.dbsr_pack_batch_prepare(jobs, 0) == -1


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
    hazards = []
    rows, bad = mod.audit(os.path.join(repo, 'deep-rawburst-sr_amd', 'libdbsr_hip.so'), hazards)
    assert len(rows) >= 40, 'expected the pipelined / weight-stationary / tiled LDS-DMA kernels'
    assert not hazards, hazards[:5]
    assert not bad, bad


def _isa_audit():
    import importlib.util
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location('isa_audit', os.path.join(repo, 'tools', 'isa_audit.py'))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_isa_audit_store_data_hazard_rule():
    """The store-data hazard rule (the ROCm 7.2 finding of DESIGN.md f2) on hand-written sequences:
    a VALU write to a store's data VGPRs right after it is flagged, for buffer and global stores; wait states
    (s_nop, other instructions) or disjoint registers clear it."""
    hz = _isa_audit().store_data_hazards
    assert hz(['buffer_store_dwordx4 v[4:7], v1, s[0:3], 0 offen', 'v_pk_mul_f32 v[4:5], v[8:9], v[10:11]'])
    assert hz(['global_store_dwordx4 v2, v[4:7], s[0:1]', 'v_mov_b32_e32 v6, 0'])
    assert hz(['global_store_dwordx4 v[2:3], v[4:7], off', 's_nop 0', 'v_add_f32_e32 v7, v1, v2'])
    assert not hz(['buffer_store_dwordx4 v[4:7], v1, s[0:3], 0 offen', 's_nop 1', 'v_pk_mul_f32 v[4:5], v[8:9], v[10:11]'])
    assert not hz(['global_store_dwordx4 v2, v[4:7], s[0:1]', 'v_mov_b32_e32 v8, 0', 'v_mov_b32_e32 v9, 0',
                   'v_mov_b32_e32 v5, 0'])
    assert not hz(['global_store_dwordx4 v2, v[4:7], s[0:1]', 'v_mov_b32_e32 v2, 0'])     # the address, not data
    assert not hz(['buffer_store_dwordx4 v[4:7], v1, s[0:3], 0 offen', 'v_cmp_gt_f32_e32 vcc, v4, v5'])


def _cfg4_decoder_descs(L, rows, full=96, W=96, s=16):
    """ConvDescs of configs[4]'s decoder (fp16, x16; decoders.py:54-62 with default_synthetic's widths) on `rows`
    LR rows of a `full`-row image: (name, desc) in launch order (host logic only, fake pointers)."""
    fm = L.FrameMap(1, 1, 0, 1)

    def desc(cin, cout, k, h, w, ldx, ldy, res=False, act=L.ACT_RELU, post=L.ACT_NONE, out_mode=L.OUT_NHWC,
             shuffle=0, precise=0, scale=1):
        d = L.ConvDesc()
        d.n_frames = 1
        d.x = L.Tensor(1, L.DBSR_F16, h * w * ldx, ldx, 0, fm)
        d.in_h, d.in_w, d.cin = h, w, cin
        d.w = 1
        d.cout, d.kh, d.kw, d.stride, d.pad, d.dil = cout, k, k, 1, k // 2, 1
        yd = L.DBSR_F32 if out_mode == L.OUT_NCHW_F32 else L.DBSR_F16
        d.y = L.Tensor(1, yd, h * w * ldy, ldy, 0, fm)
        d.out_h, d.out_w = h, w
        d.act, d.post_act = act, post
        d.res = L.Tensor(1, L.DBSR_F16, h * w * ldy, ldy, 0, fm) if res else L.NULL_TENSOR
        d.out_mode, d.shuffle, d.precise = out_mode, shuffle, precise
        if rows != full:
            d.plan_h = full * scale
        return d
    out = [('dec.init', desc(512, 64, 3, rows, W, 512, 64))]
    for i in range(5):
        out.append(('dec.pre%d.conv1' % i, desc(64, 64, 3, rows, W, 64, 64)))
        out.append(('dec.pre%d.conv2' % i, desc(64, 64, 3, rows, W, 64, 64, res=True, act=L.ACT_NONE,
                                                post=L.ACT_RELU)))
    out.append(('dec.upsample', desc(64, 32 * s * s, 1, rows, W, 64, 32, out_mode=L.OUT_SHUFFLE, shuffle=s)))
    for i in range(4):
        out.append(('dec.post%d.conv1' % i, desc(32, 32, 3, rows * s, W * s, 32, 32, scale=s)))
        out.append(('dec.post%d.conv2' % i, desc(32, 32, 3, rows * s, W * s, 32, 32, res=True, act=L.ACT_NONE,
                                                 post=L.ACT_RELU, scale=s)))
    out.append(('dec.predictor', desc(32, 3, 1, rows * s, W * s, 32, 1, out_mode=L.OUT_NCHW_F32, precise=1, scale=s)))
    return out


def test_frame_shard_slabs_dispatch_as_whole(L):
    """a frame-sharded rank's decoder slab (configs[4]: 4 ranks, 96x96 LR -> x16) takes, conv for
    conv, the whole image's kernel, tile and K split (dbsr_conv_dispatch_variant, with plan_h), so its rows of the
    prediction are bitwise the unsplit decoder's; without plan_h the 48-row slabs took other kernels (the
    round-3 regression: 16x8 weight-stationary tiles on the whole image, another kernel on the slabs)."""
    from dbsr_amd.parallel import decoder_halo_rows, decoder_slab, shard_range
    lib = L.lib()
    whole = [(n, lib.dbsr_conv_dispatch_variant(d), lib.dbsr_conv_head_ok(d)) for n, d in _cfg4_decoder_descs(L, 96)]
    assert all(v >= 0 for _, v, _ in whole)
    halo = decoder_halo_rows(5, 4, 16, True)
    unpinned_differs = False
    for r in range(4):
        y0, y1 = decoder_slab(*shard_range(96, r, 4), 96, halo)
        assert (y1 - y0) % 16 == 0
        slab = [(n, lib.dbsr_conv_dispatch_variant(d), lib.dbsr_conv_head_ok(d))
                for n, d in _cfg4_decoder_descs(L, y1 - y0)]
        assert slab == whole, (r, [(a, b) for a, b in zip(slab, whole) if a != b])
        for n, d in _cfg4_decoder_descs(L, y1 - y0):
            d.plan_h = 0
            unpinned_differs |= lib.dbsr_conv_dispatch_variant(d) != dict((a, b) for a, b, _ in whole)[n]
    assert unpinned_differs, 'the slab geometry alone no longer changes any dispatch: the test lost its teeth'


def test_plan_h_misfit_rejected(L):
    """A slab whose height cannot take the tile chosen for plan_h fails loudly instead of falling back to
    another kernel (which would change the summation order)."""
    lib = L.lib()
    d = dict(_cfg4_decoder_descs(L, 36))['dec.pre0.conv1']     # 36 rows: not a multiple of the 8-row tile
    d.plan_h = 96                                                # whole image: 16x8 weight-stationary tiles
    assert lib.dbsr_conv_kernel_for(d) == 4
    d.x.ptr, d.y.ptr = 16, 16
    assert lib.dbsr_conv2d(d, None) == -1
    assert b'plan_h' in lib.dbsr_last_error()


def _tight_conv(L, n, h, w, cin, cout, res=False, gate=False):
    """A 16-bit 3x3 conv whose output / residual / gate are tight NHWC tensors (ld == cout, c0 == 0): a lane run
    past cout at the last pixel of the last frame would leave the allocation."""
    d = L.ConvDesc()
    d.n_frames = n
    d.x = L.Tensor(1, L.DBSR_BF16, h * w * cin, cin, 0, L.FrameMap(1, 1, 0, 1))
    d.in_h, d.in_w, d.out_h, d.out_w = h, w, h, w
    d.cin, d.cout, d.kh, d.kw, d.stride, d.pad, d.dil = cin, cout, 3, 3, 1, 1, 1
    d.w = 1
    t = lambda: L.Tensor(1, L.DBSR_BF16, h * w * cout, cout, 0, L.FrameMap(1, 1, 0, 1))   # noqa: E731
    d.y = t()
    d.act = L.ACT_NONE if res else L.ACT_RELU
    d.res = t() if res else L.NULL_TENSOR
    d.post_act = L.ACT_RELU if res else L.ACT_NONE
    d.gate = t() if gate else L.NULL_TENSOR
    return d


@pytest.mark.parametrize('case', [
    # (frames, h, w, cin, cout, residual, gate, expected kernel): partial cout tiles of the pipelined kernel
    # (64-cout tiles: 80, 96; 32-cout tiles: 24) and of the weight-stationary kernel (64: 80, 40; 32: 24)
    (112, 48, 48, 128, 80, True, False, 2), (112, 48, 48, 128, 96, False, True, 2), (112, 48, 48, 128, 80, True, True, 2),
    (8, 128, 128, 64, 24, True, True, 2), (112, 48, 48, 64, 80, False, True, 4), (112, 48, 48, 64, 40, True, True, 4),
    (8, 128, 128, 32, 24, True, True, 4)])
def test_partial_cout_lanes_stay_in_pixel(L, case):
    """VERDICT r4 #5 (the 16-B read past the gate tensor of 390f678): the host model of the lanes' channel
    addressing (dbsr_conv_lane_reach, enumerating the kernels' own pipe_lane_ch / ws_lane_ch) keeps every
    residual / gate read and every store of the last, partial cout tile inside the pixel, for tight tensors."""
    n, h, w, cin, cout, res, gate, kern = case
    lib = L.lib()
    d = _tight_conv(L, n, h, w, cin, cout, res, gate)
    assert lib.dbsr_conv_kernel_for(d) == kern
    wm = 32 if cout <= 32 else 64
    assert (cout - 1) // wm * wm + wm > cout            # the case has a partial cout tile
    for which, on in ((0, True), (1, res), (2, gate)):
        r = lib.dbsr_conv_lane_reach(d, which)
        if on:
            assert 0 <= r <= cout - 1, (which, r)
        else:
            assert r == -1
    assert lib.dbsr_conv_lane_reach(d, 3) == -2


def test_conv_rejects_slices_past_ld(L):
    """A residual / gate slice that does not fit its pixel (c0 + cout > ld) is an argument error, before any
    launch."""
    lib = L.lib()
    d = _tight_conv(L, 112, 48, 48, 128, 80, res=True)
    d.x.ptr = d.y.ptr = d.res.ptr = 1 << 20
    d.res.c0 = 8
    assert lib.dbsr_conv2d(d, None) == -1
    assert b'residual slice exceeds ld' in lib.dbsr_last_error()
    d = _tight_conv(L, 112, 48, 48, 64, 80, gate=True)
    d.x.ptr = d.y.ptr = d.gate.ptr = 1 << 20
    d.gate.ld = 72
    assert lib.dbsr_conv2d(d, None) == -1
    assert b'gate slice exceeds ld' in lib.dbsr_last_error()


def _shuffle_conv(L, n, h, w, cin, cout=2048, shuffle=8, dtype=None, y_ld=32, y_c0=0):
    """The decoder's PixelShuffle upsampling conv (1x1 cin -> cout, shuffle), NHWC 16-bit, descriptor only."""
    dt = L.DBSR_F16 if dtype is None else dtype
    d = L.ConvDesc()
    d.n_frames = n
    cp = 32 if cin <= 32 else 64
    d.x = L.Tensor(1, dt, h * w * cp, cp, 0, L.FrameMap(1, 1, 0, 1))
    d.in_h, d.in_w, d.out_h, d.out_w = h, w, h, w
    d.cin, d.cout, d.kh, d.kw, d.stride, d.pad, d.dil = cin, cout, 1, 1, 1, 0, 1
    d.w = 1
    s2 = shuffle * shuffle
    d.y = L.Tensor(1, dt, h * w * s2 * y_ld, y_ld, y_c0, L.FrameMap(1, 1, 0, 1))
    d.act = L.ACT_RELU
    d.res = L.NULL_TENSOR
    d.gate = L.NULL_TENSOR
    d.out_mode, d.shuffle = L.OUT_SHUFFLE, shuffle
    return d


def test_shuffle_blur_ok_accepts_and_rejects(L):
    """dbsr_conv_shuffle_blur_ok (host-only): the decoder's upsampler at the bench shape is served; shapes the fused
    kernel cannot tile fall back to the two launches (the engine checks _ok first)."""
    lib = L.lib()
    ok = lambda d: lib.dbsr_conv_shuffle_blur_ok(ctypes.byref(d))     # noqa: E731
    assert ok(_shuffle_conv(L, 8, 48, 48, 64)) == 1                  # configs[1]'s decoder
    assert ok(_shuffle_conv(L, 1, 8, 12, 32, y_ld=48, y_c0=8)) == 1  # cin 32, a channel slice
    assert ok(_shuffle_conv(L, 8, 47, 48, 64)) == 0                  # low-res height not a multiple of 4
    assert ok(_shuffle_conv(L, 8, 48, 46, 64)) == 0                  # ... width
    assert ok(_shuffle_conv(L, 8, 48, 48, 128)) == 0                 # cin > 64 (the weights exceed the registers)
    assert ok(_shuffle_conv(L, 8, 48, 48, 64, cout=1024)) == 0       # 16 channels per sub-pixel
    assert ok(_shuffle_conv(L, 8, 48, 48, 64, cout=512, shuffle=4)) == 0
    assert ok(_shuffle_conv(L, 8, 48, 48, 64, dtype=L.DBSR_F32)) == 0
    assert ok(_shuffle_conv(L, 8, 48, 48, 64, y_ld=40, y_c0=12)) == 0   # unaligned slice
    assert ok(_shuffle_conv(L, 8, 48, 48, 64, y_ld=48, y_c0=24)) == 0   # slice past ld


def _rb_pair(L, x_ptr, y_ptr, n=2, h=32, w=64, ld=32):
    """conv1 / conv2 descs of a 32-channel ResBlock x -> y (host-only: fake device addresses)."""
    ident = L.FrameMap(1, 1, 0, 1)

    def conv(xp, yp, act, res=None, post=L.ACT_NONE):
        d = L.ConvDesc()
        d.n_frames = n
        d.x = L.Tensor(xp, L.DBSR_F16, h * w * ld, ld, 0, ident)
        d.in_h, d.in_w, d.out_h, d.out_w = h, w, h, w
        d.cin, d.cout, d.kh, d.kw, d.stride, d.pad, d.dil = 32, 32, 3, 3, 1, 1, 1
        d.w = 1 << 20
        d.y = L.Tensor(yp, L.DBSR_F16, h * w * ld, ld, 0, ident)
        d.act, d.post_act = act, post
        d.res = res if res is not None else L.NULL_TENSOR
        d.gate = L.NULL_TENSOR
        d.out_mode = L.OUT_NHWC
        return d
    mid = 1 << 40
    c1 = conv(x_ptr, mid, L.ACT_RELU)
    c2 = conv(mid, y_ptr, L.ACT_NONE, res=L.Tensor(x_ptr, L.DBSR_F16, h * w * ld, ld, 0, ident), post=L.ACT_RELU)
    return c1, c2


def test_resblock_rejects_output_aliasing_input(L):
    """the persistent ResBlock kernel reads neighbouring tiles' halos of x while other blocks
    store y, so an output overlapping x is refused by dbsr_resblock_ok and by dbsr_resblock (DBSR_E_ARG, before
    any launch); disjoint buffers are accepted."""
    lib = L.lib()
    nbytes = 2 * 32 * 64 * 32 * 2                         # 2 frames of 32x64 pixels x 32 ch x 2 B
    x = 1 << 32
    ok = lambda c1, c2: lib.dbsr_resblock_ok(ctypes.byref(c1), ctypes.byref(c2))   # noqa: E731
    assert ok(*_rb_pair(L, x, x + nbytes)) == 1                               # adjacent, disjoint
    assert ok(*_rb_pair(L, x, x)) == 0                                        # in place
    assert ok(*_rb_pair(L, x, x + nbytes - 64)) == 0                          # last pixel overlaps
    assert ok(*_rb_pair(L, x + nbytes - 64, x)) == 0                          # y's tail under x's head
    c1, c2 = _rb_pair(L, x, x)
    assert lib.dbsr_resblock(ctypes.byref(c1), ctypes.byref(c2), None) == -1                 # DBSR_E_ARG
    assert b'overlap' in lib.dbsr_last_error()


def test_constructor_variants_accepted_and_refused():
    """dbsrnet_cvpr2021 takes the reference's WeightedSum flags softmax / use_base_frame / offset_modulo (the engine
    runs them: engine.merging_variant) and refuses use_offset=False and ref_offset_noise > 0 (merging.py:91-96)."""
    import dbsr_amd
    from dbsr_amd.engine import merging_variant
    kw = dict(enc_init_dim=8, enc_num_res_blocks=1, enc_out_dim=16, dec_init_conv_dim=8, dec_num_pre_res_blocks=1,
              dec_post_conv_dim=32, dec_num_post_res_blocks=1, offset_feat_dim=8, weight_pred_proj_dim=32)
    assert merging_variant(dbsr_amd.dbsrnet_cvpr2021(**kw).merging) == (True, True, 1.0)
    net = dbsr_amd.dbsrnet_cvpr2021(**kw, softmax=False, use_base_frame=False, offset_modulo=None)
    assert merging_variant(net.merging) == (False, False, 0.0)
    assert merging_variant(dbsr_amd.dbsrnet_cvpr2021(**kw, offset_modulo=0.5).merging) == (True, True, 0.5)
    with pytest.raises(NotImplementedError, match='use_offset'):
        dbsr_amd.dbsrnet_cvpr2021(**kw, use_offset=False)
    with pytest.raises(NotImplementedError, match='ref_offset_noise'):
        dbsr_amd.dbsrnet_cvpr2021(**kw, ref_offset_noise=0.1)
    with pytest.raises(ValueError, match='offset_modulo'):
        merging_variant(dbsr_amd.dbsrnet_cvpr2021(**kw, offset_modulo=0.0).merging)
