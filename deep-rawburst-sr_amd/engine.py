"""Forward engine: turns a DBSRNet (parameter tree) into a plan of C-ABI kernel launches.

Per (B, N, H, W, dtype, device) the engine builds a Plan once:
  * persistent channels-last (NHWC) workspace buffers, zero-initialised so that channel padding is
    zero forever (kernels never write pad channels);
  * packed MFMA weights for every conv (dbsr_conv_pack_weights), done once per weight version;
  * a list of prebuilt ctypes argument tuples, one per kernel launch (~140 launches at N=14),
    all on the caller's current stream.
`run()` replays that list; with use_graph the list is captured once into a HIP graph
(torch.cuda.CUDAGraph over the current stream) and replayed as one launch.

Layout map (reference file:line per stage):
  raw     [F,H,W,8]        packed RAW, F = B*N frames              encoders.py:66
  rgb     [F,Hp,Wp,8]      x_rgb resized to a multiple of 64       encoders.py:52, pwcnet.py:262-271
  L1..L6  [F,h,w,C8]       PWC pyramid, computed ONCE per frame (the reference recomputes the
                           reference frame's pyramid for each of its N-1 pairs, encoders.py:53)
  D_l     [P,h,w,448+base] PWC decoder DenseNet buffer; each conv writes its channel slice and
                           reads a channel suffix, so torch.cat never happens (pwcnet.py:173-177)
  E       [F,H,W,512]      frame embeddings                         encoders.py:66-72
  Wf      [P,H,W,512]      warped embeddings of frames 1..N-1      encoders.py:80
  WP      [F,H,W,128]      weight-predictor input [proj | offfeat]  merging.py:77-110 (linearity split:
                           the base term is BS [B,H,W,128], one conv per burst, merging.py:87-89)
  LG      [F,H,W,512]      fusion logits (not with FUSED_WP_OUT)    merging.py:113
  FW      [F,H,W,512]      fusion weights (aux output)              merging.py:118
  FUS     [B,H,W,512]      fused embedding                          merging.py:124
  S*      [B,sH,sW,32]     post-upsampler features                  decoders.py:58-60
"""
import ctypes
import math
import os
import types

import torch

from . import _lib as L
from ._lib import IDENTITY

BACKWARP_SCALE = {5: 0.625, 4: 1.25, 3: 2.5, 2: 5.0}      # fltBackwarp, pwcnet.py:121
PWC_LEVEL_CH = {1: 16, 2: 32, 3: 64, 4: 96, 5: 128, 6: 196}
DENSE_OUT = [128, 128, 96, 64, 32]                         # pwcnet.py:123-146
DENSE_OFF = [320, 192, 96, 32, 0]                          # channel slice of each dense conv output
BASE_OFF = 448                                             # = sum(DENSE_OUT)


def r8(c):
    return (c + 7) // 8 * 8


def cpad(c):
    """Pixel stride for a tensor that convs read: dbsr_conv2d reads cin rounded up to 8 (cin <= 16)
    or 32 (cin > 16) channels (dbsr_hip.h, packed weight layout)."""
    return r8(c) if c <= 16 else (c + 31) // 32 * 32


def pack_convt(mod, device):
    """nn.ConvTranspose2d weight [cin][cout][4][4] -> [ky][kx][cout][cin8] fp32 (dbsr_conv_transpose_k4s2)."""
    w = mod.weight.detach().to(device=device, dtype=torch.float32)
    cin = w.shape[0]
    w = w.permute(2, 3, 1, 0).contiguous()
    w = torch.nn.functional.pad(w, (0, r8(cin) - cin)).contiguous()
    return w, mod.bias.detach().to(device=device, dtype=torch.float32).contiguous()


def gauss_kernel3(sd, ksz=3):
    """PixShuffleUpsampler._get_gaussian_kernel (upsampling.py:24-29) via gauss_2d (filtering.py:20-40)."""
    k = torch.arange(-(ksz - 1) / 2, (ksz + 1) / 2, dtype=torch.float32).reshape(1, -1)
    g1 = torch.exp(-1.0 / (2 * sd ** 2) * k ** 2) / (math.sqrt(2 * math.pi) * sd)
    K = g1.reshape(1, 1, -1) * g1.reshape(1, -1, 1)
    K = K / K.sum()
    return [float(v) for v in K.reshape(-1)]


def merging_variant(mer):
    """The WeightedSum constructor flags the engine honours (merging.py:23-32, 79-121) as
    (softmax, use_base_frame, offset_modulo for dbsr_flow_finalize: 0.0 = None, no remainder).
    use_offset=False and ref_offset_noise > 0 (the latter draws torch.rand inside the forward) are refused."""
    if not getattr(mer, 'use_offset', True):
        raise NotImplementedError('WeightedSum(use_offset=False) is not on the HIP path (merging.py:91)')
    if getattr(mer, 'ref_offset_noise', 0.0) > 0.0:
        raise NotImplementedError('WeightedSum(ref_offset_noise > 0) is not on the HIP path: it draws random '
                                  'reference offsets inside the forward (merging.py:92-96)')
    m = getattr(mer, 'offset_modulo', None)
    if m is not None and float(m) == 0.0:
        raise ValueError('offset_modulo must be None or nonzero (x % 0 is NaN in the reference)')
    return (bool(getattr(mer, 'softmax', True)), bool(getattr(mer, 'use_base_frame', False)),
            0.0 if m is None else float(m))


class NHWC:
    """Persistent buffer of n images of h x w pixels with ld elements per pixel."""
    def __init__(self, n, h, w, ld, dtype, device):
        self.n, self.h, self.w, self.ld, self.dtype = n, h, w, ld, dtype
        self.t = torch.zeros(n, h, w, ld, dtype=dtype, device=device)

    def d(self, c0=0, fmap=IDENTITY):
        return L.tensor_desc(self.t, self.ld, c0, img_stride=self.h * self.w * self.ld, fmap=fmap)

    def rows(self, y0, y1):
        """Rows [y0, y1) of every image as an image of y1 - y0 rows (a view: convs treat the rows outside it
        as zero padding)."""
        v = NHWC.__new__(NHWC)
        v.n, v.h, v.w, v.ld, v.dtype = self.n, y1 - y0, self.w, self.ld, self.dtype
        v.t = self.t[:, y0:y1]
        v.full_h = self.h
        v.d = lambda c0=0, fmap=IDENTITY: L.tensor_desc(v.t, v.ld, c0, img_stride=self.h * self.w * self.ld,
                                                        fmap=fmap)
        return v


class DBSRAux(dict):
    """aux of DBSRNet.forward, {'offsets', 'fusion_weights'} as dbsrnet.py:38 returns it.  'fusion_weights' is
    the reference's tensor -- fp32, contiguous [B,N,C,H,W] (merging.py:117-126) -- materialised from the
    engine's channels-last buffer by dbsr_nhwc_to_nchw_f32 the first time it is read (the reference's callers
    never read it, so a forward does not pay for the transpose); `native_fusion_weights` is the zero-copy
    [B,N,C,H,W] view of the channels-last buffer in the compute dtype."""

    def __init__(self, offsets, native_fw):
        super().__init__(offsets=offsets, fusion_weights=None)
        self.native_fusion_weights = native_fw          # [B,N,C,H,W] view of [B*N,H,W,C] storage, or None
        self._done = native_fw is None

    def _materialize(self):
        if self._done:
            return
        v = self.native_fusion_weights
        B, N, C, H, W = v.shape
        src = v.permute(0, 1, 3, 4, 2)                  # back to the storage order [B,N,H,W,C]
        out = torch.empty(B, N, C, H, W, dtype=torch.float32, device=v.device)
        L.check(L.lib().dbsr_nhwc_to_nchw_f32(B * N, H * W, C, L.tensor_desc(src, src.stride(-2), 0,
                                                                               img_stride=src.stride(1)),
                                              out.data_ptr(), L.stream_ptr(v.device)), 'dbsr_nhwc_to_nchw_f32')
        dict.__setitem__(self, 'fusion_weights', out)
        self._done = True

    def __getitem__(self, k):
        if k == 'fusion_weights':
            self._materialize()
        return dict.__getitem__(self, k)

    def get(self, k, default=None):
        if k == 'fusion_weights':
            self._materialize()
        return dict.get(self, k, default)

    def items(self):
        self._materialize()
        return dict.items(self)

    def values(self):
        self._materialize()
        return dict.values(self)

    def copy(self):
        self._materialize()
        return dict(self)


class PackedConv:
    """One nn.Conv2d packed for dbsr_conv2d.  recipe() -> (weight, bias | None) gives the source tensors
    (default: the module's own); repack() re-packs them into the same buffers, so plans and captured graphs
    that point at them stay valid."""
    def __init__(self, conv, dtype, device, stream, shuffle=1, recipe=None, rounding='nearest'):
        """rounding (16-bit dtypes): 'nearest' rounds each weight to its nearest 16-bit value; 'diffuse' rounds each
        output channel's weights in K order with the running error carried (dbsr_weights_round_diffuse: the error
        sum per channel stays within half an ulp, which the fp16 forward's error is most sensitive to)."""
        self.recipe = recipe or (lambda: (conv.weight, conv.bias))
        self.dtype, self.device, self.shuffle = dtype, device, shuffle
        self.rounding = rounding if dtype in (torch.float16, torch.bfloat16) else 'nearest'
        w, b = self.recipe()
        self.cout, self.cin, self.kh, self.kw = w.shape
        self.stride, self.pad, self.dil = conv.stride[0], conv.padding[0], conv.dilation[0]
        n = L.lib().dbsr_conv_packed_elems(self.cout, self.cin, self.kh, self.kw)
        self.w = torch.empty(n, dtype=dtype, device=device)
        self.bias = torch.empty(self.cout, dtype=torch.float32, device=device) if b is not None else None
        self.repack(stream)

    def repack(self, stream):
        w, b = self.recipe()
        w = w.detach().to(device=self.device, dtype=torch.float32).contiguous()
        b = b.detach().to(device=self.device, dtype=torch.float32).contiguous() if b is not None else None
        if self.rounding == 'diffuse':
            wr = torch.empty_like(w)
            L.check(L.lib().dbsr_weights_round_diffuse(w.data_ptr(), self.cout, self.cin, self.kh, self.kw,
                                                       L.dtype_code(self.dtype), wr.data_ptr(), stream),
                    'dbsr_weights_round_diffuse')
            w = wr                      # 16-bit-representable values: the pack's own rounding keeps them
        L.check(L.lib().dbsr_conv_pack_weights(w.data_ptr(), b.data_ptr() if b is not None else None, self.cout,
                                               self.cin, self.kh, self.kw, L.dtype_code(self.dtype), self.shuffle,
                                               self.w.data_ptr(),
                                               self.bias.data_ptr() if self.bias is not None else None, stream),
                'dbsr_conv_pack_weights')
        self._keep = (w, b)             # (the launch reads them asynchronously)

    def out_hw(self, h, w):
        return ((h + 2 * self.pad - self.dil * (self.kh - 1) - 1) // self.stride + 1,
                (w + 2 * self.pad - self.dil * (self.kw - 1) - 1) // self.stride + 1)


class Plan:
    """A forward as a flat list of C-ABI launches over preallocated buffers, on one or more lanes.

    Lane 0 is the caller's stream; every other lane is a side stream that `fork` starts (it waits for
    all lane-0 work issued so far) and `join` ends (lane 0 waits for it).  Independent sub-graphs (the
    PWC-Net alignment vs the feature encoder) overlap this way, in eager mode and inside a HIP graph
    capture alike.
    """
    FORK, JOIN = '__fork__', '__join__'
    # Two lanes: PWC-Net + the offset-feature extractor on a side stream beside the frame encoder.  Safe
    # because the LDS-DMA/MFMA conv kernels own their SIMDs (DBSR_OWN_SIMDS, csrc/common.hpp): waves of
    # another stream's kernels sharing a CU with them computed wrong values (DESIGN.md 'two-lane race').
    # tests/test_gpu_parity.py::test_bench_shape_two_lanes_bitwise holds the two lanes bit-identical to
    # one stream.  DBSR_SINGLE_STREAM=1 runs everything on the caller's stream.
    MULTI_STREAM = os.environ.get('DBSR_SINGLE_STREAM', '0') != '1'

    def __init__(self):
        self.ops = []        # (callable | FORK | JOIN, args, name, lane)
        self.keep = []
        self.work = {}       # op index -> ('flop' | 'byte', algorithmic amount per launch)
        self.kernel = {}     # op index -> kernel family (convs)
        self.hbm = {}        # op index -> algorithmic HBM bytes per launch of the fused conv kernels (bench.py)
        self.convs = []      # (ConvDesc, lane): each lane shares one split-K workspace
        self.lane = 0
        self.lanes = {0}
        self.streams = {}
        self.max_blocks = 0  # CU cap for lane-0 persistent convs issued while a side lane runs
        self.max_blocks_cap = 0
        self.early_names, self.early_cap = (), 0   # lane-0 convs capped at early_cap instead (DBSREngine.LANE0_EARLY_*)
        self.plan_rows = None  # (slab rows, whole-image rows): convs dispatch as on the whole image (plan_h)

    def add(self, name, fn, *args, work=None):
        if work is not None:
            self.work[len(self.ops)] = work
        self.ops.append((fn, args, name, self.lane))

    def fork(self, lane, device, priority=0):
        """Following ops go to side stream `lane`, ordered after everything issued so far on lane 0."""
        assert self.lane == 0 and lane != 0
        if not Plan.MULTI_STREAM:
            return
        if lane not in self.streams:
            self.streams[lane] = Plan.side_stream(device, lane, priority)
        self.lanes.add(lane)
        self.ops.append((Plan.FORK, (torch.cuda.Event(),), f'sync.fork{lane}', lane))
        self.lane = lane

    _side_streams = {}

    @staticmethod
    def side_stream(device, lane, priority):
        """One side stream per (device, lane, priority) for the whole process, shared by every plan (the plans
        of a process are ordered on the caller's stream anyway; a stream per plan only multiplied the HIP
        streams, and hence the hardware-queue sharing, of a process)."""
        dev = torch.device(device)
        key = (dev.index if dev.index is not None else torch.cuda.current_device(), lane, priority)
        st = Plan._side_streams.get(key)
        if st is None:
            st = Plan._side_streams[key] = torch.cuda.Stream(device=device, priority=priority)
        return st

    def switch(self, lane):
        """Following ops go to `lane` (an already forked side lane, or 0), with no ordering edge."""
        assert lane == 0 or lane in self.streams or not Plan.MULTI_STREAM
        self.lane = lane if Plan.MULTI_STREAM else 0

    def join(self, lane):
        """Lane 0 waits for all work issued so far on side lane `lane`; following ops go to lane 0."""
        if not Plan.MULTI_STREAM:
            return
        assert lane != 0 and lane in self.streams
        self.ops.append((Plan.JOIN, (torch.cuda.Event(),), f'sync.join{lane}', lane))
        self.lane = 0

    def conv(self, name, pc, n_frames, x, xc0, in_hw, y, yc0, act, xmap=IDENTITY, ymap=IDENTITY, res=None,
             rc0=0, rmap=IDENTITY, post_act=L.ACT_NONE, out_mode=L.OUT_NHWC, shuffle=0, y_desc=None, cin=None,
             precise=False, head=None, gate=None, gc0=0, gmap=IDENTITY):
        """Emit one conv.  head = (name, w [hc, cout] fp32, b [hc] | None, out_desc): when the library can fuse
        it (dbsr_conv_head_ok), the conv's own output is not stored and the 1x1 head + ReLU writes out_desc
        (fp32 NCHW); the returned desc then has .fused_head = True.  gate: output *= (gate > 0) (training
        dgrad: the ReLU backward of the layer that produced the forward conv's input)."""
        d = self._desc(name, pc, n_frames, x, xc0, in_hw, y, yc0, act, xmap, ymap, res, rc0, rmap, post_act,
                       out_mode, shuffle, y_desc, cin, precise, gate, gc0, gmap)
        self.convs.append((d, self.lane))
        oh, ow = d.out_h, d.out_w
        flop = 2.0 * n_frames * oh * ow * pc.cout * d.cin * pc.kh * pc.kw
        d.fused_head = bool(head is not None and L.lib().dbsr_conv_head_ok(ctypes.byref(d)))
        if d.fused_head:
            hname, hw, hb, hdesc = head
            self.keep.extend([hw, hb, hdesc])
            flop += 2.0 * n_frames * oh * ow * hw.shape[0] * hw.shape[1]
            self.add(name + '+' + hname, L.lib().dbsr_conv2d_head, ctypes.byref(d), hw.data_ptr(),
                     hb.data_ptr() if hb is not None else None, hw.shape[0], hdesc, work=('flop', flop))
            self.kernel[len(self.ops) - 1] = 'conv3x3_pipe'
            return d
        self.add(name, L.lib().dbsr_conv2d, ctypes.byref(d), work=('flop', flop))
        self.kernel[len(self.ops) - 1] = {4: 'conv3x3_ws', 7: 'conv3x3_ks128', 2: 'conv3x3_pipe', 1: 'conv3x3_tiled', 3: 'conv1x1_shuffle', 5: 'conv1x1', 6: 'conv3x3_narrow', 8: 'conv3x3_small'}.get(L.lib().dbsr_conv_kernel_for(d),
                                                                                      'conv2d_generic')
        return d

    def conv_fuse(self, name, pc, B, N, x, in_hw, ref, oth, fused, weights, xmap=IDENTITY, softmax=True):
        """The weight predictor's last conv + softmax over the burst + fusion in one launch
        (dbsr_conv_fuse_softmax: the logits never reach memory; softmax=False: dbsr_conv_fuse_relu_norm).  Returns
        the op index, or None when the library does not serve the shape (the caller then emits the conv and
        dbsr_fuse_softmax / dbsr_fuse_relu_norm)."""
        d = self._desc(name, pc, B * N, x, 0, in_hw, None, 0, L.ACT_NONE, xmap, IDENTITY, None, 0, IDENTITY,
                       L.ACT_NONE, L.OUT_NHWC, 0, L.NULL_TENSOR, None, False, None, 0, IDENTITY)
        if not L.lib().dbsr_conv_fuse_ok(ctypes.byref(d), B, N):
            return None
        H, W = in_hw
        flop = 2.0 * B * N * H * W * pc.cout * d.cin * pc.kh * pc.kw
        fn = L.lib().dbsr_conv_fuse_softmax if softmax else L.lib().dbsr_conv_fuse_relu_norm
        self.add(name, fn, ctypes.byref(d), B, N, ref, oth, fused, weights,
                 work=('flop', flop))
        self.kernel[len(self.ops) - 1] = 'conv_fuse'
        # hidden input + the N frames' features in + fusion weights out (when written) + fused out
        es, C = (4 if x.dtype == torch.float32 else 2), pc.cout
        self.hbm[len(self.ops) - 1] = es * B * H * W * (N * d.cin + N * C + (N * C if weights.ptr else 0) + C)
        return len(self.ops) - 1

    def resblock(self, name, c1, c2, n_frames, x, mid, y, hw, head=None, yc0=0):
        """ResBlock (blocks.py:81-96) x -> y (channels from yc0) as one launch (dbsr_resblock: the intermediate stays
        in the LDS; 32 channels: the decoder's post blocks, 64: the encoder / offset-feature / decoder pre blocks)
        when the library serves it; returns False otherwise (the caller then emits conv1 into `mid` and conv2).
        head = (name, w [hc, 32] fp32, b | None, out_desc): the RGB predictor fused as well (dbsr_resblock_head;
        y is then not written)."""
        d1 = self._desc(name + '.conv1', c1, n_frames, x, 0, hw, mid, 0, L.ACT_RELU, IDENTITY, IDENTITY, None, 0,
                        IDENTITY, L.ACT_NONE, L.OUT_NHWC, 0, None, None, False, None, 0, IDENTITY)
        d2 = self._desc(name + '.conv2', c2, n_frames, mid, 0, hw, y, yc0, L.ACT_NONE, IDENTITY, IDENTITY, x, 0,
                        IDENTITY, L.ACT_RELU, L.OUT_NHWC, 0, None, None, False, None, 0, IDENTITY)
        if (c1.cout == 64 and not DBSREngine.FUSED_RESBLOCK64) or \
                not L.lib().dbsr_resblock_ok(ctypes.byref(d1), ctypes.byref(d2)):
            return False
        self.convs.extend([(d1, self.lane), (d2, self.lane)])
        oh, ow = d1.out_h, d1.out_w
        flop = 2.0 * n_frames * oh * ow * (c1.cout * d1.cin * 9 + c2.cout * d2.cin * 9)
        if head is not None:
            hname, hw_, hb, hdesc = head
            self.keep.extend([hw_, hb, hdesc])
            flop += 2.0 * n_frames * oh * ow * hw_.shape[0] * hw_.shape[1]
            self.add(name + '+' + hname, L.lib().dbsr_resblock_head, ctypes.byref(d1), ctypes.byref(d2),
                     hw_.data_ptr(), hb.data_ptr() if hb is not None else None, hw_.shape[0], hdesc,
                     work=('flop', flop))
        else:
            self.add(name, L.lib().dbsr_resblock, ctypes.byref(d1), ctypes.byref(d2), work=('flop', flop))
        self.kernel[len(self.ops) - 1] = 'resblock32' if c1.cout == 32 else 'resblock64'
        # x in once; y out (16-bit) or the head's fp32 NCHW planes
        self.hbm[len(self.ops) - 1] = n_frames * oh * ow * (2 * d1.cin + (4 * head[1].shape[0] if head is not None
                                                                         else 2 * c2.cout))
        return True

    def conv_shuffle_blur(self, name, pc, n_frames, x, in_hw, y, act, k9):
        """The PixelShuffle upsampler's conv + shuffle + 3x3 Gaussian blur in one launch
        (dbsr_conv_shuffle_blur: the pre-blur tensor never reaches memory; upsampling.py:51-66).  Returns the
        desc, or None when the library does not serve the shape (the caller then emits the conv and the blur)."""
        d = self._desc(name, pc, n_frames, x, 0, in_hw, y, 0, act, IDENTITY, IDENTITY, None, 0, IDENTITY,
                       L.ACT_NONE, L.OUT_SHUFFLE, pc.shuffle, None, None, False, None, 0, IDENTITY)
        if not L.lib().dbsr_conv_shuffle_blur_ok(ctypes.byref(d)):
            return None
        kbuf = (ctypes.c_float * 9)(*k9)
        self.keep.append(kbuf)
        self.convs.append((d, self.lane))
        flop = 2.0 * n_frames * d.out_h * d.out_w * pc.cout * d.cin
        self.add(name, L.lib().dbsr_conv_shuffle_blur, ctypes.byref(d), kbuf, work=('flop', flop))
        self.kernel[len(self.ops) - 1] = 'conv1x1_shuffle_blur'
        # low-res input in, the blurred high-res output out (16-bit)
        s = pc.shuffle
        self.hbm[len(self.ops) - 1] = 2 * n_frames * d.out_h * d.out_w * (d.cin + pc.cout // (s * s) * s * s)
        return d

    def _desc(self, name, pc, n_frames, x, xc0, in_hw, y, yc0, act, xmap, ymap, res, rc0, rmap, post_act, out_mode,
              shuffle, y_desc, cin, precise, gate, gc0, gmap):
        oh, ow = pc.out_hw(*in_hw)
        assert cin is None or cin == pc.cin, (name, cin, pc.cin)
        d = L.ConvDesc()
        d.n_frames = n_frames
        d.x = x.d(xc0, xmap)
        d.in_h, d.in_w = in_hw
        d.cin = pc.cin if cin is None else cin
        d.w = pc.w.data_ptr()
        d.bias = pc.bias.data_ptr() if pc.bias is not None else None
        d.cout, d.kh, d.kw, d.stride, d.pad, d.dil = pc.cout, pc.kh, pc.kw, pc.stride, pc.pad, pc.dil
        d.y = y_desc if y_desc is not None else y.d(yc0, ymap)
        d.out_h, d.out_w = oh, ow               # (OUT_SHUFFLE: the kernel scales by `shuffle` itself)
        d.act = act
        d.res = res.d(rc0, rmap) if res is not None else L.NULL_TENSOR
        d.gate = gate.d(gc0, gmap) if gate is not None else L.NULL_TENSOR
        d.post_act = post_act
        d.out_mode, d.shuffle = out_mode, shuffle
        d.workspace, d.workspace_bytes = None, 0
        d.precise = 1 if precise else 0
        d.max_blocks = (self.early_cap if name in self.early_names and self.max_blocks else self.max_blocks) \
            if self.lane == 0 else 0
        if self.plan_rows is not None:
            slab, full = self.plan_rows
            if oh % slab == 0:
                d.plan_h = full * (oh // slab)
        self.keep.append(d)
        return d

    def finalize_workspace(self, device):
        """Allocate one fp32 split-K scratch per lane (the convs of a lane run in order on its stream;
        lanes run concurrently) and point every ConvDesc at its lane's scratch."""
        assert self.lane == 0, 'unjoined side lane'
        self.ws = {}
        for lane in sorted(self.lanes):
            ds = [d for d, ln in self.convs if ln == lane]
            need = max([L.lib().dbsr_conv_workspace_bytes(d) for d in ds] + [0])
            self.ws[lane] = torch.zeros(max(need // 4, 1), dtype=torch.float32, device=device)
            for d in ds:
                d.workspace, d.workspace_bytes = self.ws[lane].data_ptr(), need

    def run(self, stream):
        main = torch.cuda.current_stream()
        if self.streams:
            assert main.cuda_stream == stream, 'Plan.run: lanes fork from the current stream'
        for fn, args, name, lane in self.ops:
            if fn is Plan.FORK:
                args[0].record(main)
                self.streams[lane].wait_event(args[0])
            elif fn is Plan.JOIN:
                args[0].record(self.streams[lane])
                main.wait_event(args[0])
            else:
                rc = fn(*args, stream if lane == 0 else self.streams[lane].cuda_stream)
                if rc != 0:
                    L.check(rc, name)

    def run_list(self, ops, stream):
        """Launch `ops` (no fork/join entries) in order on one stream."""
        for fn, args, name, lane in ops:
            if fn is Plan.FORK or fn is Plan.JOIN:
                continue
            rc = fn(*args, stream)
            if rc != 0:
                L.check(rc, name)

    def time_ops(self, stream, reps=10, full_chip=True):
        """Average device time (ms) of each op, each launched `reps` times back to back between two
        HIP events on `stream` (all lanes serialised onto it; fork/join entries report 0).

        full_chip: the lane-0 convs that the plan caps to part of the CUs while the PWC-Net lane runs beside
        them (max_blocks) are timed uncapped, i.e. as kernels on the whole chip -- serialised here, nothing
        else runs beside them, so a capped time would price the idle CUs into the kernel."""
        capped = [(d, d.max_blocks) for d, _ in self.convs if d.max_blocks] if full_chip else []
        for d, _ in capped:
            d.max_blocks = 0
        try:
            return self._time_ops(stream, reps)
        finally:
            for d, mb in capped:
                d.max_blocks = mb

    def time_ops_in_step(self, stream, reps=3, hold_cycles=40_000_000):
        """Average device time (ms) of each op inside a forward run the way the step runs it: every lane on its
        own stream, the side lane concurrent with lane 0 and the lane-0 convs capped while it runs.  Each op is
        bracketed by HIP events on the stream it runs on; the whole forward is queued behind a spin kernel
        (`hold_cycles`) first, so host launch gaps never fall inside an op's events.  Unlike time_ops, the
        durations include the sharing of the chip between the lanes (they overlap: their sum exceeds the step)."""
        main = torch.cuda.current_stream()
        assert main.cuda_stream == stream, 'time_ops_in_step: lanes fork from the current stream'
        tot = [0.0] * len(self.ops)
        for _ in range(reps):
            torch.cuda._sleep(hold_cycles)
            evs = []
            for fn, args, name, lane in self.ops:
                if fn is Plan.FORK:
                    args[0].record(main)
                    self.streams[lane].wait_event(args[0])
                    evs.append(None)
                    continue
                if fn is Plan.JOIN:
                    args[0].record(self.streams[lane])
                    main.wait_event(args[0])
                    evs.append(None)
                    continue
                st = main if lane == 0 else self.streams[lane]
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                rc = fn(*args, stream if lane == 0 else st.cuda_stream)
                if rc != 0:
                    L.check(rc, name)
                e1.record(st)
                evs.append((e0, e1))
            torch.cuda.synchronize()
            for i, ev in enumerate(evs):
                if ev is not None:
                    tot[i] += ev[0].elapsed_time(ev[1])
        return [(name, t / reps) for (fn, args, name, lane), t in zip(self.ops, tot)]

    def _time_ops(self, stream, reps):
        out = []
        for fn, args, name, lane in self.ops:
            if fn is Plan.FORK or fn is Plan.JOIN:
                out.append((name, 0.0))
                continue
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            fn(*args, stream)
            # the reps queue up behind a spin kernel, so they run back to back on the device: a short kernel
            # (~10 us) is otherwise timed at the host's launch rate (ctypes + HIP launch per call)
            torch.cuda._sleep(2_000_000)
            e0.record()
            for _ in range(reps):
                fn(*args, stream)
            e1.record()
            e1.synchronize()
            out.append((name, e0.elapsed_time(e1) / reps))
        return out


class _Weights:
    """All packed weights of a DBSRNet / PWCNet for one (dtype, device)."""
    def __init__(self, dtype, device, stream, rounding='nearest'):
        self.dtype, self.device, self.stream, self.rounding = dtype, device, stream, rounding

    def conv(self, module, shuffle=1, recipe=None):
        return PackedConv(module, self.dtype, self.device, self.stream, shuffle=shuffle, recipe=recipe,
                          rounding=self.rounding)


def _param_signature(module):
    return tuple((p.data_ptr(), p._version) for p in module.parameters())


# ==================================================================================================
# PWC-Net sub-plan
# ==================================================================================================
class PWCPlanner:
    """Packs PWC-Net weights and emits the PWC part of a plan (pwcnet.py:221-231 + :262-279)."""
    FUSED_DENSE = True        # 16-bit coarse levels (<= 64 pixels per pair): dbsr_pwc_dense
    FUSED_EXTRACT = True      # 16-bit 64x64 frames: the whole feature pyramid in one launch (dbsr_pwc_extract)
    FUSED_PREP = True         # 16-bit: each decoder level's ConvTs, backwarp, correlation, assembly in one launch
    def __init__(self, pwc_module, W):
        net = pwc_module.net
        ex = net.netExtractor
        self.ext = []
        for lvl in ['netOne', 'netTwo', 'netThr', 'netFou', 'netFiv', 'netSix']:
            seq = getattr(ex, lvl)
            self.ext.append([W.conv(seq[0]), W.conv(seq[2]), W.conv(seq[4])])
        self.dec = {}
        for level, name in zip([2, 3, 4, 5, 6], ['netTwo', 'netThr', 'netFou', 'netFiv', 'netSix']):
            d = getattr(net, name)
            ent = {'dense': [W.conv(getattr(d, n)[0]) for n in ['netOne', 'netTwo', 'netThr', 'netFou', 'netFiv']],
                   'flow': W.conv(d.netSix[0])}
            if level < 6:
                ent['upflow'] = pack_convt(d.netUpflow, W.device)
                ent['upfeat'] = pack_convt(d.netUpfeat, W.device)
                if W.dtype != torch.float32:
                    # 16-bit rows [(ky*4+kx)*2 + co][cin32] for dbsr_pwc_level_prep's MFMA ConvT
                    wt = ent['upfeat'][0]
                    cin = wt.shape[-1]
                    ent['upfeat16'] = torch.nn.functional.pad(wt.reshape(32, cin), (0, (cin + 31) // 32 * 32 - cin)) \
                        .to(W.dtype).contiguous()
            self.dec[level] = ent
        self.ref = [W.conv(net.netRefiner.netMain[i]) for i in range(0, 13, 2)]
        self._W, self._refiner, self._ref_center = W, net.netRefiner, {}

    def ref_center(self, i):
        """Refiner conv i reduced to its centre tap (a 1x1 conv), packed once."""
        if i not in self._ref_center:
            m = self._refiner.netMain[2 * i]
            self._ref_center[i] = self._W.conv(types.SimpleNamespace(
                weight=m.weight.detach()[:, :, 1:2, 1:2].contiguous(), bias=m.bias, stride=(1,), padding=(0,),
                dilation=(1,)))
        return self._ref_center[i]

    def build(self, plan, dtype, device, nF, Hp, Wp, P, first_map, second_map, rgb, flow_out, rgb_map=IDENTITY):
        """Emit: extractor over the nF frames rgb_map(0..nF-1) of `rgb` ([*,Hp,Wp,8]); decoders over P pairs
        whose first/second features are frames first_map(p) / second_map(p) of the extractor's outputs;
        refined flow (fp32, 2 ch) into `flow_out` ([P,Hp/4,Wp/4,2])."""
        lib = L.lib()
        # ---- feature pyramid (Extractor.forward, pwcnet.py:103-111), once per frame ----
        levels = {}
        if PWCPlanner.FUSED_EXTRACT and dtype != torch.float32 and lib.dbsr_pwc_extract_supported(Hp, Wp):
            # all six levels in one launch, activations in LDS (csrc/pwc_fused.hip)
            convs = (L.PwcExtConv * 18)()
            lv = (L.Tensor * 6)()
            hw, flop = (Hp, Wp), 0.0
            for k in range(6):
                C = PWC_LEVEL_CH[k + 1]
                oh, ow = self.ext[k][0].out_hw(*hw)
                levels[k + 1] = NHWC(nF, oh, ow, cpad(C), dtype, device)
                lv[k] = levels[k + 1].d(0)
                for j in range(3):
                    pc = self.ext[k][j]
                    convs[3 * k + j] = L.PwcExtConv(pc.w.data_ptr(), pc.bias.data_ptr(), pc.cin, pc.cout, pc.stride)
                    flop += 2.0 * nF * oh * ow * pc.cout * pc.cin * 9
                hw = (oh, ow)
            plan.keep.extend([convs, lv])
            plan.add('pwc.extract', lib.dbsr_pwc_extract, nF, Hp, Wp, rgb.d(0, rgb_map), convs, lv, work=('flop', flop))
            plan.kernel[len(plan.ops) - 1] = 'pwc_extract'
        else:
            x, hw = rgb, (Hp, Wp)
            for k in range(6):
                C = PWC_LEVEL_CH[k + 1]
                oh, ow = self.ext[k][0].out_hw(*hw)
                ta = NHWC(nF, oh, ow, cpad(C), dtype, device)
                tb = NHWC(nF, oh, ow, cpad(C), dtype, device)
                lv = NHWC(nF, oh, ow, cpad(C), dtype, device)
                plan.conv(f'pwc.ext{k + 1}.0', self.ext[k][0], nF, x, 0, hw, ta, 0, L.ACT_LRELU,
                          xmap=rgb_map if k == 0 else IDENTITY)
                plan.conv(f'pwc.ext{k + 1}.2', self.ext[k][1], nF, ta, 0, (oh, ow), tb, 0, L.ACT_LRELU)
                plan.conv(f'pwc.ext{k + 1}.4', self.ext[k][2], nF, tb, 0, (oh, ow), lv, 0, L.ACT_LRELU)
                levels[k + 1] = lv
                plan.keep.extend([ta, tb])      # every buffer a launch touches lives as long as the plan
                x, hw = lv, (oh, ow)
        plan.keep.append(levels)
        # ---- decoders, coarse to fine (pwcnet.py:225-229, Decoder.forward :153-184) ----
        prev = None
        for level in [6, 5, 4, 3, 2]:
            feat = levels[level]
            h, w, C = feat.h, feat.w, PWC_LEVEL_CH[level]
            base_real = 81 if level == 6 else 81 + C + 4
            ld = BASE_OFF + cpad(base_real)
            D = NHWC(P, h, w, ld, dtype, device)
            ent = self.dec[level]
            if PWCPlanner.FUSED_PREP and dtype != torch.float32 and lib.dbsr_pwc_level_prep_supported(h, w, C):
                # ConvT x2 + backwarp + correlation + assembly in one launch (csrc/pwc_fused.hip)
                if prev is None:
                    pargs = (L.NULL_TENSOR, 0, L.NULL_TENSOR, None, None, None, None)
                else:
                    pD, pflow, pbase = prev
                    wf, bf = ent['upflow']
                    bt = ent['upfeat'][1]
                    pargs = (pD.d(0), BASE_OFF + pbase, pflow.d(0), wf.data_ptr(), bf.data_ptr(),
                             ent['upfeat16'].data_ptr(), bt.data_ptr())
                plan.add(f'pwc.dec{level}.prep', lib.dbsr_pwc_level_prep, P, h, w, C, BACKWARP_SCALE.get(level, 1.0),
                         feat.d(0, first_map), feat.d(0, second_map), D.d(BASE_OFF), *pargs)
            else:
                if prev is None:
                    second = feat.d(0, second_map)
                else:
                    pD, pflow, pbase = prev
                    fu = NHWC(P, h, w, 8, torch.float32, device)     # upflow (2 ch; ld 8 for the 8-wide ConvT reads)
                    fe = NHWC(P, h, w, 2, torch.float32, device)     # upfeat
                    wt, bs = ent['upflow']
                    plan.add(f'pwc.dec{level}.upflow', lib.dbsr_conv_transpose_k4s2, P, pD.h, pD.w, 2, 2, pflow.d(0),
                             wt.data_ptr(), bs.data_ptr(), fu.d(0))
                    wt, bs = ent['upfeat']
                    plan.add(f'pwc.dec{level}.upfeat', lib.dbsr_conv_transpose_k4s2, P, pD.h, pD.w, BASE_OFF + pbase,
                             2, pD.d(0), wt.data_ptr(), bs.data_ptr(), fe.d(0))
                    ws = NHWC(P, h, w, cpad(C), dtype, device)
                    plan.add(f'pwc.dec{level}.backwarp', lib.dbsr_backwarp, P, h, w, C, feat.d(0, second_map), fu.d(0),
                             BACKWARP_SCALE[level], ws.d(0))
                    plan.add(f'pwc.dec{level}.assemble', lib.dbsr_pwc_assemble, P, h, w, C, feat.d(0, first_map),
                             fu.d(0), fe.d(0), D.d(BASE_OFF))
                    second = ws.d(0)
                    plan.keep.extend([fu, fe, ws])
                plan.add(f'pwc.dec{level}.corr', lib.dbsr_correlation, P, h, w, C, feat.d(0, first_map), second,
                         D.d(BASE_OFF), 1)
            fl = NHWC(P, h, w, 8, torch.float32, device)    # 2 ch (ld 8: read by the next level's ConvT)
            if PWCPlanner.FUSED_DENSE and dtype != torch.float32 and lib.dbsr_pwc_dense_supported(h, w, ld):
                # coarse level: the DenseNet + flow conv in one launch with D in LDS (csrc/pwc_dense.hip)
                convs = (L.PwcDenseConv * 6)()
                cin, flop = base_real, 0.0
                for i, pc in enumerate(ent['dense'] + [ent['flow']]):
                    start = 0 if i == 5 else (BASE_OFF if i == 0 else DENSE_OFF[i - 1])
                    cg = cpad(pc.cin) // 8
                    convs[i] = L.PwcDenseConv(pc.w.data_ptr(), pc.bias.data_ptr() if pc.bias is not None else None,
                                              9 * cg * 8, cg, start, pc.cout, DENSE_OFF[i] if i < 5 else 0)
                    flop += 2.0 * P * h * w * pc.cout * pc.cin * 9
                plan.keep.append(convs)
                plan.add(f'pwc.dec{level}.dense', lib.dbsr_pwc_dense, P, h, w, D.d(0), BASE_OFF, convs, fl.d(0),
                         work=('flop', flop))
                plan.kernel[len(plan.ops) - 1] = 'pwc_dense'
                cin = base_real + sum(DENSE_OUT)
            else:
                cin = base_real
                for i, (pc, off) in enumerate(zip(ent['dense'], DENSE_OFF)):
                    start = BASE_OFF if i == 0 else DENSE_OFF[i - 1]
                    plan.conv(f'pwc.dec{level}.dense{i}', pc, P, D, start, (h, w), D, off, L.ACT_LRELU, cin=cin)
                    cin += DENSE_OUT[i]
                plan.conv(f'pwc.dec{level}.flow', ent['flow'], P, D, 0, (h, w), None, 0, L.ACT_NONE, cin=cin,
                          y_desc=fl.d(0))
            plan.keep.extend([D, fl])
            prev = (D, fl, base_real)
        # ---- refiner (pwcnet.py:186-207) + residual flow (:231) ----
        D2, fl2, base2 = prev
        h, w = D2.h, D2.w
        chans = [128, 128, 128, 96, 64, 32]
        bufs = [NHWC(P, h, w, cpad(c), dtype, device) for c in chans]
        x, xc0, cin = D2, 0, BASE_OFF + base2
        for i in range(6):
            pc = self.ref[i]
            if pc.dil >= h and pc.dil >= w and pc.kh == 3:
                # dilation >= the level size (refiner 4, d 16, on the 16x16 level of a 64x64 frame): every
                # off-centre tap reads zero padding, so the conv is exactly its centre tap as a 1x1 conv
                pc = self.ref_center(i)
            plan.conv(f'pwc.refiner{i}', pc, P, x, xc0, (h, w), bufs[i], 0, L.ACT_LRELU, cin=cin)
            x, xc0, cin = bufs[i], 0, chans[i]
        plan.conv('pwc.refiner6', self.ref[6], P, x, 0, (h, w), None, 0, L.ACT_NONE, y_desc=flow_out.d(0),
                  res=fl2)
        plan.keep.extend(bufs)


# ==================================================================================================
# DBSR engine
# ==================================================================================================
class DBSREngine:
    LANE0_CU_SHARE = 0.5      # CU share of lane 0's persistent convs while the PWC lane runs (tools/capbench.sh)
    # the first LANE0_EARLY_CONVS encoder convs (enc.init, enc.res0.conv1, ...) at CU share LANE0_EARLY_SHARE instead:
    # PWC-Net's coarse levels (1x1 .. 8x8 pixels per pair) leave most of the chip idle while they run
    LANE0_EARLY_CONVS = 0
    LANE0_EARLY_SHARE = 0.5
    # bf16: fuse the RGB predictor into the last decoder ResBlock conv (False: separate fp32 kernel)
    FUSED_HEAD = True
    # PixelShuffle upsampler conv + shuffle + blur in one kernel (dbsr_conv_shuffle_blur)
    FUSED_UPSAMPLE_BLUR = True
    # ResBlocks as one kernel each where the library serves them (dbsr_resblock: the decoder's 32-channel post blocks;
    # the encoder's, the offset-feature extractor's and the decoder's 64-channel pre blocks)
    FUSED_RESBLOCK = True
    FUSED_RESBLOCK64 = True   # (A/B switch for the 64-channel kernel alone)
    # the warp of the other frames + their feature projection in one launch (dbsr_warp_project; 16-bit, 512 channels,
    # with the linearity split, whose projections go straight into the weight-predictor input).  Off: measured slower
    # than the two launches it replaces at the bench shape (230 vs 186 us, tools/bench_wp.py)
    FUSED_WARP_PROJ = False
    # weight-predictor input conv split into a per-frame [proj, offfeat] conv + a per-burst base conv
    LINEAR_SPLIT = True
    # weight-predictor output conv + softmax + fusion in one kernel (dbsr_conv_fuse_softmax: the fp32 logits never
    # reach memory; softmax=False: dbsr_conv_fuse_relu_norm) wherever the library serves the shape
    # (16-bit, N = 14, cout % 128 == 0); otherwise dbsr_conv2d into a logits buffer + dbsr_fuse_softmax / _relu_norm
    FUSED_WP_OUT = True
    # 16-bit weight rounding of the DBSR convs: 'diffuse' (dbsr_weights_round_diffuse: each output channel's rounding
    # errors carried along its K, their sum within half an ulp) or 'nearest'.  At configs[1] the fp16 prediction's
    # RMS error against the fp32 oracle: nearest 4.5e-4, diffuse 3.2e-4 (tools/precision_attrib.py)
    WEIGHT_ROUNDING = 'diffuse'

    def __init__(self, net):
        self.net = net
        self.dtype = net.compute_dtype
        self.zero_flow = bool(getattr(net, 'zero_flow', False))   # part of every plan (no PWC-Net ops)
        self.device = None
        self.sig = None
        self.plans = {}
        self.slots = {}
        self.graphs = {}
        self.weights_stale = False

    def matches(self, net):
        return (net is self.net and self.dtype == net.compute_dtype and self.sig == _param_signature(net)
                and self.zero_flow == bool(getattr(net, 'zero_flow', False)))

    def _pack(self, device):
        net = self.net
        stream = L.stream_ptr(device)
        # the DBSR convs' 16-bit weights by error-diffusion rounding (DBSREngine.WEIGHT_ROUNDING); PWC-Net's by
        # round-to-nearest (diffusing them moved the fp16 prediction's error by nothing and the offsets' max error up)
        W = _Weights(self.dtype, device, stream, rounding=DBSREngine.WEIGHT_ROUNDING)
        enc, mer, dec = net.encoder, net.merging, net.decoder
        self.pwc = PWCPlanner(enc.alignment_net, _Weights(self.dtype, device, stream))
        self.enc_init = W.conv(enc.init_layer[0])
        self.enc_res = [(W.conv(b.conv1[0]), W.conv(b.conv2[0])) for b in enc.res_layers]
        self.enc_out = W.conv(enc.out_layer[0])
        self.proj = W.conv(mer.feat_project_layer[0])
        ofe = list(mer.offset_feat_extractor)
        self.ofe_init = W.conv(ofe[0][0])
        self.ofe_res = [(W.conv(b.conv1[0]), W.conv(b.conv2[0])) for b in ofe[1:]]
        wp = list(mer.weight_predictor)
        self.wp_init = W.conv(wp[0][0])
        # linearity split of the first weight-predictor conv (merging.py:87-113): its input is
        # [base, proj_f - base, offfeat_f] with base = proj of the burst's reference frame (use_base_frame) or the
        # burst mean of the projections, so
        # conv(W)(input) = conv([W_diff | W_off])([proj_f, offfeat_f]) + conv(W_base - W_diff)(base): the second
        # term is one conv per burst instead of per frame, and the merge-prep copy of base / diff disappears
        # constructor variants (merging.py:79-121): use_base_frame=False takes the burst mean of the projections as
        # the base (dbsr_burst_mean, then the base conv: the split's algebra holds for any base); softmax=False
        # normalises relu(logits) over the burst (dbsr_fuse_relu_norm); offset_modulo goes to flow_finalize
        self.softmax, self.ref_base, self.offset_modulo = merging_variant(mer)
        pd = mer.feat_project_layer[0].out_channels
        self.wp_split = None
        if DBSREngine.LINEAR_SPLIT and pd % 32 == 0:
            c0 = wp[0][0]
            geo = types.SimpleNamespace(stride=(1,), padding=c0.padding, dilation=c0.dilation)
            rest = lambda: (c0.weight.detach().float()[:, pd:], c0.bias)                               # noqa: E731
            base = lambda: (c0.weight.detach().float()[:, :pd] - c0.weight.detach().float()[:, pd:2 * pd], None)  # noqa: E731
            self.wp_split = (W.conv(geo, recipe=rest), W.conv(geo, recipe=base))
        elif not self.ref_base:
            raise NotImplementedError('use_base_frame=False runs on the linearity split: needs project_dim % 32 == 0 '
                                      '(and DBSREngine.LINEAR_SPLIT)')
        self.wp_res = [(W.conv(b.conv1[0]), W.conv(b.conv2[0])) for b in wp[1:-1]]
        self.wp_out = W.conv(wp[-1][0])
        self.dec_init = W.conv(dec.init_layer[0])
        self.dec_pre = [(W.conv(b.conv1[0]), W.conv(b.conv2[0])) for b in dec.pre_res_layers]
        up = dec.upsample_layer
        self.s = up.upsample_factor
        self.dec_up = W.conv(up.conv_layer[0], shuffle=self.s)
        self.blur = gauss_kernel3(up.gauss_blur_sd, up.gauss_ksz) if up.gauss_blur_sd is not None else None
        if self.blur is not None and up.gauss_ksz != 3:
            raise NotImplementedError('gauss_ksz != 3')
        self.dec_post = [(W.conv(b.conv1[0]), W.conv(b.conv2[0])) for b in dec.post_res_layers]
        # the RGB predictor runs fp32 math on bf16 features (0.2 GFLOP/burst; removes ~40 % of the bf16
        # PSNR delta, tools/bf16_sensitivity.py)
        self.pred = PackedConv(dec.predictor[0], torch.float32, device, stream)
        pm = dec.predictor[0]
        self.head_w = pm.weight.detach().to(device=device, dtype=torch.float32).reshape(pm.out_channels, -1).contiguous()
        self.head_b = (pm.bias.detach().to(device=device, dtype=torch.float32).contiguous()
                       if pm.bias is not None else None)
        self.device = device
        self.sig = _param_signature(net)
        self.plans, self.slots, self.graphs = {}, {}, {}
        self.weights_stale = False

    def refresh_weights(self):
        """Re-pack the DBSR (non-PWC) weights in place after an optimizer updated the parameters through their
        storage (DBSRTrainer.step's Adam kernel: no version bump, no new storage): plans and captured graphs
        keep pointing at the same packed buffers.  PWC-Net is frozen in training (encoders.py:56-61)."""
        stream = L.stream_ptr(self.device)
        convs = [self.enc_init, self.enc_out, self.proj, self.ofe_init, self.wp_init, self.wp_out, self.dec_init,
                 self.dec_up, self.pred]
        for lst in (self.enc_res, self.ofe_res, self.wp_res, self.dec_pre, self.dec_post):
            for c1, c2 in lst:
                convs += [c1, c2]
        if self.wp_split is not None:
            convs += list(self.wp_split)
        for pc in convs:
            pc.repack(stream)
        pm = self.net.decoder.predictor[0]
        self.head_w.copy_(pm.weight.detach().reshape(pm.out_channels, -1))
        if self.head_b is not None:
            self.head_b.copy_(pm.bias.detach())
        self.weights_stale = False

    def _resblocks(self, plan, name, blocks, n, hw, bufs, x_idx, dtype, head=None):
        """ResBlock chain (blocks.py:81-96) over ping-pong buffers; returns index of the result buffer
        (and, with `head`, whether the head got fused into the last conv -- see Plan.conv)."""
        a = x_idx
        fused = False
        for i, (c1, c2) in enumerate(blocks):
            b, c = [j for j in range(3) if j != a]
            hd = head if head is not None and i == len(blocks) - 1 else None
            if DBSREngine.FUSED_RESBLOCK and \
                    plan.resblock(f'{name}{i}', c1, c2, n, bufs[a], bufs[b], bufs[c], hw, head=hd):
                fused = hd is not None
                a = c
                continue
            plan.conv(f'{name}{i}.conv1', c1, n, bufs[a], 0, hw, bufs[b], 0, L.ACT_RELU)
            d = plan.conv(f'{name}{i}.conv2', c2, n, bufs[b], 0, hw, bufs[c], 0, L.ACT_NONE, res=bufs[a],
                          post_act=L.ACT_RELU, head=head if i == len(blocks) - 1 else None)
            fused = d.fused_head
            a = c
        return (a, fused) if head is not None else a

    def _emit_flow(self, plan, grp, N, H, W, sh):
        """PWC-Net flow of the group's pairs -> offsets and the offset-feature input (flow_finalize); returns
        the group's (still empty) weight-predictor input buffer WP."""
        dt, dev = self.dtype, self.device
        lib = L.lib()
        g0, g1 = grp
        Bg, Fg, Pg = g1 - g0, (g1 - g0) * N, (g1 - g0) * (N - 1)
        off_f, off_p = g0 * N, g0 * (N - 1)
        Hp, Wp = sh['Hp'], sh['Wp']
        hw = (H, W)
        fmap = (1, 1, off_f, 0)                       # frame f of the group -> frame off_f + f of the batch
        if not self.zero_flow:
            flow_out = NHWC(Pg, Hp // 4, Wp // 4, 2, torch.float32, dev)
            self.pwc.build(plan, dt, dev, Fg, Hp, Wp, Pg, first_map=(N - 1, N, 0, 0), second_map=(N - 1, N, 1, 1),
                           rgb=sh['rgb'], flow_out=flow_out, rgb_map=fmap)
            plan.add('flow_finalize', lib.dbsr_flow_finalize, Bg, N, Hp // 4, Wp // 4, flow_out.d(0), H, W, Hp, Wp,
                     sh['offsets'][off_p:].data_ptr(), self.offset_modulo, sh['om'].d(0, fmap))
            plan.keep.append(flow_out)
        # (zero flow: offsets and om stay zero from initialisation)
        pd, od = self.proj.cout, self.ofe_init.cout
        # weight-predictor input: [base, diff, offfeat] (merging.py:110), or [proj, offfeat] with the split
        oc = pd if self.wp_split is not None else 2 * pd
        WP = NHWC(Fg, H, W, oc + od, dt, dev)
        plan.keep.append(WP)
        return WP

    def _emit_ofe(self, plan, grp, N, H, W, sh, WP):
        """Offset-feature extractor (merging.py:85-87) of the group -> WP[..., oc:]."""
        dt, dev = self.dtype, self.device
        g0, g1 = grp
        Fg = (g1 - g0) * N
        fmap = (1, 1, g0 * N, 0)
        hw = (H, W)
        pd, od = self.proj.cout, self.ofe_init.cout
        oc = pd if self.wp_split is not None else 2 * pd
        o = [NHWC(Fg, H, W, od, dt, dev) for _ in range(3)]
        plan.conv('merge.ofe.init', self.ofe_init, Fg, sh['om'], 0, hw, o[0], 0, L.ACT_RELU, xmap=fmap)
        a = 0
        if not self.ofe_res:
            raise NotImplementedError('num_offset_feat_extractor_res must be >= 1')
        for k, (c1, c2) in enumerate(self.ofe_res):
            b, c = [j for j in range(3) if j != a]
            last = k == len(self.ofe_res) - 1
            if DBSREngine.FUSED_RESBLOCK and plan.resblock(f'merge.ofe.res{k}', c1, c2, Fg, o[a], o[b],
                                                           WP if last else o[c], hw, yc0=oc if last else 0):
                a = c
                continue
            plan.conv(f'merge.ofe.res{k}.conv1', c1, Fg, o[a], 0, hw, o[b], 0, L.ACT_RELU)
            if last:
                plan.conv(f'merge.ofe.res{k}.conv2', c2, Fg, o[b], 0, hw, WP, oc, L.ACT_NONE, res=o[a],
                          post_act=L.ACT_RELU)
            else:
                plan.conv(f'merge.ofe.res{k}.conv2', c2, Fg, o[b], 0, hw, o[c], 0, L.ACT_NONE, res=o[a],
                          post_act=L.ACT_RELU)
                a = c
        plan.keep.append(o)

    def _emit_base(self, plan, grp, N, H, W, sh, WP):
        """Linearity split: the reference frames' projection into WP[..., :pd] and the per-burst base conv
        (merging.py:77-89).  Needs only the encoder, so the first group's runs on lane 0 beside the
        alignment chain; returns the base-term buffer BS (None with use_base_frame=False: the mean base needs
        every frame's projection, _emit_mean_base)."""
        g0, g1 = grp
        Bg = g1 - g0
        rest, basec = self.wp_split
        plan.conv('merge.proj_ref', self.proj, Bg, sh['E'], 0, (H, W), WP, 0, L.ACT_RELU, xmap=(1, N, g0 * N, 1),
                  ymap=(1, N, 0, 1))
        if not self.ref_base:
            return None
        BS = NHWC(Bg, H, W, r8(basec.cout), self.dtype, self.device)
        plan.conv('merge.wp.base', basec, Bg, WP, 0, (H, W), BS, 0, L.ACT_NONE, xmap=(1, N, 0, 1))
        plan.keep.append(BS)
        return BS

    def _emit_mean_base(self, plan, grp, N, H, W, WP):
        """use_base_frame=False (merging.py:81-82): the burst mean of all frames' projections WP[..., :pd]
        (dbsr_burst_mean, fp32 sum) -> MB, then the per-burst base conv on it -> BS."""
        g0, g1 = grp
        Bg = g1 - g0
        basec = self.wp_split[1]
        pd = self.proj.cout
        MB = NHWC(Bg, H, W, cpad(pd), self.dtype, self.device)
        plan.add('merge.base_mean', L.lib().dbsr_burst_mean, Bg, N, H * W, pd, WP.d(0), MB.d(0),
                 work=('byte', (N + 1.0) * Bg * H * W * pd * (4 if self.dtype == torch.float32 else 2)))
        BS = NHWC(Bg, H, W, r8(basec.cout), self.dtype, self.device)
        plan.conv('merge.wp.base', basec, Bg, MB, 0, (H, W), BS, 0, L.ACT_NONE)
        plan.keep.extend([MB, BS])
        return BS

    def _emit_warp(self, plan, grp, N, H, W, sh, WP):
        """Warp of the group's other frames (encoders.py:80) and, with the linearity split, their projection
        straight into WP[..., :pd] (merging.py:77): needs the offsets, not the offset features."""
        dt, dev = self.dtype, self.device
        g0, g1 = grp
        Pg = (g1 - g0) * (N - 1)
        off_f, off_p = g0 * N, g0 * (N - 1)
        C, E = self.enc_out.cout, sh['E']
        Wf = NHWC(max(Pg, 1), H, W, C, dt, dev)
        es = 4 if dt == torch.float32 else 2
        if Pg > 0:
            pd = self.proj.cout
            fused = (self.wp_split is not None and DBSREngine.FUSED_WARP_PROJ and dt != torch.float32 and C == 512
                     and pd % 16 == 0 and pd <= 64 and self.proj.kh == 1 and self.proj.cin == C)
            if fused:
                # warp + the projection of the warped frames in one launch (the 512-channel warped frames are not
                # read back from HBM); the op stays in the warp family, its bytes + the projection's output
                plan.add('warp+proj', L.lib().dbsr_warp_project, Pg, H, W, C, E.d(0, (N - 1, N, 1 + off_f, 1)),
                         sh['offsets'][off_p:].data_ptr(), 2 * H * W, Wf.d(0), self.proj.w.data_ptr(),
                         self.proj.bias.data_ptr() if self.proj.bias is not None else None, pd,
                         WP.d(0, (N - 1, N, 1, 1)),
                         work=('byte', 2.0 * Pg * C * H * W * es + 8.0 * Pg * H * W + 1.0 * Pg * pd * H * W * es))
                plan.kernel[len(plan.ops) - 1] = 'warp'
            else:
                plan.add('warp', L.lib().dbsr_warp_bilinear, Pg, H, W, C, E.d(0, (N - 1, N, 1 + off_f, 1)),
                         sh['offsets'][off_p:].data_ptr(), 2 * H * W, Wf.d(0),
                         work=('byte', 2.0 * Pg * C * H * W * es + 8.0 * Pg * H * W))
                if self.wp_split is not None:
                    plan.conv('merge.proj_oth', self.proj, Pg, Wf, 0, (H, W), WP, 0, L.ACT_RELU,
                              ymap=(N - 1, N, 1, 1))
        plan.keep.append(Wf)
        return Wf

    def _emit_merge(self, plan, grp, N, H, W, sh, WP, BS=None, Wf=None):
        """Warp (encoders.py:80) + projections, weight predictor (merging.py:61-113) of the group; returns
        the weight predictor's last hidden buffer and the warped embeddings Wf.  BS / Wf: the group's base
        term / warped frames (with their projections) if _emit_base / _emit_warp already ran (with the split,
        _emit_base always has: BS None then means the mean base, computed here)."""
        dt, dev = self.dtype, self.device
        lib = L.lib()
        g0, g1 = grp
        Bg, Fg, Pg = g1 - g0, (g1 - g0) * N, (g1 - g0) * (N - 1)
        off_f = g0 * N
        PJ = sh['PJ']
        hw = (H, W)
        pd = self.proj.cout
        if Wf is None:
            Wf = self._emit_warp(plan, grp, N, H, W, sh, WP)
        q = [NHWC(Fg, H, W, self.wp_init.cout, dt, dev) for _ in range(3)]
        if self.wp_split is not None:
            # the base term once per burst, added (broadcast over the burst's frames) as the residual of the
            # per-frame [proj, offfeat] conv before its ReLU
            rest = self.wp_split[0]
            if BS is None:            # (use_base_frame=False: every frame's projection is in WP by now)
                BS = self._emit_mean_base(plan, grp, N, H, W, WP)
            plan.conv('merge.wp.init', rest, Fg, WP, 0, hw, q[0], 0, L.ACT_NONE, res=BS, rmap=(N, 1, 0, 0),
                      post_act=L.ACT_RELU)
        else:
            if Pg > 0:
                plan.conv('merge.proj_oth', self.proj, Pg, Wf, 0, hw, PJ, 0, L.ACT_RELU,
                          ymap=(N - 1, N, 1 + off_f, 1))
            plan.add('merge.prep', lib.dbsr_merge_prep, Bg, N, H * W, pd, PJ.d(0, (1, 1, off_f, 0)), WP.d(0))
            plan.conv('merge.wp.init', self.wp_init, Fg, WP, 0, hw, q[0], 0, L.ACT_RELU)
        i = self._resblocks(plan, 'merge.wp.res', self.wp_res, Fg, hw, q, 0, dt)
        plan.keep.append(q)
        return q[i], Wf

    def _emit_logits(self, plan, Fg, H, W, h):
        """The weight predictor's last conv (merging.py:55-57) into a logits buffer LG [Fg,H,W,C]."""
        LG = NHWC(Fg, H, W, self.enc_out.cout, self.dtype, self.device)
        plan.conv('merge.wp.out', self.wp_out, Fg, h, 0, (H, W), LG, 0, L.ACT_NONE)
        plan.keep.append(LG)
        return LG

    def _build(self, B, N, H, W, mode='full', first_frame=0):
        """mode 'full': the whole forward.  mode 'partial' (frame-sharded fusion): stop after
        the weight predictor and emit dbsr_fuse_partial statistics of frames [first_frame, N) into
        bufs['stats'] instead of the fusion and the decoder (those run in `_build_combine`).

        Lanes: PWC-Net and the flow finalize run on side lane 1 while lane 0 runs the encoder, the reference
        frames' projections and the base term; after the flow join, the offset-feature extractor runs on lane 1
        beside the warp and the other frames' projections on lane 0; then merge + fusion + decoder on lane 0.
        Single-stream mode issues the same launches in the same order on one stream."""
        dt, dev = self.dtype, self.device
        lib = L.lib()
        plan = Plan()
        F, P = B * N, B * (N - 1)
        C = self.enc_out.cout
        hw = (H, W)
        bufs = {}
        bufs['burst'] = torch.zeros(B, N, 4, H, W, dtype=torch.float32, device=dev)
        raw = NHWC(F, H, W, 8, dt, dev)
        Hp, Wp = int(math.ceil(H / 64.0) * 64), int(math.ceil(W / 64.0) * 64)
        rgb = NHWC(F, Hp, Wp, 8, dt, dev)
        bufs['offsets'] = torch.zeros(P, 2, H, W, dtype=torch.float32, device=dev)
        om = NHWC(F, H, W, 8, dt, dev)
        E = NHWC(F, H, W, C, dt, dev)
        PJ = NHWC(F, H, W, r8(self.proj.cout), dt, dev) if self.wp_split is None else None
        sh = {'rgb': rgb, 'offsets': bufs['offsets'], 'om': om, 'E': E, 'PJ': PJ, 'Hp': Hp, 'Wp': Wp}
        grp = (0, B)
        plan.add('pack_burst', lib.dbsr_pack_burst, B, N, H, W, bufs['burst'].data_ptr(), raw.d(0), Hp, Wp,
                 rgb.d(0) if not self.zero_flow else L.NULL_TENSOR)
        # lane-0 persistent convs issued while the side lane runs leave part of the CUs to it
        plan_cap = int(torch.cuda.get_device_properties(dev).multi_processor_count * DBSREngine.LANE0_CU_SHARE) \
            if Plan.MULTI_STREAM else 0
        plan.fork(1, dev, priority=0)
        WP = self._emit_flow(plan, grp, N, H, W, sh)          # PWC-Net on lane 1
        plan.switch(0)
        plan.max_blocks = plan.max_blocks_cap = plan_cap
        if plan_cap and DBSREngine.LANE0_EARLY_CONVS:
            names = ['enc.init'] + [f'enc.res{i}.conv{j}' for i in range(len(self.enc_res)) for j in (1, 2)]
            plan.early_names = set(names[:DBSREngine.LANE0_EARLY_CONVS])
            plan.early_cap = int(torch.cuda.get_device_properties(dev).multi_processor_count *
                                 DBSREngine.LANE0_EARLY_SHARE)
        # ---------------- encoder (encoders.py:66-72), whole batch ----------------
        e = [NHWC(F, H, W, r8(self.enc_init.cout), dt, dev) for _ in range(3)]
        plan.conv('enc.init', self.enc_init, F, raw, 0, hw, e[0], 0, L.ACT_RELU)
        i = self._resblocks(plan, 'enc.res', self.enc_res, F, hw, e, 0, dt)
        plan.conv('enc.out', self.enc_out, F, e[i], 0, hw, E, 0, L.ACT_RELU)
        if self.wp_split is None:
            plan.conv('merge.proj_ref', self.proj, B, E, 0, hw, PJ, 0, L.ACT_RELU, xmap=(1, N, 0, 1),
                      ymap=(1, N, 0, 1))
        plan.keep.extend([raw, rgb, om, e, E, PJ])
        FW = NHWC(F, H, W, C, dt, dev) if mode == 'full' else None
        if mode == 'full':
            bufs['pred'] = torch.zeros(B, 3, H * self.s, W * self.s, dtype=torch.float32, device=dev)
        plan.fuse_ops = []
        es = 4 if dt == torch.float32 else 2
        # the base term needs only the encoder: lane 0 computes it before waiting for PWC-Net (its projections
        # write WP channels [0, pd); the side lane writes the offset features at [pd, ..))
        BS = self._emit_base(plan, grp, N, H, W, sh, WP) if self.wp_split is not None else None
        plan.join(1)                      # lane 0 waits for the flow
        plan.max_blocks = 0
        plan.switch(1)                    # offsets are in: offset features on lane 1 ...
        self._emit_ofe(plan, grp, N, H, W, sh, WP)
        plan.switch(0)
        Wf = self._emit_warp(plan, grp, N, H, W, sh, WP)      # ... beside the warp + projections
        plan.join(1)
        h, Wf = self._emit_merge(plan, grp, N, H, W, sh, WP, BS=BS, Wf=Wf)
        if mode == 'partial':
            # (softmax=False and use_base_frame=False are refused by forward_partial: their statistics do not
            # combine across frame shards with dbsr_fuse_combine's log-sum-exp)
            LG = self._emit_logits(plan, B * N, H, W, h)
            ST = torch.zeros(B, H, W, 3 * C, dtype=torch.float32, device=dev)
            plan.add('merge.fuse_partial', lib.dbsr_fuse_partial, B, N, H * W, C, first_frame, LG.d(0),
                     E.d(0, (1, N, 0, 1)), Wf.d(0), ST.data_ptr())
            bufs['stats'] = ST
        else:
            FUS = NHWC(B, H, W, C, dt, dev)
            feats = [E.d(0, (1, N, 0, 1)), Wf.d(0), FUS.d(0), FW.d(0)]
            idx = plan.conv_fuse('merge.wp.out+fuse', self.wp_out, B, N, h, hw, *feats, softmax=self.softmax) \
                if DBSREngine.FUSED_WP_OUT else None
            if idx is not None:
                plan.fuse_ops.append((idx, plan.ops[idx][1], FW.d(0), None))
            else:
                LG = self._emit_logits(plan, B * N, H, W, h)
                args = [B, N, H * W, C, LG.d(0)] + feats
                if self.softmax:
                    plan.add('merge.fuse', lib.dbsr_fuse_softmax, *args)
                else:   # merging.py:119-121
                    plan.add('merge.fuse_relu_norm', lib.dbsr_fuse_relu_norm, *args)
                plan.fuse_ops.append((len(plan.ops) - 1, args, FW.d(0),
                                      ((2.0 * N + 1) * B * C * H * W * es, 1.0 * N * B * C * H * W * es)))
            self._decoder(plan, B, H, W, FUS, bufs, pred_out=bufs['pred'])
            plan.keep.append(FUS)
        plan.max_blocks = 0
        plan.keep.append(FW)
        plan.finalize_workspace(dev)
        plan.bufs = bufs
        plan.FW = FW
        plan.shape = (B, N, H, W)
        return plan

    def _decoder(self, plan, B, H, W, FUS, bufs, pred_out=None):
        """ResPixShuffleConv (decoders.py:54-62) on the fused embedding FUS [B,H,W,C] -> pred_out (a [B,3,sH,sW]
        fp32 view; default: a new bufs['pred'])."""
        dt, dev = self.dtype, self.device
        lib = L.lib()
        hw = (H, W)
        S = self.s
        gd = self.dec_init.cout
        g = [NHWC(B, H, W, gd, dt, dev) for _ in range(3)]
        plan.conv('dec.init', self.dec_init, B, FUS, 0, hw, g[0], 0, L.ACT_RELU)
        i = self._resblocks(plan, 'dec.pre', self.dec_pre, B, hw, g, 0, dt)
        pc = self.dec_up.cout // (S * S)
        sh = [NHWC(B, H * S, W * S, pc, dt, dev) for _ in range(3)]
        a = 0
        # conv + PixelShuffle + blur in one kernel where the library serves the shape (the pre-blur tensor, 75.5 MB
        # at the bench shape, then never round-trips through HBM; bitwise equal to the two launches)
        if self.blur is not None and DBSREngine.FUSED_UPSAMPLE_BLUR and \
                plan.conv_shuffle_blur('dec.upsample+blur', self.dec_up, B, g[i], hw, sh[1], L.ACT_RELU,
                                       self.blur) is not None:
            a = 1
        else:
            plan.conv('dec.upsample', self.dec_up, B, g[i], 0, hw, sh[0], 0, L.ACT_RELU, out_mode=L.OUT_SHUFFLE,
                      shuffle=S)
            if self.blur is not None:
                kbuf = (ctypes.c_float * 9)(*self.blur)
                plan.keep.append(kbuf)
                plan.add('dec.blur', lib.dbsr_gauss_blur3, B, H * S, W * S, pc, sh[0].d(0), kbuf, sh[1].d(0))
                a = 1
        if pred_out is None:
            pred_out = bufs['pred'] = torch.zeros(B, 3, H * S, W * S, dtype=torch.float32, device=dev)
        pdesc = L.tensor_desc(pred_out, 1, 0, img_stride=3 * H * S * W * S, dtype=torch.float32)
        # 16-bit (fp16 / bf16): the last post ResBlock and the RGB predictor in one kernel -- dbsr_resblock_head where
        # the fused ResBlock serves the shape, else the pipelined conv2's epilogue 4 (dbsr_conv2d_head); the block's
        # 32-channel output never reaches HBM and the head runs fp32 on its unrounded value (decoders.py:59-61)
        head = None
        if dt != torch.float32 and self.dec_post and DBSREngine.FUSED_HEAD:
            head = ('predictor', self.head_w, self.head_b, pdesc)
        if head is not None:
            i, fused = self._resblocks(plan, 'dec.post', self.dec_post, B, (H * S, W * S), sh, a, dt, head=head)
        else:
            i, fused = self._resblocks(plan, 'dec.post', self.dec_post, B, (H * S, W * S), sh, a, dt), False
        if not fused:
            plan.conv('dec.predictor', self.pred, B, sh[i], 0, (H * S, W * S), None, 0, L.ACT_RELU,
                      out_mode=L.OUT_NCHW_F32, y_desc=pdesc, precise=(dt != torch.float32))
        plan.keep.extend([g, sh])

    @staticmethod
    def _capture(plan, dev):
        """One HIP graph of the whole plan (side lanes become parallel branches of the graph).

        The side lane's stream has normal priority.  With a high-priority side stream (round 2), engines built
        later in the same process replayed their graph at ~1,750 instead of ~2,930 bursts/s, run after run;
        at priority 0 six engines in a row all ran at 2,919-2,935.  Per-lane graphs replayed on the plan's
        own streams were stable as well but ~2.5 % slower (tools/lane_ab.py)."""
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            plan.run(L.stream_ptr(dev))
        return g

    def _set_fw(self, plan, want):
        for idx, args, fw_desc, nbytes in plan.fuse_ops:
            fn, _, name, lane = plan.ops[idx]
            a = list(args)
            a[-1] = fw_desc if want else L.NULL_TENSOR
            plan.ops[idx] = (fn, tuple(a), name, lane)
            if nbytes is not None:            # (the fused conv's work stays its FLOPs)
                plan.work[idx] = ('byte', nbytes[0] + (nbytes[1] if want else 0.0))

    # Output slots per shape.  Slots 0..OUTPUT_SLOTS-2 hand out views of their static output buffers (pred,
    # offsets, fusion weights; no copy inside the timed step) and are reused only once no tensor from their
    # previous forward is referenced anywhere (storage use counts); the last slot is clone-only, for when
    # the caller still holds every zero-copy slot's outputs.  Each slot is its own plan (and HIP graph).
    OUTPUT_SLOTS = 3

    @staticmethod
    def _uses(t):
        return torch._C._storage_Use_Count(t.untyped_storage()._cdata)

    def _outputs(self, plan):
        return [plan.bufs['pred'], plan.bufs['offsets']] + ([plan.FW.t] if plan.FW is not None else [])

    def _slot_free(self, plan):
        return all(self._uses(t) <= b for t, b in zip(self._outputs(plan), plan.out_base))

    def _new_slot(self, key):
        plan = self._build(*key)
        plan.out_base = [self._uses(t) for t in self._outputs(plan)]
        self.slots.setdefault(key, []).append(plan)
        if len(self.slots[key]) == 1:
            self.plans[key] = plan            # slot 0 is the shape's reference plan (bench.py, tests)
        return plan

    def forward(self, burst):
        if not burst.is_cuda:
            raise RuntimeError('DBSRNet (MI355X engine) needs the burst on a HIP device; got %s' % burst.device)
        if burst.dim() != 5 or burst.shape[2] != 4:
            raise ValueError('burst must be [B,N,4,H,W]')
        B, N, _, H, W = burst.shape
        if N < 2:
            raise ValueError('burst needs at least 2 frames')
        dev = burst.device
        if self.device != dev or self.sig != _param_signature(self.net):
            self._pack(dev)
        elif self.weights_stale:
            self.refresh_weights()
        key = (B, N, H, W)
        if key not in self.slots:
            self._new_slot(key)
        slots = self.slots[key]
        nzc = DBSREngine.OUTPUT_SLOTS - 1               # zero-copy slots
        if getattr(self.net, 'graph_zero_copy', False):
            si = 0                                      # opt-in: always slot 0, overwritten by the next forward
        else:
            si = next((i for i, p in enumerate(slots[:nzc]) if self._slot_free(p)), None)
            if si is None and len(slots) < nzc:
                self._new_slot(key)
                si = len(slots) - 1
        copy = si is None
        if copy:
            while len(slots) < DBSREngine.OUTPUT_SLOTS:
                self._new_slot(key)
            si = DBSREngine.OUTPUT_SLOTS - 1
        plan = self.slots[key][si]
        want_fw = bool(getattr(self.net, 'return_fusion_weights', True))
        self._set_fw(plan, want_fw)
        stream = L.stream_ptr(dev)
        plan.bufs['burst'].copy_(burst.to(torch.float32), non_blocking=True)
        if getattr(self.net, 'use_graph', False):
            g = self.graphs.get((key, si, want_fw))
            if g is None:
                plan.run(stream)                      # warm-up outside capture
                g = self._capture(plan, dev)
                self.graphs[(key, si, want_fw)] = g
            g.replay()
        else:
            plan.run(stream)
        pred, offs = plan.bufs['pred'], plan.bufs['offsets']
        fw_t = plan.FW.t if want_fw else None
        if copy:
            pred, offs = pred.clone(), offs.clone()
            fw_t = fw_t.clone() if want_fw else None
        # [B*N,H,W,C] channels-last storage viewed as the reference's [B,N,C,H,W]; fp32 NCHW on first read
        native = fw_t.view(B, N, H, W, -1).permute(0, 1, 4, 2, 3) if want_fw else None
        return pred.view(pred.shape), DBSRAux(offs.view(B, N - 1, 2, H, W), native)

    # ---------------- frame-sharded fusion (BASELINE configs[4]) ----------------
    def decoder_halo(self):
        """LR rows of context the decoder needs beyond a row slab for the slab's prediction to be exact: one per
        LR 3x3 conv (init + pre ResBlocks) plus the HR 3x3 convs (blur + post ResBlocks) in LR rows."""
        from .parallel import decoder_halo_rows
        return decoder_halo_rows(len(self.dec_pre), len(self.dec_post), self.s, self.blur is not None)

    def _build_combine(self, R, B, H, W, rows=None):
        """dbsr_fuse_combine of R ranks' gathered statistics -> FUS, then the decoder -- over all rows, or (frame
        sharding with a split decoder) over LR rows `rows` = [lo, hi) widened by decoder_halo() rows on each side
        (the prediction of [lo, hi) is then exactly the unsplit one)."""
        dt, dev = self.dtype, self.device
        C = self.enc_out.cout
        plan = Plan()
        bufs = {'gathered': torch.zeros(R, B, H, W, 3 * C, dtype=torch.float32, device=dev)}
        FUS = NHWC(B, H, W, C, dt, dev)
        plan.add('merge.fuse_combine', L.lib().dbsr_fuse_combine, R, B, H * W, C, bufs['gathered'].data_ptr(),
                 FUS.d(0))
        if rows is None:
            self._decoder(plan, B, H, W, FUS, bufs)
            plan.valid = (0, H * self.s)
        else:
            lo, hi = rows
            from .parallel import decoder_slab
            y0, y1 = decoder_slab(lo, hi, H, self.decoder_halo())
            # every conv takes the whole image's kernel, tile and K split (plan_h), so the slab's rows are
            # bitwise the unsplit decoder's: kernel choice never depends on the slab height
            plan.plan_rows = (y1 - y0, H)
            self._decoder(plan, B, y1 - y0, W, FUS.rows(y0, y1), bufs)
            plan.plan_rows = None
            plan.valid = ((lo - y0) * self.s, (hi - y0) * self.s)
        plan.keep.append(FUS)
        plan.finalize_workspace(dev)
        plan.bufs = bufs
        return plan

    def _ready(self, burst):
        if not burst.is_cuda:
            raise RuntimeError('DBSRNet (MI355X engine) needs the burst on a HIP device; got %s' % burst.device)
        if self.device != burst.device or self.sig != _param_signature(self.net):
            self._pack(burst.device)
        elif self.weights_stale:
            self.refresh_weights()

    def forward_partial(self, burst, first_frame):
        """Encoder, alignment, warp and weight predictor of a frame shard `burst` [B,n,4,H,W] (frame 0 =
        the burst's reference frame, needed by every shard for the warp and base_feat), then the fusion
        statistics of frames [first_frame, n).  Returns (stats [B,H,W,3C] fp32 -- the plan's static
        buffer, overwritten by the next call -- and offsets [B,n-1,2,H,W])."""
        self._ready(burst)
        B, N, _, H, W = burst.shape
        if N < 2:
            raise ValueError('a frame shard needs the reference frame and at least one other frame')
        if not (self.softmax and self.ref_base):
            raise NotImplementedError('frame-sharded fusion needs softmax=True and use_base_frame=True: the '
                                      'shards\' log-sum-exp statistics (dbsr_fuse_partial) combine only the softmax, '
                                      'and a mean base needs every frame\'s projection')
        key = ('partial', B, N, H, W, int(first_frame))
        plan = self.plans.get(key)
        if plan is None:
            plan = self.plans[key] = self._build(B, N, H, W, mode='partial', first_frame=int(first_frame))
        plan.bufs['burst'].copy_(burst.to(torch.float32), non_blocking=True)
        plan.run(L.stream_ptr(burst.device))
        return plan.bufs['stats'], plan.bufs['offsets'].view(B, N - 1, 2, H, W)

    def gathered_buffer(self, R, B, H, W, rows=None):
        """The combine plan's input buffer [R,B,H,W,3C] fp32: all-gather the ranks' stats straight into it."""
        if self.device is None:
            raise RuntimeError('gathered_buffer: run forward_partial first (the engine packs its weights there)')
        key = ('combine', R, B, H, W, rows)
        plan = self.plans.get(key)
        if plan is None:
            plan = self.plans[key] = self._build_combine(R, B, H, W, rows)
        return plan.bufs['gathered']

    def combine_decode(self, gathered, rows=None):
        """Log-sum-exp combine of gathered [R,B,H,W,3C] statistics + decoder -> pred [B,3,sH,sW] (clone); with
        rows = [lo, hi) (LR rows) only the prediction rows [s*lo, s*hi), from a decoder run on that slab plus
        its halo."""
        self._ready(gathered)
        R, B, H, W = gathered.shape[:4]
        rows = None if rows is None else (int(rows[0]), int(rows[1]))
        buf = self.gathered_buffer(R, B, H, W, rows)
        if buf.data_ptr() != gathered.data_ptr():
            buf.copy_(gathered, non_blocking=True)
        plan = self.plans[('combine', R, B, H, W, rows)]
        plan.run(L.stream_ptr(gathered.device))
        a, b = plan.valid
        return plan.bufs['pred'][:, :, a:b].clone()


# ==================================================================================================
# standalone PWC-Net (the alignment sub-seam, pwcnet.py:248-281)
# ==================================================================================================
class PWCEngine:
    def __init__(self, module):
        self.module = module
        self.dtype = module.compute_dtype
        self.sig = None
        self.device = None
        self.plans = {}

    def matches(self, module):
        return module is self.module and self.dtype == module.compute_dtype and self.sig == _param_signature(module)

    def forward(self, source_img, target_img):
        if not source_img.is_cuda:
            raise RuntimeError('PWCNet (MI355X engine) needs inputs on a HIP device')
        H, W = source_img.shape[-2:]
        src = source_img.reshape(-1, 3, H, W)
        tgt = target_img.reshape(-1, 3, H, W)
        if self.module.rgb2bgr:
            src, tgt = src[:, [2, 1, 0]], tgt[:, [2, 1, 0]]
        P = src.shape[0]
        dev = src.device
        if self.device != dev or self.sig != _param_signature(self.module):
            self.pwc = PWCPlanner(self.module, _Weights(self.dtype, dev, L.stream_ptr(dev)))
            self.device, self.sig, self.plans = dev, _param_signature(self.module), {}
        key = (P, H, W)
        plan = self.plans.get(key)
        lib = L.lib()
        if plan is None:
            plan = Plan()
            Hp, Wp = int(math.ceil(H / 64.0) * 64), int(math.ceil(W / 64.0) * 64)
            # frames 0..P-1 = target (tenFirst), P..2P-1 = source (tenSecond): pwcnet.py:273
            inp = torch.zeros(2 * P, 1, 4, H, W, dtype=torch.float32, device=dev)
            rgb = NHWC(2 * P, Hp, Wp, 8, self.dtype, dev)
            flow_out = NHWC(P, Hp // 4, Wp // 4, 2, torch.float32, dev)
            offs = torch.zeros(P, 2, H, W, dtype=torch.float32, device=dev)
            plan.add('pack_rgb', lib.dbsr_pack_burst, 2 * P, 1, H, W, inp.data_ptr(), L.NULL_TENSOR, Hp, Wp, rgb.d(0))
            self.pwc.build(plan, self.dtype, dev, 2 * P, Hp, Wp, P, first_map=IDENTITY, second_map=(1, 1, P, 1),
                           rgb=rgb, flow_out=flow_out)
            # B = P bursts of N = 2 frames -> pair p = burst p
            plan.add('flow_finalize', lib.dbsr_flow_finalize, P, 2, Hp // 4, Wp // 4, flow_out.d(0), H, W, Hp, Wp,
                     offs.data_ptr(), 1.0, L.NULL_TENSOR)
            plan.keep.extend([rgb, flow_out])
            plan.finalize_workspace(dev)
            plan.inp, plan.offs = inp, offs
            self.plans[key] = plan
        # pack_burst expects 4 planes (R, G1, G2, B) -> put G in both green planes so mean(G1,G2) = G
        v = plan.inp.view(2, P, 4, H, W)
        for dst, srcimg in ((v[0], tgt), (v[1], src)):
            dst[:, 0] = srcimg[:, 0]
            dst[:, 1] = srcimg[:, 1]
            dst[:, 2] = srcimg[:, 1]
            dst[:, 3] = srcimg[:, 2]
        plan.run(L.stream_ptr(dev))
        return plan.offs.clone()
