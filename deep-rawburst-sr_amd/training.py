"""Training step of the DBSR network on the HIP kernels (BASELINE.json configs[3]; SURVEY §8e training
row, §8f rank 3).

The reference step (trainers/simple_trainer.py:78-81 with actors/dbsr_actors.py:27-47 and the
train_settings/dbsr/default_synthetic.py:85-96 objective / optimizer):

    pred, _ = net(burst); loss = L1(pred, frame_gt, boundary_ignore=40)
    optimizer.zero_grad(); loss.backward(); optimizer.step()        # Adam, lr 1e-4

PWC-Net is frozen (train_alignmentnet=False: its forward runs under no_grad, encoders.py:56-61), so
only the 3.64 M DBSR parameters train.  Multi-GPU: the reference wraps the net in nn.DataParallel
(admin/multigpu.py:8-14); here one process per GPU runs its shard of the global batch and the fp32
gradients are averaged by bucketed RCCL all-reduces (torch.distributed) that start as soon as the
backward of a bucket's layers has been issued, overlapping the rest of the backward.

Every op of the step is a C-ABI launch (libdbsr_hip.so): the forward reuses the inference plan's
kernels with every saved activation in its own buffer, conv dgrad is dbsr_conv2d on dgrad-packed
weights with the gate/residual epilogue (ReLU and ResBlock backward fused into the conv), conv wgrad
is dbsr_conv_wgrad (MFMA), and the remaining backward ops and Adam are the train_ops kernels.
"""
import ctypes
import math

import torch
import torch.distributed as dist

from . import _lib as L
from ._lib import IDENTITY
from .engine import NHWC, Plan, PWCPlanner, _Weights, cpad, gauss_kernel3, merging_variant, r8


class _WS:
    """Placeholder for a scratch pointer patched in once the plan knows its largest request."""
    def __init__(self, kind, nbytes):
        self.kind, self.nbytes = kind, int(nbytes)


class PackedW:
    """Packed MFMA weights built from a fp32 torch-layout weight tensor (re-packed after every update)."""
    def __init__(self, w, b, dtype, device, shuffle=1, stride=1, pad=None, dil=1):
        self.src_w, self.src_b = w, b
        self.cout, self.cin, self.kh, self.kw = w.shape
        self.stride, self.dil = stride, dil
        self.pad = self.kh // 2 if pad is None else pad
        self.shuffle = shuffle
        self.dtype = dtype
        self.w = torch.empty(L.lib().dbsr_conv_packed_elems(self.cout, self.cin, self.kh, self.kw), dtype=dtype,
                             device=device)
        self.bias = torch.empty(self.cout, dtype=torch.float32, device=device) if b is not None else None

    def out_hw(self, h, w):
        return ((h + 2 * self.pad - self.dil * (self.kh - 1) - 1) // self.stride + 1,
                (w + 2 * self.pad - self.dil * (self.kw - 1) - 1) // self.stride + 1)

    def pack_args(self):
        return (self.src_w.data_ptr(), self.src_b.data_ptr() if self.src_b is not None else None, self.cout, self.cin,
                self.kh, self.kw, L.dtype_code(self.dtype), self.shuffle, self.w.data_ptr(),
                self.bias.data_ptr() if self.bias is not None else None)


class TConv:
    """A trainable nn.Conv2d: forward-packed weights, dgrad weights (transposed + flipped, packed), and
    where its gradients live in the flat gradient buffer."""
    def __init__(self, mod, trainer, dtype, device, shuffle=1):
        self.mod = mod
        w, b = mod.weight, mod.bias
        self.fwd = PackedW(w.data, b.data if b is not None else None, dtype, device, shuffle=shuffle)
        co, ci, kh, kw = w.shape
        self.wt = torch.empty(ci, co, kh, kw, dtype=torch.float32, device=device)
        self.bwd = PackedW(self.wt, None, dtype, device)
        self.gw = trainer.grad_view(w)
        self.gb = trainer.grad_view(b) if b is not None else None
        self.cout, self.cin, self.k = co, ci, kh

    def sub_dgrad(self, lo, hi, dtype, device):
        """dgrad weights producing only input channels [lo, hi) (a slice of wt: rows of the dgrad conv)."""
        p = PackedW(self.wt[lo:hi], None, dtype, device)
        self.extra = getattr(self, 'extra', []) + [p]
        return p

    def pack_jobs(self):
        """This conv's repacks as dbsr_pack_job entries (dbsr_conv_pack_weights_batch): the forward weights and
        every dgrad copy, the latter straight from the module's weight (no fp32 transpose pass)."""
        code = L.dtype_code(self.fwd.dtype)
        w = self.mod.weight
        f = self.fwd
        jobs = [L.PackJob(w=w.data_ptr(), bias=f.src_b.data_ptr() if f.src_b is not None else None,
                          w_packed=f.w.data_ptr(), bias_out=f.bias.data_ptr() if f.bias is not None else None,
                          cout=f.cout, cin=f.cin, kh=f.kh, kw=f.kw, dtype=code, shuffle=f.shuffle)]
        for p in [self.bwd] + getattr(self, 'extra', []):
            # p packs rows [lo, lo + p.cout) of wt = w transposed (ci, co) and flipped
            lo = (p.src_w.data_ptr() - self.wt.data_ptr()) // (4 * self.cout * self.k * self.k)
            jobs.append(L.PackJob(w=w.data_ptr(), bias=None, w_packed=p.w.data_ptr(),
                                  bias_out=p.bias.data_ptr() if p.bias is not None else None, cout=p.cout, cin=p.cin,
                                  kh=p.kh, kw=p.kw, dtype=code, shuffle=1, transposed=1, lo=lo, src_cin=self.cin))
        return jobs

    def repack_ops(self, plan):
        lib = L.lib()
        plan.add('pack.' + self.name, lib.dbsr_conv_pack_weights, *self.fwd.pack_args())
        w = self.mod.weight
        plan.add('dgradw.' + self.name, lib.dbsr_dgrad_weights, w.data_ptr(), self.cout, self.cin, self.k, self.k,
                 self.wt.data_ptr())
        for p in [self.bwd] + getattr(self, 'extra', []):
            plan.add('packT.' + self.name, lib.dbsr_conv_pack_weights, *p.pack_args())


class DBSRTrainer:
    """One optimisation step per call on the HIP kernels: step(burst, frame_gt) -> loss (device scalar).

    net: a dbsr_amd DBSRNet on a HIP device (compute dtype bf16 or fp32).  Its DBSR parameters are
    re-pointed into one flat fp32 buffer (the optimizer's master copy; the module sees the updates);
    `flat_grad` holds the step's gradients in the same layout (decoder first, then merging, then
    encoder: the order the backward completes them, so the bucketed all-reduce can start early).
    """
    # re-pack every conv's weights in one launch (dbsr_conv_pack_weights_batch, bitwise the per-conv
    # pack / dgrad-transpose / pack launches it replaces: False runs those, for A/B and the equality test)
    BATCH_REPACK = True
    # forward: the weight predictor's output conv fused with the softmax + fusion (as the inference engine's
    # DBSREngine.FUSED_WP_OUT); False: the conv into a logits buffer + dbsr_fuse_softmax
    FUSED_WP_OUT = True

    def __init__(self, net, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, boundary_ignore=40, process_group=None,
                 bucket_bytes=4 << 20, optimizer=True):
        dev = next(net.parameters()).device
        if dev.type != 'cuda':
            raise RuntimeError('DBSRTrainer needs the network on a HIP device')
        self.net, self.dev, self.dtype = net, dev, net.compute_dtype
        if self.dtype == torch.float16:
            # no loss scaling: the L1 gradient 1/count (~4.7e-8 at configs[3]) is below fp16's smallest
            # subnormal, so an fp16 backward would underflow to zero
            raise ValueError('DBSRTrainer: train in torch.bfloat16 or torch.float32 (fp16 has no loss scaling here)')
        self.lr, self.betas, self.eps, self.bi = lr, betas, eps, boundary_ignore
        if getattr(net.encoder, 'train_alignmentnet', False):
            # the reference then backpropagates into PWC-Net (encoders.py:56-57); the HIP backward stops at the
            # flows, so refuse rather than train without alignment gradients
            raise NotImplementedError('DBSRTrainer: train_alignmentnet=True (PWC-Net training) is not on the HIP '
                                      'backward; build the net with train_alignmentnet=False (dbsrnet_cvpr2021 default)')
        softmax, ref_base, self.offset_modulo = merging_variant(net.merging)
        if not (softmax and ref_base):
            # the backward kernels are the softmax's (dbsr_fuse_backward) and the reference-frame base's
            # (dbsr_merge_prep_backward); the inference engine runs these variants, training does not
            raise NotImplementedError('DBSRTrainer: WeightedSum(softmax=False / use_base_frame=False) is not on the '
                                      'HIP backward (dbsrnet_cvpr2021 defaults: softmax=True, use_base_frame=True)')
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if (dist.is_available() and dist.is_initialized()) else 1
        # PWC-Net runs without gradients (train_alignmentnet=False: encoders.py:58-61); its parameters are left
        # as the caller set them -- they never receive a .grad from this backward
        mods = self._trainable_convs()
        self.params = []
        for m in mods:
            self.params.append(m.weight)
            if m.bias is not None:
                self.params.append(m.bias)
        n = sum(p.numel() for p in self.params)
        self.flat = torch.empty(n, dtype=torch.float32, device=dev)
        self.flat_grad = torch.zeros(n, dtype=torch.float32, device=dev)
        # Adam moments (not allocated when an external optimizer steps the parameters: the autograd path)
        self.exp_avg = torch.zeros(n if optimizer else 0, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(n if optimizer else 0, dtype=torch.float32, device=dev)
        self.offset = {}
        o = 0
        for p in self.params:
            k = p.numel()
            self.flat[o:o + k].copy_(p.detach().reshape(-1).float())
            p.data = self.flat[o:o + k].view(p.shape)
            self.offset[id(p)] = (o, k)
            o += k
        self.n_params = n
        self.bucket_bytes = bucket_bytes
        self.step_count = 0
        self.plans = {}
        self.loss = torch.zeros(1, dtype=torch.float32, device=dev)
        self.use_graph = True         # step(): replay the plan as HIP graphs after its first (eager) run
        self._pack()

    def _trainable_convs(self):
        return trainable_convs(self.net)

    def grad_view(self, p):
        o, k = self.offset[id(p)]
        return self.flat_grad.data_ptr() + 4 * o

    def _pack(self):
        net, dt, dev = self.net, self.dtype, self.dev
        enc, mer, dec = net.encoder, net.merging, net.decoder
        T = lambda m, shuffle=1: TConv(m, self, dt, dev, shuffle)                     # noqa: E731
        self.pwc = PWCPlanner(enc.alignment_net, _Weights(dt, dev, L.stream_ptr(dev)))
        self.enc_init = T(enc.init_layer[0])
        self.enc_res = [(T(b.conv1[0]), T(b.conv2[0])) for b in enc.res_layers]
        self.enc_out = T(enc.out_layer[0])
        self.proj = T(mer.feat_project_layer[0])
        ofe = list(mer.offset_feat_extractor)
        self.ofe_init = T(ofe[0][0])
        self.ofe_res = [(T(b.conv1[0]), T(b.conv2[0])) for b in ofe[1:]]
        wp = list(mer.weight_predictor)
        self.wp_init = T(wp[0][0])
        self.wp_res = [(T(b.conv1[0]), T(b.conv2[0])) for b in wp[1:-1]]
        self.wp_out = T(wp[-1][0])
        self.dec_init = T(dec.init_layer[0])
        self.dec_pre = [(T(b.conv1[0]), T(b.conv2[0])) for b in dec.pre_res_layers]
        up = dec.upsample_layer
        self.s = up.upsample_factor
        self.dec_up = T(up.conv_layer[0], shuffle=self.s)
        self.blur = gauss_kernel3(up.gauss_blur_sd, up.gauss_ksz) if up.gauss_blur_sd is not None else None
        self.dec_post = [(T(b.conv1[0]), T(b.conv2[0])) for b in dec.post_res_layers]
        self.pred = T(dec.predictor[0])
        if self.pred.cin != 32:
            # the predictor's forward / backward (dbsr_head_forward / dbsr_head_backward) take 32 input channels,
            # the reference's default dec_post_conv_dim: refuse here, not at the first step
            raise NotImplementedError('DBSRTrainer: dec_post_conv_dim = %d; the HIP predictor head trains 32 '
                                      'channels (dbsrnet_cvpr2021 default)' % self.pred.cin)
        # dgrad of the weight predictor's first conv, split: [base | diff] (ungated, to merge-prep) and the
        # offset features (gated by the offset-feature extractor's ReLU output)
        pd = self.proj.cout
        self.wp_init_bd = self.wp_init.sub_dgrad(0, 2 * pd, dt, dev)
        self.wp_init_of = self.wp_init.sub_dgrad(2 * pd, self.wp_init.cin, dt, dev)
        self.tconvs = [self.enc_init, self.enc_out, self.proj, self.ofe_init, self.wp_init, self.wp_out, self.dec_init,
                       self.dec_up, self.pred]
        for lst in (self.enc_res, self.ofe_res, self.wp_res, self.dec_pre, self.dec_post):
            for c1, c2 in lst:
                self.tconvs += [c1, c2]
        names = {id(m): n for n, m in net.named_modules()}
        for tc in self.tconvs:
            tc.name = names[id(tc.mod)]

    # ------------------------------------------------------------------------------------------------
    def _build(self, B, N, H, W):
        dt, dev, lib = self.dtype, self.dev, L.lib()
        plan = Plan()
        plan.lane = 0
        F, P = B * N, B * (N - 1)
        C = self.enc_out.cout
        hw = (H, W)
        S = self.s
        bufs = {'burst': torch.zeros(B, N, 4, H, W, dtype=torch.float32, device=dev)}
        ws_req = []

        def ws(kind, nbytes):
            w = _WS(kind, nbytes)
            ws_req.append(w)
            return w

        def wgrad(name, tc, n, h, w, x, xc0, dy, dyc0, xmap=IDENTITY, dymap=IDENTITY, accumulate=0, cin=None, cout=None):
            """weight gradient, and the bias gradient (when the conv has one) from the same pass over dy"""
            ci = tc.cin if cin is None else cin
            co = tc.cout if cout is None else cout
            need = lib.dbsr_conv_wgrad_workspace_bytes(n, h, w, ci, co, tc.k)
            work = ('flop', 2.0 * n * h * w * ci * co * tc.k * tc.k)
            if tc.gb is None:
                plan.add('wgrad.' + name, lib.dbsr_conv_wgrad, n, h, w, x.d(xc0, xmap), ci, dy.d(dyc0, dymap), co,
                         tc.k, tc.gw, accumulate, ws('wg', need), need, work=work)
            else:
                plan.add('wgrad.' + name, lib.dbsr_conv_wgrad_bias, n, h, w, x.d(xc0, xmap), ci, dy.d(dyc0, dymap),
                         co, tc.k, tc.gw, tc.gb, accumulate, ws('wg', need), need, work=work)
            plan.kernel[len(plan.ops) - 1] = 'conv_wgrad'

        # ================= forward with saved activations =================
        if DBSRTrainer.BATCH_REPACK:
            # every conv's forward and dgrad weights re-packed from the updated fp32 master in one launch
            jobs = [j for tc in self.tconvs for j in tc.pack_jobs()]
            arr = (L.PackJob * len(jobs))(*jobs)
            nblk = lib.dbsr_pack_batch_prepare(arr, len(jobs))
            if nblk < 0:
                L.check(-1, 'dbsr_pack_batch_prepare')
            table = torch.frombuffer(bytearray(arr), dtype=torch.uint8).to(dev)
            plan.keep.append(table)
            plan.add('repack.all', lib.dbsr_conv_pack_weights_batch, table.data_ptr(), len(jobs), nblk)
        else:
            for tc in self.tconvs:
                tc.repack_ops(plan)
        raw = NHWC(F, H, W, 8, dt, dev)
        Hp, Wp = int(math.ceil(H / 64.0) * 64), int(math.ceil(W / 64.0) * 64)
        rgb = NHWC(F, Hp, Wp, 8, dt, dev)
        offsets = torch.zeros(P, 2, H, W, dtype=torch.float32, device=dev)
        om = NHWC(F, H, W, 8, dt, dev)
        plan.add('pack_burst', lib.dbsr_pack_burst, B, N, H, W, bufs['burst'].data_ptr(), raw.d(0), Hp, Wp, rgb.d(0))
        flow_out = NHWC(P, Hp // 4, Wp // 4, 2, torch.float32, dev)
        self.pwc.build(plan, dt, dev, F, Hp, Wp, P, first_map=(N - 1, N, 0, 0), second_map=(N - 1, N, 1, 1), rgb=rgb,
                       flow_out=flow_out)
        plan.add('flow_finalize', lib.dbsr_flow_finalize, B, N, Hp // 4, Wp // 4, flow_out.d(0), H, W, Hp, Wp,
                 offsets.data_ptr(), self.offset_modulo, om.d(0))

        def res_fwd(name, blocks, n, hw_, x, xc0, width, last_out=None):
            """ResBlocks with every activation kept: returns [(x, xc0, t, y, yc0)] per block."""
            saved = []
            for i, (c1, c2) in enumerate(blocks):
                t = NHWC(n, hw_[0], hw_[1], r8(width), dt, dev)
                if i == len(blocks) - 1 and last_out is not None:
                    y, yc0 = last_out
                else:
                    y, yc0 = NHWC(n, hw_[0], hw_[1], r8(width), dt, dev), 0
                plan.conv(f'{name}{i}.conv1', c1.fwd, n, x, xc0, hw_, t, 0, L.ACT_RELU)
                plan.conv(f'{name}{i}.conv2', c2.fwd, n, t, 0, hw_, y, yc0, L.ACT_NONE, res=x, rc0=xc0,
                          post_act=L.ACT_RELU)
                saved.append((x, xc0, t, y, yc0))
                x, xc0 = y, yc0
            return saved

        pd, od = self.proj.cout, self.ofe_init.cout
        WP = NHWC(F, H, W, 2 * pd + od, dt, dev)
        o0 = NHWC(F, H, W, od, dt, dev)
        plan.conv('ofe.init', self.ofe_init.fwd, F, om, 0, hw, o0, 0, L.ACT_RELU)
        ofe_s = res_fwd('ofe.res', self.ofe_res, F, hw, o0, 0, od, last_out=(WP, 2 * pd))
        e0 = NHWC(F, H, W, r8(self.enc_init.cout), dt, dev)
        plan.conv('enc.init', self.enc_init.fwd, F, raw, 0, hw, e0, 0, L.ACT_RELU)
        enc_s = res_fwd('enc.res', self.enc_res, F, hw, e0, 0, self.enc_init.cout)
        e_last = enc_s[-1][3] if enc_s else e0
        E = NHWC(F, H, W, C, dt, dev)
        plan.conv('enc.out', self.enc_out.fwd, F, e_last, 0, hw, E, 0, L.ACT_RELU)
        PJ = NHWC(F, H, W, r8(pd), dt, dev)
        plan.conv('proj_ref', self.proj.fwd, B, E, 0, hw, PJ, 0, L.ACT_RELU, xmap=(1, N, 0, 1), ymap=(1, N, 0, 1))
        Wf = NHWC(max(P, 1), H, W, C, dt, dev)
        plan.add('warp', lib.dbsr_warp_bilinear, P, H, W, C, E.d(0, (N - 1, N, 1, 1)), offsets.data_ptr(), 2 * H * W,
                 Wf.d(0))
        plan.conv('proj_oth', self.proj.fwd, P, Wf, 0, hw, PJ, 0, L.ACT_RELU, ymap=(N - 1, N, 1, 1))
        plan.add('merge_prep', lib.dbsr_merge_prep, B, N, H * W, pd, PJ.d(0), WP.d(0))
        qw = self.wp_init.cout
        q0 = NHWC(F, H, W, qw, dt, dev)
        plan.conv('wp.init', self.wp_init.fwd, F, WP, 0, hw, q0, 0, L.ACT_RELU)
        wp_s = res_fwd('wp.res', self.wp_res, F, hw, q0, 0, qw)
        q_last = wp_s[-1][3] if wp_s else q0
        FUS = NHWC(B, H, W, C, dt, dev)
        FW = NHWC(F, H, W, C, dt, dev)
        # the weight predictor's output conv + softmax + fusion in one launch (dbsr_conv_fuse_softmax, fp32 logits
        # that never reach memory: the backward needs only the weights FW, merging.py:116-124) where the library
        # serves the shape; else the conv into 16-bit logits + dbsr_fuse_softmax
        LG = None
        if not (DBSRTrainer.FUSED_WP_OUT and plan.conv_fuse('wp.out+fuse', self.wp_out.fwd, B, N, q_last, hw,
                                                             E.d(0, (1, N, 0, 1)), Wf.d(0), FUS.d(0), FW.d(0))
                is not None):
            LG = NHWC(F, H, W, C, dt, dev)
            plan.conv('wp.out', self.wp_out.fwd, F, q_last, 0, hw, LG, 0, L.ACT_NONE)
            plan.add('fuse', lib.dbsr_fuse_softmax, B, N, H * W, C, LG.d(0), E.d(0, (1, N, 0, 1)), Wf.d(0), FUS.d(0),
                     FW.d(0))
        gd = self.dec_init.cout
        g0 = NHWC(B, H, W, gd, dt, dev)
        plan.conv('dec.init', self.dec_init.fwd, B, FUS, 0, hw, g0, 0, L.ACT_RELU)
        pre_s = res_fwd('dec.pre', self.dec_pre, B, hw, g0, 0, gd)
        g_last = pre_s[-1][3] if pre_s else g0
        pc = self.dec_up.cout // (S * S)
        HS, WS = H * S, W * S
        S0 = NHWC(B, HS, WS, pc, dt, dev)
        plan.conv('dec.upsample', self.dec_up.fwd, B, g_last, 0, hw, S0, 0, L.ACT_RELU, out_mode=L.OUT_SHUFFLE,
                  shuffle=S)
        if self.blur is not None:
            S1 = NHWC(B, HS, WS, pc, dt, dev)
            kbuf = (ctypes.c_float * 9)(*self.blur)
            kflip = (ctypes.c_float * 9)(*self.blur[::-1])       # correlation^T = correlation with the flipped kernel
            plan.keep.extend([kbuf, kflip])
            plan.add('dec.blur', lib.dbsr_gauss_blur3, B, HS, WS, pc, S0.d(0), kbuf, S1.d(0))
        else:
            S1 = S0
        post_s = res_fwd('dec.post', self.dec_post, B, (HS, WS), S1, 0, pc)
        h_last = post_s[-1][3] if post_s else S1
        hc = self.pred.cout
        pred = torch.zeros(B, hc, HS, WS, dtype=torch.float32, device=dev)
        # the predictor on its own (h_last is kept for the backward): fp32 weights, fp32 NCHW out
        pmod = self.pred.mod
        plan.add('dec.predictor', lib.dbsr_head_forward, B, HS * WS, h_last.d(0), pc, pmod.weight.data_ptr(),
                 pmod.bias.data_ptr() if pmod.bias is not None else None, hc, pred.data_ptr(),
                 work=('flop', 2.0 * B * HS * WS * pc * hc))
        bufs['pred'] = pred
        bufs['offsets'] = offsets
        bufs['gt'] = torch.zeros(B, 3, HS, WS, dtype=torch.float32, device=dev)

        # ================= backward =================
        plan.add('zero_grad', lib.dbsr_zero, self.flat_grad.data_ptr(), self.flat_grad.numel() * 4)
        buckets = []                     # (op index after which this bucket's grads are final, lo, hi)

        def mark_bucket(tc_list):
            lo = min(self.offset[id(p)][0] for tc in tc_list for p in ([tc.mod.weight] + ([tc.mod.bias] if tc.mod.bias is not None else [])))
            hi = max(sum(self.offset[id(p)]) for tc in tc_list for p in ([tc.mod.weight] + ([tc.mod.bias] if tc.mod.bias is not None else [])))
            buckets.append((len(plan.ops), lo, hi))

        dP = NHWC(B, HS, WS, 8, dt, dev)
        nlb = (B * HS * WS + 255) // 256
        plan.fwd_end = len(plan.ops)            # ops[:fwd_end]: the forward with saved activations (+ grad zeroing)
        plan.add('l1_loss_bwd', lib.dbsr_l1_loss_backward, B, 3, HS, WS, self.bi, pred.data_ptr(),
                 bufs['gt'].data_ptr(), dP.d(0), self.loss.data_ptr(), ws('l1', 4 * nlb), 4 * nlb)
        # autograd: the same backward from an upstream dL/dpred instead of the built-in L1 objective
        bufs['gpred'] = torch.zeros(B, 3, HS, WS, dtype=torch.float32, device=dev)
        plan.grad_in_op = (lib.dbsr_relu_grad, (B, 3, HS, WS, pred.data_ptr(), bufs['gpred'].data_ptr(), dP.d(0)),
                           'relu_grad', 0)
        # predictor backward in one pass over dP and h_last: its dgrad gated by h_last's ReLU, weight and bias grads
        gh = NHWC(B, HS, WS, r8(pc), dt, dev)
        need = lib.dbsr_head_backward_workspace_bytes(B, HS * WS, pc, hc)
        plan.add('bwd.dec.predictor', lib.dbsr_head_backward, B, HS * WS, h_last.d(0), pc, dP.d(0),
                 pmod.weight.data_ptr(), hc, gh.d(0), self.pred.gw, self.pred.gb, 0, ws('hb', need), need,
                 work=('flop', 4.0 * B * HS * WS * pc * hc))

        def res_bwd(name, blocks, saved, n, hw_, g, gc0, gate_first):
            """ResBlock backward (blocks.py:81-96) from g = dL/dy * [y > 0]; returns the gradient w.r.t. the
            chain's input, gated by that input's ReLU when gate_first (else ungated)."""
            for i in reversed(range(len(blocks))):
                c1, c2 = blocks[i]
                x, xc0, t, y, yc0 = saved[i]
                dt_ = NHWC(n, hw_[0], hw_[1], t.ld, dt, dev)
                plan.conv(f'bwd.{name}{i}.conv2', c2.bwd, n, g, gc0, hw_, dt_, 0, L.ACT_NONE, gate=t)
                wgrad(f'{name}{i}.conv2', c2, n, hw_[0], hw_[1], t, 0, g, gc0)
                dx = NHWC(n, hw_[0], hw_[1], t.ld, dt, dev)
                gate = x if (i > 0 or gate_first) else None
                plan.conv(f'bwd.{name}{i}.conv1', c1.bwd, n, dt_, 0, hw_, dx, 0, L.ACT_NONE, res=g, rc0=gc0,
                          gate=gate, gc0=xc0 if gate is not None else 0)
                wgrad(f'{name}{i}.conv1', c1, n, hw_[0], hw_[1], x, xc0, dt_, 0)
                plan.keep.extend([dt_, dx])         # launches hold raw pointers: the plan owns every buffer
                g, gc0 = dx, 0
            return g, gc0

        dS1, _ = res_bwd('dec.post', self.dec_post, post_s, B, (HS, WS), gh, 0, gate_first=False)
        if self.blur is not None:
            dS0 = NHWC(B, HS, WS, pc, dt, dev)
            plan.add('bwd.dec.blur', lib.dbsr_gauss_blur3, B, HS, WS, pc, dS1.d(0), kflip, dS0.d(0))
        else:
            dS0 = dS1
        dU = NHWC(B, H, W, self.dec_up.cout, dt, dev)
        plan.add('bwd.dec.unshuffle', lib.dbsr_unshuffle_gate, B, H, W, S, pc, dS0.d(0), S0.d(0), dU.d(0))
        wgrad('dec.upsample', self.dec_up, B, H, W, g_last, 0, dU, 0)
        gp = NHWC(B, H, W, gd, dt, dev)
        plan.conv('bwd.dec.upsample', self.dec_up.bwd, B, dU, 0, hw, gp, 0, L.ACT_NONE, gate=g_last)
        gi, _ = res_bwd('dec.pre', self.dec_pre, pre_s, B, hw, gp, 0, gate_first=True)
        if not pre_s:
            pass
        wgrad('dec.init', self.dec_init, B, H, W, FUS, 0, gi, 0)
        dFUS = NHWC(B, H, W, C, dt, dev)
        plan.conv('bwd.dec.init', self.dec_init.bwd, B, gi, 0, hw, dFUS, 0, L.ACT_NONE)
        mark_bucket([self.pred, self.dec_up, self.dec_init] + [c for blk in self.dec_pre + self.dec_post for c in blk])
        # fusion
        dLG = NHWC(F, H, W, C, dt, dev)
        dF0 = NHWC(B, H, W, C, dt, dev)
        dWfF = NHWC(max(P, 1), H, W, C, dt, dev)
        plan.add('bwd.fuse', lib.dbsr_fuse_backward, B, N, H * W, C, FW.d(0), E.d(0, (1, N, 0, 1)), Wf.d(0), FUS.d(0),
                 dFUS.d(0), dLG.d(0), dF0.d(0), dWfF.d(0))
        # weight predictor
        wgrad('wp.out', self.wp_out, F, H, W, q_last, 0, dLG, 0)
        gq = NHWC(F, H, W, qw, dt, dev)
        plan.conv('bwd.wp.out', self.wp_out.bwd, F, dLG, 0, hw, gq, 0, L.ACT_NONE, gate=q_last)
        gq0, _ = res_bwd('wp.res', self.wp_res, wp_s, F, hw, gq, 0, gate_first=True)
        wgrad('wp.init', self.wp_init, F, H, W, WP, 0, gq0, 0)
        dWP = NHWC(F, H, W, 2 * pd + od, dt, dev)
        plan.conv('bwd.wp.init.bd', self.wp_init_bd, F, gq0, 0, hw, dWP, 0, L.ACT_NONE)
        plan.conv('bwd.wp.init.of', self.wp_init_of, F, gq0, 0, hw, dWP, 2 * pd, L.ACT_NONE, gate=WP, gc0=2 * pd)
        # offset-feature extractor (its input, offsets % 1 from the frozen PWC-Net, takes no gradient)
        go, _ = res_bwd('ofe.res', self.ofe_res, ofe_s, F, hw, dWP, 2 * pd, gate_first=True)
        wgrad('ofe.init', self.ofe_init, F, H, W, om, 0, go, 0)
        # merge prep + projection
        dPJ = NHWC(F, H, W, r8(pd), dt, dev)
        plan.add('bwd.merge_prep', lib.dbsr_merge_prep_backward, B, N, H * W, pd, dWP.d(0), PJ.d(0), dPJ.d(0))
        wgrad('proj.ref', self.proj, B, H, W, E, 0, dPJ, 0, xmap=(1, N, 0, 1), dymap=(1, N, 0, 1))
        if P > 0:
            wgrad('proj.oth', self.proj, P, H, W, Wf, 0, dPJ, 0, dymap=(N - 1, N, 1, 1), accumulate=1)
        mark_bucket([self.wp_out, self.wp_init, self.ofe_init, self.proj] +
                    [c for blk in self.wp_res + self.ofe_res for c in blk])
        dEref = NHWC(B, H, W, C, dt, dev)
        plan.conv('bwd.proj.ref', self.proj.bwd, B, dPJ, 0, hw, dEref, 0, L.ACT_NONE, xmap=(1, N, 0, 1), res=dF0)
        dWf = NHWC(max(P, 1), H, W, C, dt, dev)
        dE = NHWC(F, H, W, C, dt, dev)
        if P > 0:
            plan.conv('bwd.proj.oth', self.proj.bwd, P, dPJ, 0, hw, dWf, 0, L.ACT_NONE, xmap=(N - 1, N, 1, 1), res=dWfF)
            # warp backward (owner-computes gather, no atomics) straight into the other frames' encoder-output
            # gradient, gated by the encoder's output ReLU (encoders.py:66-80)
            need = lib.dbsr_warp_backward_gather_workspace_bytes(P, H, W)
            plan.add('bwd.warp', lib.dbsr_warp_backward_gather, P, H, W, C, dWf.d(0), offsets.data_ptr(), 2 * H * W,
                     E.d(0, (N - 1, N, 1, 1)), dE.d(0, (N - 1, N, 1, 1)), ws('wb', need), need)
        plan.add('bwd.enc.gate', lib.dbsr_gate_copy, B, H * W, C, dEref.d(0), E.d(0, (1, N, 0, 1)),
                 dE.d(0, (1, N, 0, 1)))
        # encoder
        wgrad('enc.out', self.enc_out, F, H, W, e_last, 0, dE, 0)
        ge = NHWC(F, H, W, r8(self.enc_init.cout), dt, dev)
        plan.conv('bwd.enc.out', self.enc_out.bwd, F, dE, 0, hw, ge, 0, L.ACT_NONE, gate=e_last)
        ge0, _ = res_bwd('enc.res', self.enc_res, enc_s, F, hw, ge, 0, gate_first=True)
        wgrad('enc.init', self.enc_init, F, H, W, raw, 0, ge0, 0)
        mark_bucket([self.enc_init, self.enc_out] + [c for blk in self.enc_res for c in blk])
        # ---- scratch: one buffer per kind, as large as its largest request ----
        sizes = {}
        for w in ws_req:
            sizes[w.kind] = max(sizes.get(w.kind, 0), w.nbytes)
        scratch = {k: torch.zeros(max(v // 4, 1), dtype=torch.float32, device=dev) for k, v in sizes.items()}
        for i, (fn, args, name, lane) in enumerate(plan.ops):
            if any(isinstance(a, _WS) for a in args):
                plan.ops[i] = (fn, tuple(scratch[a.kind].data_ptr() if isinstance(a, _WS) else a for a in args), name,
                               lane)
        plan.finalize_workspace(dev)
        plan.keep.extend([raw, rgb, om, flow_out, WP, o0, e0, E, PJ, Wf, q0, LG, FUS, FW, g0, S0, S1, dP, gh, dS0, dU,
                          gp, dFUS, dLG, dF0, dWfF, gq, dWP, dPJ, dEref, dWf, dE, ge, ofe_s, enc_s, wp_s, pre_s,
                          post_s, scratch])
        plan.bufs = bufs
        plan.buckets = buckets
        plan.FW, plan.gen = FW, 0
        plan.graphs, plan.eager_runs = None, 0      # HIP graphs of the step's segments (DBSRTrainer.step)
        return plan

    # ------------------------------------------------------------------------------------------------
    def step(self, burst, frame_gt):
        """One training step on this rank's bursts [B,N,4,H,W] and ground truth [B,3,sH,sW]; returns the
        rank-local loss (device tensor, shape [1])."""
        B, N, _, H, W = burst.shape
        key = (B, N, H, W)
        plan = self.plans.get(key)
        if plan is None:
            plan = self.plans[key] = self._build(B, N, H, W)
        plan.bufs['burst'].copy_(burst.to(torch.float32), non_blocking=True)
        plan.bufs['gt'].copy_(frame_gt.to(torch.float32), non_blocking=True)
        stream = L.stream_ptr(self.dev)
        # segments of the op list between the gradient buckets' completion points: each segment is one HIP
        # graph replay (after one eager step), and a bucket's all-reduce is issued right after its segment
        cuts = [0] + ([b[0] for b in plan.buckets] if self.world > 1 else []) + [len(plan.ops)]
        segs = [(a, b) for a, b in zip(cuts[:-1], cuts[1:]) if b > a]
        if self.use_graph and plan.graphs is None and plan.eager_runs > 0:
            plan.graphs = []
            for a, b in segs:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    plan.run_list(plan.ops[a:b], L.stream_ptr(self.dev))
                plan.graphs.append(g)
        works = []
        bi = 0
        for si, (a, b) in enumerate(segs):
            if plan.graphs is not None:
                plan.graphs[si].replay()
            else:
                plan.run_list(plan.ops[a:b], stream)
            while bi < len(plan.buckets) and plan.buckets[bi][0] == b:
                if self.world > 1:
                    _, lo, hi = plan.buckets[bi]
                    works.append(allreduce_bucket(self.flat_grad, lo, hi, self.pg))
                bi += 1
        plan.eager_runs += 1
        for w_ in works:
            w_.wait()
        self.step_count += 1
        L.check(L.lib().dbsr_adam_step(self.n_params, self.flat.data_ptr(), self.flat_grad.data_ptr(),
                                       self.exp_avg.data_ptr(), self.exp_avg_sq.data_ptr(), self.lr, self.betas[0],
                                       self.betas[1], self.eps, self.step_count, 1.0 / self.world, stream), 'adam')
        # the inference engine packs from the module parameters (now updated in place through their storage):
        # it re-packs them into its existing buffers at its next forward, keeping its plans and graphs
        eng = getattr(self.net, '_engine', None)
        if eng is not None:
            eng.weights_stale = True
        return self.loss.clone()          # (self.loss is the plan's buffer, overwritten by the next step)

    def forward_backward(self, burst, frame_gt):
        """Loss and gradients only (no all-reduce, no optimizer step): for tests."""
        B, N, _, H, W = burst.shape
        key = (B, N, H, W)
        plan = self.plans.get(key)
        if plan is None:
            plan = self.plans[key] = self._build(B, N, H, W)
        plan.bufs['burst'].copy_(burst.to(torch.float32), non_blocking=True)
        plan.bufs['gt'].copy_(frame_gt.to(torch.float32), non_blocking=True)
        plan.run(L.stream_ptr(self.dev))
        return self.loss, plan.bufs['pred']

    # ---- autograd through DBSRNet.forward (the reference's own loop: pred, _ = net(burst); objective(pred,
    # gt).backward(); optimizer.step(); actors/dbsr_actors.py:27-47, trainers/simple_trainer.py:78-81) ----
    def _plan(self, shape):
        B, N, _, H, W = shape
        key = (B, N, H, W)
        plan = self.plans.get(key)
        if plan is None:
            plan = self.plans[key] = self._build(B, N, H, W)
        return plan

    def forward_saved(self, burst):
        """The training forward with every activation kept in the plan's buffers: (pred, offsets, fusion
        weights, token).  The activations stay valid until the next forward of the same shape; `token`
        names them for backward_from."""
        plan = self._plan(burst.shape)
        plan.bufs['burst'].copy_(burst.to(torch.float32), non_blocking=True)
        plan.run_list(plan.ops[:plan.fwd_end], L.stream_ptr(self.dev))
        plan.gen += 1
        B, N, _, H, W = burst.shape
        fw = plan.FW.t.clone().view(B, N, H, W, -1).permute(0, 1, 4, 2, 3)
        return plan.bufs['pred'].clone(), plan.bufs['offsets'].view(B, N - 1, 2, H, W).clone(), fw, \
            (plan, plan.gen)

    def backward_from(self, token, gpred):
        """Gradients of the DBSR parameters (list in self.params order, fp32) from dL/dpred of the forward
        that returned `token`."""
        plan, gen = token
        if plan.gen != gen:
            raise RuntimeError('DBSRNet training: backward() after another forward of the same burst shape -- the '
                               'saved activations are gone (one forward per backward, as in the reference loop)')
        plan.bufs['gpred'].copy_(gpred.to(torch.float32), non_blocking=True)
        fn, args, name, _ = plan.grad_in_op
        L.check(fn(*args, L.stream_ptr(self.dev)), name)
        plan.run_list(plan.ops[plan.fwd_end + 1:], L.stream_ptr(self.dev))
        return [self.flat_grad[o:o + k].view(p.shape).clone() for p in self.params for (o, k) in [self.offset[id(p)]]]

    def grads(self):
        """{parameter name: gradient} views of the flat gradient buffer."""
        names = {id(p): n for n, p in self.net.named_parameters()}
        return {names[id(p)]: self.flat_grad[o:o + k].view(p.shape) for p in self.params
                for (o, k) in [self.offset[id(p)]]}


def trainable_convs(net):
    """The DBSR convs that train, in the order their gradients complete in the backward (decoder, then
    merging, then encoder); the flat parameter / gradient buffers follow this order (weight, bias)."""
    dec, mer, enc = net.decoder, net.merging, net.encoder
    mods = [dec.predictor[0]]
    for b in reversed(list(dec.post_res_layers)):
        mods += [b.conv2[0], b.conv1[0]]
    mods.append(dec.upsample_layer.conv_layer[0])
    for b in reversed(list(dec.pre_res_layers)):
        mods += [b.conv2[0], b.conv1[0]]
    mods.append(dec.init_layer[0])
    wp = list(mer.weight_predictor)
    mods.append(wp[-1][0])
    for b in reversed(wp[1:-1]):
        mods += [b.conv2[0], b.conv1[0]]
    mods.append(wp[0][0])
    ofe = list(mer.offset_feat_extractor)
    for b in reversed(ofe[1:]):
        mods += [b.conv2[0], b.conv1[0]]
    mods.append(ofe[0][0])
    mods.append(mer.feat_project_layer[0])
    mods.append(enc.out_layer[0])
    for b in reversed(list(enc.res_layers)):
        mods += [b.conv2[0], b.conv1[0]]
    mods.append(enc.init_layer[0])
    return mods


def flat_layout(net):
    """[(parameter name, numel)] of the flat buffers, and the (lo, hi) element ranges of the three
    gradient buckets (decoder, merging, encoder) that the backward completes in that order."""
    names = {id(p): n for n, p in net.named_parameters()}
    layout, bounds, o = [], {}, 0
    for m in trainable_convs(net):
        for p in [m.weight] + ([m.bias] if m.bias is not None else []):
            n = names[id(p)]
            layout.append((n, p.numel()))
            part = n.split('.')[0]
            lo, hi = bounds.get(part, (o, o))
            bounds[part] = (min(lo, o), o + p.numel())
            o += p.numel()
    return layout, [bounds['decoder'], bounds['merging'], bounds['encoder']]


def allreduce_bucket(flat_grad, lo, hi, group=None):
    """Start the sum all-reduce of one gradient bucket (RCCL on HIP tensors, gloo on CPU tensors); the
    caller scales by 1/world (folded into the Adam step)."""
    return dist.all_reduce(flat_grad[lo:hi], group=group, async_op=True)


class _DBSRTrainForward(torch.autograd.Function):
    """DBSRNet.forward under autograd: the HIP training forward (activations saved) and, on backward, the
    HIP backward from dL/dpred into the DBSR parameters' gradients (PWC-Net is frozen, encoders.py:56-61)."""

    @staticmethod
    def forward(ctx, burst, engine, *params):
        pred, offs, fw, token = engine.forward_saved(burst)
        ctx.engine, ctx.token = engine, token
        ctx.mark_non_differentiable(offs, fw)
        return pred, offs, fw

    @staticmethod
    def backward(ctx, gpred, goffs, gfw):
        if gpred is None:
            return (None, None) + tuple(None for _ in ctx.engine.params)
        return (None, None) + tuple(ctx.engine.backward_from(ctx.token, gpred.contiguous()))


def _aliased(eng):
    """Every trained parameter still lives in the trainer's flat buffer (p.data = ..., load_state_dict(assign=True)
    or a device move replace the storage; the trainer would then pack a stale copy)."""
    cur = [p for m in trainable_convs(eng.net) for p in [m.weight] + ([m.bias] if m.bias is not None else [])]
    if len(cur) != len(eng.params) or any(a is not b for a, b in zip(cur, eng.params)):
        return False                                   # new Parameter objects (load_state_dict(assign=True))
    base = eng.flat.data_ptr()
    return all(p.data_ptr() == base + 4 * eng.offset[id(p)][0] and p.device == eng.dev and
               p.dtype == torch.float32 for p in eng.params)


def train_forward(net, burst):
    """pred, {'offsets', 'fusion_weights'} of DBSRNet.forward with autograd to the DBSR parameters."""
    eng = getattr(net, '_train_engine', None)
    if eng is None or eng.net is not net or eng.dtype != net.compute_dtype or not _aliased(eng):
        eng = net._train_engine = DBSRTrainer(net, optimizer=False)
    pred, offs, fw = _DBSRTrainForward.apply(burst, eng, *eng.params)
    from .engine import DBSRAux
    return pred, DBSRAux(offs, fw)
