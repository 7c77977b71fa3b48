/* dbsr_hip.h — C ABI of libdbsr_hip.so, the MI355X (gfx950) kernels of the DBSR forward path.
 *
 * Plain pointers, sizes and a hipStream_t passed as void*.  No torch types.  Every entry point
 * returns 0 on success, a positive hipError_t on a HIP launch error, or a negative DBSR_E_* code on
 * an argument error (dbsr_last_error() gives the message).  All pointers are device pointers unless
 * a comment says otherwise.  Entry points are stateless and launch on the given stream only (no
 * allocation, no synchronisation), so a caller may capture them into a hipGraph.
 *
 * Activation layout ("NHWC"): an image is H*W pixels, each pixel `ld` elements apart; a tensor's
 * channels live at [c0, c0+C) of each pixel.  Images of a batch are `img_stride` elements apart and
 * a dbsr_frame_map selects which stored image a logical frame index refers to.
 *
 * Reference interfaces these replace (paths relative to the reference repo):
 *   dbsr_correlation          external/pwcnet/correlation/correlation.py:278-330 (FunctionCorrelation,
 *                             :385) incl. the leaky_relu applied by its callers, pwcnet.py:161,169
 *   dbsr_backwarp             models/alignment/pwcnet.py:16-38 (backwarp)
 *   dbsr_warp_bilinear        models/layers/warp.py:19-46 (warp), called at models/dbsr/encoders.py:80
 *   dbsr_fuse_softmax         models/dbsr/merging.py:116-126 (softmax over the burst + weighted sum)
 *   dbsr_fuse_partial/combine the same softmax-fusion split over frame-sharded ranks (log-sum-exp combine)
 *   dbsr_conv2d               nn.Conv2d (+ReLU/LeakyReLU, ResBlock residual, PixelShuffle epilogue)
 *                             as composed by models/layers/blocks.py:46-96, upsampling.py:51-58,
 *                             models/alignment/pwcnet.py:45-207, models/dbsr/{encoders,merging,decoders}.py
 *   dbsr_conv_transpose_k4s2  nn.ConvTranspose2d(k=4,s=2,p=1), pwcnet.py:119-120,166-167
 *   dbsr_pack_burst           encoders.py:52-54 (x_rgb) + pwcnet.py:262-271 (resize to a multiple of 64)
 *   dbsr_flow_finalize        pwcnet.py:274-279 (x20 bilinear upsample + rescale) + merging.py:98-105
 *                             (offsets_all = cat(0, offsets) % offset_modulo)
 *   dbsr_gauss_blur3          upsampling.py:59-65 (depthwise Gaussian, zero padding)
 *   dbsr_merge_prep           merging.py:79-89 (base_feat_proj, feat_diff_proj)
 *   dbsr_pwc_assemble         pwcnet.py:171 (cat([tenVolume, tenFirst, tenFlow, tenFeat]))
 *   dbsr_pwc_extract          pwcnet.py:45-111 (Extractor: the whole six-level feature pyramid)
 *   dbsr_pwc_level_prep       pwcnet.py:153-171 (a decoder level's ConvTs, backwarp, correlation, cat)
 */
#ifndef DBSR_HIP_H
#define DBSR_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DBSR_ABI_VERSION 22

enum { DBSR_F32 = 0, DBSR_BF16 = 1, DBSR_F16 = 2 };
enum { DBSR_ACT_NONE = 0, DBSR_ACT_RELU = 1, DBSR_ACT_LRELU = 2 };      /* LeakyReLU slope 0.1 */
enum { DBSR_OUT_NHWC = 0, DBSR_OUT_SHUFFLE = 1, DBSR_OUT_NCHW_F32 = 2 };
enum { DBSR_E_ARG = -1, DBSR_E_UNSUPPORTED = -2 };

/* logical frame f -> stored image (f / fpg) * group_stride + group_offset + (f % fpg) * inner_stride.
 * Identity: {1, 1, 0, 1}.  inner_stride 0 broadcasts one stored image to a group (e.g. every PWC
 * pair of a burst reading that burst's reference frame). */
typedef struct dbsr_frame_map {
    int fpg;
    int group_stride;
    int group_offset;
    int inner_stride;
} dbsr_frame_map;

typedef struct dbsr_tensor {          /* a channel slice of a batch of NHWC images */
    void* ptr;
    int dtype;                        /* DBSR_F32 / DBSR_BF16 / DBSR_F16 */
    long long img_stride;             /* elements between stored images */
    int ld;                           /* elements between pixels */
    int c0;                           /* first channel */
    dbsr_frame_map map;
} dbsr_tensor;

/* Implicit-GEMM convolution on MFMA.  out = post_act(act(conv(x) + bias) + residual).
 * Weights must be packed by dbsr_conv_pack_weights (dtype = x.dtype).
 * out_mode DBSR_OUT_SHUFFLE writes PixelShuffle(shuffle) of the result (the packed weights must have
 * been packed with the same shuffle factor); DBSR_OUT_NCHW_F32 writes an fp32 NCHW tensor
 * (y.img_stride = Cout*out_h*out_w, ld/c0 ignored). */
typedef struct dbsr_conv_desc {
    int n_frames;
    dbsr_tensor x;  int in_h, in_w, cin;
    const void* w;  const float* bias;  int cout, kh, kw, stride, pad, dil;
    dbsr_tensor y;  int out_h, out_w;
    int act;
    dbsr_tensor res;                  /* res.ptr == NULL: no residual */
    int post_act;
    int out_mode, shuffle;
    void* workspace;                  /* optional fp32 scratch for split-K (may be NULL) */
    size_t workspace_bytes;
    int precise;                      /* 1: bf16 activations x fp32-packed weights on fp32 MFMA (fp32 out) */
    int max_blocks;                   /* > 0: cap on the persistent kernel's workgroups (CUs it occupies),
                                         leaving the rest of the chip to concurrent streams; 0 = all CUs */
    dbsr_tensor gate;                 /* gate.ptr != NULL: out = (gate > 0) ? out : 0 after the residual --
                                         the ReLU backward of the layer that produced the conv's input
                                         (training dgrad); NHWC, output dtype; not with shuffle/NCHW out */
    int plan_h;                       /* > 0: choose the kernel, tile and K split as for an image plan_h output
                                         rows tall (0 = out_h).  A frame-sharded rank decodes a row slab of the
                                         whole image (decoders.py:54-62 run on all rows by the reference); with
                                         plan_h = the whole image's rows the slab takes exactly the whole-image
                                         plan's kernels, so its rows are bitwise the unsplit ones.  The slab's
                                         out_h must suit the chosen tile (multiples of 16 always do) */
} dbsr_conv_desc;

/* Packed weight layout: [cout_pad][kgp*8] with k-group kg = (ky*kw+kx)*(cinp/8) + c/8, where
 * cinp = cin <= 16 ? round_up(cin, 8) : round_up(cin, 32), kgp = round_up(kh*kw*cinp/8, 4),
 * cout_pad = round_up(cout, 64).  The conv reads input channels [c0, c0+cinp) of every pixel, so the
 * caller's slice must extend that far and channels [cin, cinp) must hold finite values (zeros).
 * For 3x3 convs with cin > 16 the row layout is followed (bf16 packing) by a chunk-major copy for
 * the pipelined kernel: 1-KiB pieces [cout_pad/16][cinp/32][tap][4 k-groups][16 co][8], so
 * dbsr_conv_packed_elems returns twice the row layout's size for them. */
size_t dbsr_conv_packed_elems(int cout, int cin, int kh, int kw);
/* w_f32: torch layout [cout][cin][kh][kw] fp32 (device).  bias_f32 may be NULL.  With shuffle > 1
 * the output channels are permuted for the DBSR_OUT_SHUFFLE epilogue (and bias_out likewise). */
int dbsr_conv_pack_weights(const float* w_f32, const float* bias_f32, int cout, int cin, int kh, int kw,
                           int dtype, int shuffle, void* w_packed, float* bias_out, void* stream);
/* Batched repack (ABI 22; the training step re-packs every trainable conv after each optimizer update: one launch
 * instead of dbsr_conv_pack_weights + dbsr_dgrad_weights + dbsr_conv_pack_weights per conv, ~260 launches at the
 * configs[3] shape).  A job packs one conv exactly as dbsr_conv_pack_weights(w, bias, cout, cin, kh, kw, dtype,
 * shuffle, w_packed, bias_out) would (bitwise), where for transposed = 1 the weights are the dgrad conv's taken
 * straight from the source conv's w (torch layout [cin][src_cin][kh][kw] of that conv, i.e. its cout = this job's
 * cin): this job's output channel o, input channel c, tap (ky, kx) is w[c][lo + o][kh-1-ky][kw-1-kx] -- what
 * dbsr_dgrad_weights followed by packing rows [lo, lo + cout) of its result gives (training.py: TConv.sub_dgrad).
 * blk0 is filled by dbsr_pack_batch_prepare. */
typedef struct dbsr_pack_job {
    const float* w;
    const float* bias;      /* NULL: no bias (bias_out, if set, gets zeros); ignored when transposed */
    void* w_packed;
    float* bias_out;        /* may be NULL */
    int cout, cin, kh, kw;  /* the packed conv's shape */
    int dtype, shuffle;
    int transposed, lo, src_cin;
    int pad_;
    long long blk0;         /* first 256-element block of this job in the launch (set by dbsr_pack_batch_prepare) */
} dbsr_pack_job;
/* Validates the n jobs (as dbsr_conv_pack_weights does) and fills their blk0; returns the launch's block count, or
 * -1 on a bad job (dbsr_last_error).  The caller then copies the job array to device memory once (it stays valid
 * while the weights' and outputs' addresses do) and launches it with dbsr_conv_pack_weights_batch, which is
 * graph-capturable. */
long long dbsr_pack_batch_prepare(dbsr_pack_job* jobs, int n);
int dbsr_conv_pack_weights_batch(const dbsr_pack_job* jobs_dev, int n, long long n_blocks, void* stream);
int dbsr_conv2d(const dbsr_conv_desc* d, void* stream);
/* Error-diffusion rounding of conv weights to the 16-bit dtype (ABI 19; replaces the implicit round-to-nearest of
 * the fp32 -> bf16/fp16 cast of the module's weights): w_out (fp32, torch layout [cout][cin][kh][kw], not aliasing
 * w) = per output channel, its K = kh*kw*cin weights in packed K order (tap-major, then input channel) rounded in
 * sequence with the running error carried, q_k = round(w_k - e_k), e_{k+1} = e_k + q_k - w_k.  Each value is
 * exactly representable in dtype (so dbsr_conv_pack_weights keeps it); the carried error stays within half an ulp
 * of the channel's largest weight, so each value is within one such ulp of w_k and the sum of a channel's errors
 * within half of one.  cin*kh*kw <= 10368. */
int dbsr_weights_round_diffuse(const float* w, int cout, int cin, int kh, int kw, int dtype, float* w_out,
                               void* stream);
/* Kernel selection for dbsr_conv2d (process-wide; for A/B testing): 2 (default) = pipelined
 * persistent 3x3 kernel for the large bf16 trunk convs (3x3/s1/p1/d1, cin > 16, width a multiple of
 * 48 or 64, height a multiple of 8, >= 256 tiles), else the two-barrier LDS-tiled 3x3 kernel where it
 * applies (3x3, stride 1, pad == dilation in {1,2,4,8}, cin > 16, out >= 8x8, NHWC out), else the
 * generic implicit-GEMM kernel; 1 = no pipelined kernel; 0 = generic kernel only; 3 = as 2 but the
 * pipelined kernel at any tile count (tests); 4 = as 2 without the weight-stationary kernels (both the Cin <= 64
 * one and the K-split 128-channel one); 5 = as 2 without the K-split 128-channel kernel (ABI 21).  Under 2 the
 * 16-bit 128 -> 128 3x3/s1/p1 convs of >= 128 tiles of 16 x 8 pixels (merging.py:86-90, 98-101: the weight
 * predictor's input conv and ResBlocks) run on the K-split weight-stationary kernel (kernel_for 7), which sums
 * each output as (input channels 0-63) + (64-127) in fp32, not in the pipelined kernel's order. */
int dbsr_set_conv_algo(int algo);
/* Which kernel dbsr_conv2d would launch for `d` under the current selection: 5 pointwise projection
 * (16-bit 1x1, cin 32..512 a power of two, cout 32 | 64, no residual: merging.py:34), 4 weight-stationary,
 * 3 PixelShuffle upsampler (bf16 1x1 with DBSR_OUT_SHUFFLE, 32 channels per sub-pixel), 2 pipelined,
 * 6 narrow-output 3x3 (16-bit, cout <= 4, cin >= 256, pad 1: the PWC level-2 flow head), 7 K-split
 * weight-stationary 128 -> 128 3x3 (ABI 21), 8 small-input 3x3 (16-bit, cin <= 8, cout a multiple of 16 up to 64,
 * no residual / gate: the encoder's and offset-feature extractor's first convs, ABI 21), 1 LDS-tiled, 0 generic. */
int dbsr_conv_kernel_for(const dbsr_conv_desc* d);
/* The full dispatch decision for `d`: kernel_for * 1000000 + the variant (weight-stationary: tile width*100 +
 * height; pipelined: tile config; LDS-tiled: cout tile*1000 + pixel tile; generic: cout tile*10000 + pixel
 * tile*1000 + K split; precise: pixel tile).  Two descs with equal variants sum every output in the same
 * order (the frame-sharding tests compare a slab's variants with the whole image's). */
int dbsr_conv_dispatch_variant(const dbsr_conv_desc* d);
/* Host model of the highest channel of a pixel (c0 included) that any lane of the kernel dbsr_conv2d would
 * launch for `d` touches in y (which 0: stores), the residual (1) or the gate (2) -- including the lanes of a
 * partial cout tile past cout, which the pipelined and weight-stationary kernels point at their tile's first
 * run; -1 when that tensor is unused or y is not NHWC; -2 on a bad argument.  dbsr_conv2d returns DBSR_E_ARG
 * when it is >= the tensor's ld (a run past the last pixel of the last frame would leave the allocation). */
int dbsr_conv_lane_reach(const dbsr_conv_desc* d, int which);
/* A 32-channel ResBlock conv2 fused with a 1x1 head (the decoder's last post-ResBlock + RGB predictor,
 * decoders.py:59-61 / blocks.py:94-96): t = ReLU(conv(x) + bias + residual) stays in registers (d->y is
 * not written) and out = ReLU(head_w . t + head_b) is stored fp32 NCHW (head_out.img_stride =
 * head_cout*out_h*out_w).  head_w: fp32 [head_cout][32] (the torch [head_cout][32][1][1] weight),
 * head_b: fp32 [head_cout] or NULL, head_cout 1..4.  Requires dbsr_conv_head_ok(d). */
int dbsr_conv2d_head(const dbsr_conv_desc* d, const float* head_w, const float* head_b, int head_cout,
                     dbsr_tensor head_out, void* stream);
/* PixelShuffle upsampler + Gaussian blur in one launch (ABI 16; upsampling.py:51-66, replaces the pair
 * dbsr_conv2d(d) -> dbsr_gauss_blur3 of decoders.py:57's upsample_layer): y = blur3(PixelShuffle(act(conv1x1(x)
 * + bias))), k9 = the 3x3 blur kernel (host, row-major; separable, as the reference's Gaussian is, else
 * DBSR_E_ARG), zero padding at the output frame's borders.  `d`
 * describes the upsampling conv as for dbsr_conv2d (out_mode DBSR_OUT_SHUFFLE, weights packed with shuffle);
 * y receives the blurred output.  Bitwise equal to the two-call path.  Requires dbsr_conv_shuffle_blur_ok(d):
 * 16-bit, 1x1 conv cin <= 64 -> 2048 (32 channels x PixelShuffle(8)), low-res frame a multiple of 4 x 4,
 * NHWC slices aligned to 8 channels. */
int dbsr_conv_shuffle_blur(const dbsr_conv_desc* d, const float* k9, void* stream);
int dbsr_conv_shuffle_blur_ok(const dbsr_conv_desc* d);
/* A whole ResBlock in one launch (ABI 17; blocks.py:81-96, replaces the pair of dbsr_conv2d calls of a decoder
 * post-ResBlock, decoders.py:46-49, or -- 64 channels -- of a decoder pre-ResBlock, decoders.py:41-44): y = relu(x + conv2(relu(conv1(x)))).  c1 = conv1 as for dbsr_conv2d
 * (x -> its y, act ReLU), c2 = conv2 (its x, y, residual = c1's input, act none, post-act ReLU); c1->y and c2->x
 * name the intermediate, which this call neither reads nor writes (it stays on chip).  Bitwise equal to the two
 * calls.  Requires dbsr_resblock_ok(c1, c2): 16-bit 3x3/s1/p1 convs C -> C, C = 32 (frames a multiple of 32 x 16)
 * or C = 64 (ABI 19; frames a multiple of 16 x 8, at most 2 tiles of 16 x 8 per CU -- the decoder's pre-ResBlocks;
 * at the encoder's 2016 tiles the two weight-stationary launches measured faster), NHWC slices aligned to 8
 * channels, and y not overlapping x (blocks read neighbouring tiles' halos of x while others store y: an in-place
 * call is refused with DBSR_E_ARG); c1->max_blocks caps the persistent grid. */
int dbsr_resblock(const dbsr_conv_desc* c1, const dbsr_conv_desc* c2, void* stream);
int dbsr_resblock_ok(const dbsr_conv_desc* c1, const dbsr_conv_desc* c2);
/* dbsr_resblock with the decoder's RGB predictor fused (ABI 18; decoders.py:59-61, the last post-ResBlock + the
 * 1x1 32 -> head_cout conv + ReLU, as dbsr_conv2d_head computes it): the block's fp32 output stays in registers
 * and out = ReLU(head_w . t + head_b) is stored fp32 NCHW (head_out.img_stride = head_cout*h*w); c2->y is not
 * written.  head_w fp32 [head_cout][32], head_b [head_cout] or NULL, head_cout 1..4; requires dbsr_resblock_ok. */
int dbsr_resblock_head(const dbsr_conv_desc* c1, const dbsr_conv_desc* c2, const float* head_w, const float* head_b,
                       int head_cout, dbsr_tensor head_out, void* stream);
/* 1 when dbsr_conv2d_head accepts `d`: pipelined shape (16-bit 3x3/s1/p1, width % 64 == 0, height % 8 == 0,
 * >= 256 tiles), cout == 32, residual, act none, post-act ReLU.  (The engine prefers dbsr_resblock_head, the whole
 * last post-ResBlock + head in one launch, where dbsr_resblock_ok serves the shape.) */
int dbsr_conv_head_ok(const dbsr_conv_desc* d);
/* Scratch bytes dbsr_conv2d would use for split-K on `d` (0 = no split).  Convs whose grid cannot fill
 * the chip split K into slices that store fp32 partials to `workspace`; a second launch sums them in
 * slice order (deterministic) and applies the epilogue.  With a smaller/NULL workspace the conv simply
 * runs unsplit.  One workspace may be shared by all convs issued on one stream. */
size_t dbsr_conv_workspace_bytes(const dbsr_conv_desc* d);

/* 81-channel cost volume of (first, second) over displacements [-4,4]^2, divided by C, followed by
 * LeakyReLU(0.1) when leaky != 0.  first/second/out: NHWC slices; out channel (dy+4)*9+(dx+4). */
int dbsr_correlation(int n_pairs, int h, int w, int c, dbsr_tensor first, dbsr_tensor second,
                     dbsr_tensor out, int leaky, void* stream);

/* Backward of dbsr_correlation (correlation.py:105-233, K3/K4) w.r.t. both inputs: gout = dL/d(out),
 * out = the forward output (read only when leaky != 0, for the LeakyReLU slope). */
int dbsr_correlation_backward(int n_pairs, int h, int w, int c, dbsr_tensor first, dbsr_tensor second,
                              dbsr_tensor out, dbsr_tensor gout, int leaky, dbsr_tensor dfirst, dbsr_tensor dsecond,
                              void* stream);

/* PWC-Net backwarp of `in` (C channels) by flow*scale (flow: NHWC fp32 slice with 2 channels),
 * bilinear, zero padding, validity mask (weight mass > 0.999). */
int dbsr_backwarp(int n, int h, int w, int c, dbsr_tensor in, dbsr_tensor flow, float scale,
                  dbsr_tensor out, void* stream);

/* DBSR warp: bilinear sample of feat at (x + fx, y + fy), zero padding.  flow: fp32 NCHW
 * [n][2][h][w] (the `offsets` tensor), flow_img_stride elements per image. */
int dbsr_warp_bilinear(int n, int h, int w, int c, dbsr_tensor feat, const float* flow,
                       long long flow_img_stride, dbsr_tensor out, void* stream);
/* dbsr_warp_bilinear fused with the 1x1 feature projection of the warped frames (ABI 20; encoders.py:80 then
 * merging.py:34-36,75 on the warped embeddings): out = warp(feat) exactly as dbsr_warp_bilinear stores it, and
 * proj_out = ReLU(proj_w . out + proj_b) computed from those stored 16-bit values (fp32 accumulation; equal to
 * dbsr_conv2d of the 1x1 conv on `out` up to the K summation order).  c == 512, 16-bit feat / out / proj_out of one
 * dtype; proj_w = the 1x1 conv's weights packed by dbsr_conv_pack_weights (cin 512), proj_b fp32 or NULL,
 * proj_cout 16 / 32 / 48 / 64; proj_out image f of the n warped frames, channels [c0, c0 + proj_cout). */
int dbsr_warp_project(int n, int h, int w, int c, dbsr_tensor feat, const float* flow, long long flow_img_stride,
                      dbsr_tensor out, const void* proj_w, const float* proj_b, int proj_cout, dbsr_tensor proj_out,
                      void* stream);

/* Softmax over the burst of logits[b,n] and weighted sum of feats[b,n].  Frame (b,n): logits image
 * b*N+n; feature image: n==0 -> ref (map applied to b), n>0 -> oth (map applied to b*(N-1)+n-1).
 * weights (optional, ptr NULL to skip): NHWC images b*N+n.  fused: NHWC images b. */
int dbsr_fuse_softmax(int B, int N, int hw, int c, dbsr_tensor logits, dbsr_tensor ref, dbsr_tensor oth,
                      dbsr_tensor fused, dbsr_tensor weights, void* stream);

/* WeightedSum with softmax=False (ABI 20; merging.py:117-121): weights = relu(logits) / (sum over the burst of
 * relu(logits) + 1e-12), fused = sum_n weights * features; arguments and addressing as dbsr_fuse_softmax. */
int dbsr_fuse_relu_norm(int B, int N, int hw, int c, dbsr_tensor logits, dbsr_tensor ref, dbsr_tensor oth,
                        dbsr_tensor fused, dbsr_tensor weights, void* stream);
/* The burst mean of per-frame NHWC maps (ABI 20; merging.py:81-82, use_base_frame=False: the mean projected
 * embedding as the base): out image b = (sum_n in image b*N+n) / N over c channels (fp32 sum, n in order). */
int dbsr_burst_mean(int B, int N, int hw, int c, dbsr_tensor in, dbsr_tensor out, void* stream);

/* The weight predictor's last conv fused with the softmax over the burst and the weighted sum
 * (models/dbsr/merging.py:55-57,113-124): logits = conv(d) + bias for the B*N frames
 * of d->x (frame b*N+n of burst b) never reach memory and are never rounded -- each (burst, 16x2 pixels,
 * 128 channels) super-tile keeps all N frames' fp32 logits in its waves' accumulators; weights = softmax over
 * the N frames (fp32, stored in the conv dtype), fused = sum_n weights * features (fp32, stored in the dtype).
 * ref / oth / fused / weights address as in dbsr_fuse_softmax (c = d->cout; weights.ptr NULL: no aux output);
 * d->y, d->res are unused; d->max_blocks caps the persistent grid (rounded down to a multiple of 8, at least 8).  Requires dbsr_conv_fuse_ok(d, B, N):
 * 16-bit 3x3/s1/p1/d1, cin > 16, cout % 128 == 0 (<= 512), d->n_frames == B*N, N == 14, width % 16 == 0,
 * height % 2 == 0, and frame maps affine in (burst, frame); the feature / output tensors need ld and c0
 * multiples of 8 with c0 + cout <= ld (DBSR_E_ARG otherwise). */
int dbsr_conv_fuse_softmax(const dbsr_conv_desc* d, int B, int N, dbsr_tensor ref, dbsr_tensor oth,
                           dbsr_tensor fused, dbsr_tensor weights, void* stream);
/* As dbsr_conv_fuse_softmax with the ReLU normalisation of WeightedSum(softmax=False) (ABI 20; merging.py:119-121):
 * weights = relu(logits) / (sum over the burst of relu(logits) + 1e-12), the fp32 logits never rounded. */
int dbsr_conv_fuse_relu_norm(const dbsr_conv_desc* d, int B, int N, dbsr_tensor ref, dbsr_tensor oth,
                             dbsr_tensor fused, dbsr_tensor weights, void* stream);
int dbsr_conv_fuse_ok(const dbsr_conv_desc* d, int B, int N);

/* Frame-sharded fusion (the softmax over the burst of models/dbsr/merging.py:116-124
 * split over ranks holding disjoint frame subsets).  dbsr_fuse_partial: statistics of the local frames
 * n in [first_frame, N) (same logits/ref/oth addressing as dbsr_fuse_softmax) into stats, fp32
 * [B][hw][3c] = (m = max_n l | s = sum e^(l-m) | a = sum e^(l-m) f).  dbsr_fuse_combine: R such blocks
 * laid out back to back (an all-gather of the ranks' stats) -> fused = sum_r a_r e^(m_r-M) /
 * sum_r s_r e^(m_r-M), M = max_r m_r; equal to the unsharded fusion up to fp32 rounding order. */
int dbsr_fuse_partial(int B, int N, int hw, int c, int first_frame, dbsr_tensor logits, dbsr_tensor ref,
                      dbsr_tensor oth, float* stats, void* stream);
int dbsr_fuse_combine(int R, int B, int hw, int c, const float* stats, dbsr_tensor fused, void* stream);

/* ConvTranspose2d(cin -> cout<=4, k=4, s=2, p=1): in NHWC slice [n][h][w], out NHWC fp32 [n][2h][2w].
 * w: fp32 repacked as [ky][kx][cout][cin8] (torch's [cin][cout][4][4] permuted, channels zero-padded
 * to cin8 = round_up(cin, 8)); bias [cout] fp32.  Reads input channels [c0, c0+cin8). */
int dbsr_conv_transpose_k4s2(int n, int h, int w, int cin, int cout, dbsr_tensor in, const float* wgt,
                             const float* bias, dbsr_tensor out, void* stream);

/* burst [B][N][4][H][W] fp32 (NCHW frames) -> raw: NHWC 4-channel slice (frames b*N+n);
 * rgb: NHWC 3-channel slice [B*N][Hp][Wp] = bilinear(align_corners=False) resize of (R,(G1+G2)/2,B). */
int dbsr_pack_burst(int B, int N, int H, int W, const float* burst, dbsr_tensor raw, int Hp, int Wp,
                    dbsr_tensor rgb, void* stream);

/* flow: NHWC fp32 2-ch slice [P][hf][wf] (P = B*(N-1) pairs).  offsets: fp32 NCHW [P][2][H][W] =
 * 20*bilinear(flow -> H x W) * (W/Wp, H/Hp).  offs_mod (optional): NHWC 2-ch slice, images b*N+n,
 * = offsets % modulo (torch.remainder) with zeros for n == 0 (merging.py:98-105); modulo 0 = offset_modulo None
 * (the offsets themselves). */
int dbsr_flow_finalize(int B, int N, int hf, int wf, dbsr_tensor flow, int H, int W, int Hp, int Wp,
                       float* offsets, float modulo, dbsr_tensor offs_mod, void* stream);

/* Depthwise 3x3 filter with zero padding on an NHWC slice of C channels. k: 9 floats (host). */
int dbsr_gauss_blur3(int n, int h, int w, int c, dbsr_tensor in, const float* k_host, dbsr_tensor out,
                     void* stream);

/* proj: NHWC images b*N+n (C channels).  out: [base = proj[b,0] | diff = proj[b,n]-proj[b,0]]
 * written at out.c0 .. out.c0+2C. */
int dbsr_merge_prep(int B, int N, int hw, int c, dbsr_tensor proj, dbsr_tensor out, void* stream);

/* cat([vol(81, already in place), first(C), flow(2), feat(2)]) for PWC decoder level inputs:
 * writes first/flow/feat into out channels [c0+81, c0+81+C+4). first: map pair->ref frame. */
int dbsr_pwc_assemble(int n_pairs, int h, int w, int c, dbsr_tensor first, dbsr_tensor flow,
                      dbsr_tensor feat, dbsr_tensor out, void* stream);

/* Fused PWC decoder DenseNet of one coarse level (pwcnet.py:153-184, levels with <= 64 pixels per
 * pair): the five LeakyReLU dense convs and the flow conv over D [P][h][w][ld] (16-bit; base channels
 * already assembled), dense outputs written into D's channels [0, dense_ch), flow (fp32, 2 ch) to flow.
 * convs[0..4]: dense, convs[5]: flow; weights packed by dbsr_conv_pack_weights (3x3, cin > 16). */
typedef struct {
    const void* w;
    const float* bias;
    int kp, cg;          /* packed K (= 9 * cg * 8) and 8-channel input groups per tap (cg % 4 == 0) */
    int start;           /* first input channel in D */
    int cout, out_off;   /* output channels, their offset in D (ignored for the flow conv) */
} dbsr_pwc_dense_conv;
int dbsr_pwc_dense(int P, int h, int w, dbsr_tensor D, int dense_ch, const dbsr_pwc_dense_conv* convs,
                   dbsr_tensor flow, void* stream);
/* 1 if dbsr_pwc_dense has an LDS tile for an h x w level with ld channels in D (else use dbsr_conv2d). */
int dbsr_pwc_dense_supported(int h, int w, int ld);

/* The PWC-Net feature pyramid (Extractor.forward, pwcnet.py:103-111) of F 64x64 frames in one launch:
 * convs[3l + j] = level l+1's conv j (j = 0: 3x3 stride 2, j = 1, 2: 3x3 stride 1), channels 3 -> 16 -> 32 ->
 * 64 -> 96 -> 128 -> 196, each + bias + LeakyReLU(0.1); weights packed by dbsr_conv_pack_weights (16-bit).
 * rgb: the 8-channel packed frames [F][64][64] (dbsr_pack_burst); levels[l]: NHWC [F][64 >> (l+1)]^2 with
 * ld = the padded width (16, 32, 64, 96, 128, 224), written in full (pad channels as zeros).
 * Requires dbsr_pwc_extract_supported(Hp, Wp) (Hp = Wp = 64) and 16-bit activations. */
typedef struct {
    const void* w;
    const float* bias;
    int cin, cout, stride;
} dbsr_pwc_ext_conv;
int dbsr_pwc_extract(int F, int Hp, int Wp, dbsr_tensor rgb, const dbsr_pwc_ext_conv* convs,
                     const dbsr_tensor* levels, void* stream);
int dbsr_pwc_extract_supported(int Hp, int Wp);
/* One PWC decoder level's input (Decoder.forward, pwcnet.py:153-171) in one launch, per pair p:
 * upflow = ConvT(prev_flow), upfeat = ConvT(prev_D channels [0, prev_cin)) (k4 s2 p1; w_upflow as for
 * dbsr_conv_transpose_k4s2, fp32 [4][4][2][8]; w_upfeat 16-bit (D's dtype) [4][4][2][round_up(prev_cin, 32)],
 * i.e. rows (ky*4+kx)*2+co, zero-padded channels), warped = backwarp(second, upflow * scale) (dbsr_backwarp),
 * D[c0 + 0..80] = LeakyReLU(correlation(first, warped)) (dbsr_correlation), D[c0 + 81 ..] = [first | upflow |
 * upfeat] (dbsr_pwc_assemble).  prev_D.ptr == NULL: the coarsest level (no warp, correlation only).  first /
 * second: 16-bit level features (c0 0, ld >= the padded width) with pair -> frame maps; D: 16-bit, c0 = the
 * base channels.  Requires dbsr_pwc_level_prep_supported(h, w, c) (the level fits one block's LDS). */
int dbsr_pwc_level_prep(int P, int h, int w, int c, float scale, dbsr_tensor first, dbsr_tensor second, dbsr_tensor D,
                        dbsr_tensor prev_D, int prev_cin, dbsr_tensor prev_flow, const float* w_upflow,
                        const float* b_upflow, const void* w_upfeat, const float* b_upfeat, void* stream);
int dbsr_pwc_level_prep_supported(int h, int w, int c);

/* ---------------- BurstSR scoring: SpatialColorAlignment (spatial_color_alignment.py:23-108) ----------------
 * fp32 NCHW planes.  rh / rw are PyTorch's internal source-coordinate ratios, 1 / scale_factor. */
/* F.interpolate(bilinear, align_corners=False, scale_factor) of `planes` planes, times mul
 * (spatial_color_alignment.py:96-101: flow_ds = interpolate(flow, 1/8) * 1/8, frame_gt_ds). */
int dbsr_resize_bilinear(int planes, int ih, int iw, const float* in, int oh, int ow, float rh, float rw, float mul,
                         float* out, void* stream);
/* apply_kernel (filtering.py:56-63): reflect padding + ksz x ksz filter (k_host: ksz*ksz floats, ksz odd <= 9). */
int dbsr_gauss_reflect(int planes, int h, int w, int ksz, const float* k_host, const float* in, float* out,
                       void* stream);
/* match_colors' least squares (spatial_color_alignment.py:36-44): per image, C[3][3] minimising
 * ||Q C - R|| over the [bi, h-bi) x [bi, w-bi) crop of the smoothed images ref (R) and q (Q). */
int dbsr_color_fit(int n, int h, int w, int bi, const float* ref, const float* q, float* c_mat, void* stream);
/* match_colors' transform + validity mask (spatial_color_alignment.py:45-67): out = test^T C per pixel,
 * valid (uint8) = bilinear-upsampled (err < thresh on the crop, 0 in the bi border) > 0.9. */
int dbsr_color_apply(int n, int h, int w, int bi, const float* ref, const float* q, const float* c_mat, float thresh,
                     const float* test, int oh, int ow, float rh, float rw, float* out, unsigned char* valid,
                     void* stream);

/* ---------------- training step (BASELINE configs[3]; trainers/simple_trainer.py:78-81) ----------------
 * Backward of the DBSR part (PWC-Net is frozen, encoders.py:56-61).  Conv dgrad = dbsr_conv2d with the
 * weights of dbsr_dgrad_weights (W'[ci][co][ky][kx] = W[co][ci][kh-1-ky][kw-1-kx]) packed as a normal
 * conv, and the gate / residual epilogue for the ReLU / ResBlock backward (blocks.py:81-96). */

/* Conv weight gradient, k = 1 or 3 (stride 1, pad k/2): dw[co][ci][ky][kx] (fp32, torch layout) =
 * sum_p dy[p][co] * x[p + (ky-1, kx-1)][ci]; accumulate != 0 adds to dw.  x / dy: NHWC slices of the
 * same dtype (cin / cout channels, ld and c0 multiples of 16 B, channels up to the next 16 B finite).
 * Deterministic: fp32 partials per block (workspace) summed in a fixed order. */
size_t dbsr_conv_wgrad_workspace_bytes(int n_frames, int h, int w, int cin, int cout, int k);
int dbsr_conv_wgrad(int n_frames, int h, int w, dbsr_tensor x, int cin, dbsr_tensor dy, int cout, int k,
                    float* dw, int accumulate, void* workspace, size_t workspace_bytes, void* stream);
/* dbsr_conv_wgrad plus the conv's bias gradient in the same pass over dy (ABI 14): db[co] (+)= sum_p dy[p][co]
 * (fp32 [cout], deterministic; db NULL = none).  Replaces the weight and bias halves of nn.Conv2d's backward
 * (torch.nn.grad.conv2d_weight + grad_output.sum((0, 2, 3)), which the reference's training step gets from
 * autograd: actors/dbsr_actors.py:27-47).  Same workspace as dbsr_conv_wgrad. */
/* Which wgrad kernel 16-bit dbsr_conv_wgrad(_bias) runs: 1 (default) the LDS-DMA ring kernel, 0 the register-
 * staged one (fp32 always runs the latter).  Both sum dw in the same order (bitwise equal); db is equal up to
 * fp32 summation order (the ring kernel sums it from the dY fragments of its tap-5 wave). */
int dbsr_set_wgrad_algo(int algo);
int dbsr_conv_wgrad_bias(int n_frames, int h, int w, dbsr_tensor x, int cin, dbsr_tensor dy, int cout, int k,
                         float* dw, float* db, int accumulate, void* workspace, size_t workspace_bytes, void* stream);
/* The decoder's RGB predictor as the training step runs it (ABI 14; decoders.py:61, a 1x1 conv 32 -> hc plus
 * ReLU, kept apart from the last post-ResBlock conv because the backward needs that conv's output h):
 *   dbsr_head_forward:  out (fp32 NCHW [n][hc][hw]) = ReLU(w . h + b); w fp32 [hc][cin] (torch layout), b
 *                       fp32 [hc] or NULL.
 *   dbsr_head_backward: dh = [h > 0] * (w^T . dp) (the predictor's dgrad gated by h's ReLU), dw[c][i] (+)=
 *                       sum_p dp[p][c] h[p][i], db[c] (+)= sum_p dp[p][c] (db NULL = none); deterministic.
 * h / dh: NHWC (cin == 32, ld/c0 multiples of 16 B); dp: NHWC with 8 readable channels (hc used), as
 * dbsr_l1_loss_backward writes it.  hc 1..4.  Replace nn.Conv2d(32, 3, 1)'s forward and autograd backward in
 * the reference's training step (actors/dbsr_actors.py:27-47). */
int dbsr_head_forward(int n, int hw, dbsr_tensor h, int cin, const float* w, const float* b, int hc, float* out,
                      void* stream);
size_t dbsr_head_backward_workspace_bytes(int n, int hw, int cin, int hc);
int dbsr_head_backward(int n, int hw, dbsr_tensor h, int cin, dbsr_tensor dp, const float* w, int hc, dbsr_tensor dh,
                       float* dw, float* db, int accumulate, void* workspace, size_t workspace_bytes, void* stream);
/* out[c] (+)= sum over the n*hw pixels of t[.][c] (conv bias gradient), fp32; deterministic. */
size_t dbsr_chan_sum_workspace_bytes(int n, int hw, int c);
int dbsr_chan_sum(int n, int hw, int c, dbsr_tensor t, float* out, int accumulate, void* workspace,
                  size_t workspace_bytes, void* stream);
/* L1 loss of pred vs gt (fp32 NCHW [B][C][H][W]) with boundary_ignore (image_quality_v2.py:24-66) into
 * *loss (device), and its gradient through the predictor ReLU: dpre (NHWC, C channels) = [pred > 0] *
 * sign(pred - gt) / count inside the crop, 0 outside.  workspace: >= ceil(B*H*W/256) floats. */
int dbsr_l1_loss_backward(int B, int C, int H, int W, int boundary_ignore, const float* pred, const float* gt,
                          dbsr_tensor dpre, float* loss, void* workspace, size_t workspace_bytes, void* stream);
/* The RGB predictor's ReLU backward from an upstream gradient (autograd through DBSRNet.forward with any
 * objective): dpre (NHWC, C channels, compute dtype) = [pred > 0] * gout; pred / gout fp32 NCHW [B][C][H][W]. */
int dbsr_relu_grad(int B, int C, int H, int W, const float* pred, const float* gout, dbsr_tensor dpre, void* stream);
/* PixelShuffle(s) + ReLU backward (upsampling.py:51-58): du[b][y][x][c*s*s + i*s + j] =
 * ds[b][y*s+i][x*s+j][c] * [gate > 0] (gate = the upsampler's forward output). */
int dbsr_unshuffle_gate(int B, int H, int W, int s, int c, dbsr_tensor ds, dbsr_tensor gate, dbsr_tensor du,
                        void* stream);
/* Softmax-fusion backward (merging.py:116-124), addressing as dbsr_fuse_softmax: dref / doth = w * dfused,
 * dlogits = w * dfused * (f - fused); weights = the forward's normalised weights. */
int dbsr_fuse_backward(int B, int N, int hw, int c, dbsr_tensor weights, dbsr_tensor ref, dbsr_tensor oth,
                       dbsr_tensor fused, dbsr_tensor dfused, dbsr_tensor dlogits, dbsr_tensor dref,
                       dbsr_tensor doth, void* stream);
/* merge-prep backward (merging.py:79-89) + the projection ReLU: dwp channels [0,c) = d base, [c,2c) = d diff
 * of images b*N+n -> dproj = [proj > 0] * (n == 0 ? sum_n dbase - sum_{n>=1} ddiff : ddiff). */
int dbsr_merge_prep_backward(int B, int N, int hw, int c, dbsr_tensor dwp, dbsr_tensor proj, dbsr_tensor dproj,
                             void* stream);
/* warp backward w.r.t. the features (warp.py:19-46): dfeat32[fmap(p)] += bilinear scatter of dout[p]
 * (fp32 atomics; dfeat32 images dfeat_img_stride floats apart, pixels c floats apart). */
int dbsr_warp_backward(int n, int h, int w, int c, dbsr_tensor dout, const float* flow, long long flow_img_stride,
                       float* dfeat32, dbsr_frame_map fmap, long long dfeat_img_stride, void* stream);
/* encoder output gradient (encoders.py:66-80): de[b*N+n] = [e > 0] * (n == 0 ? dref[b] : dsrc32[b*N+n]). */
int dbsr_enc_grad_gate(int B, int N, int hw, int c, dbsr_tensor dref, const float* dsrc32, dbsr_tensor e,
                       dbsr_tensor de, void* stream);
/* warp backward w.r.t. the features (warp.py:19-46) as an owner-computes gather, replacing the atomics of
 * dbsr_warp_backward: dfeat[p] = [gate[p] > 0] * (bilinear-transpose of dout[p]) (gate.ptr NULL: no gate),
 * written whole (no accumulation, no fp32 scratch); c channels (c, ld, c0 multiples of 8), dout / gate / dfeat
 * of one dtype.  The contributions are binned per destination pixel by a counting sort in `workspace` (any
 * flow field); each pixel's fp32 sum runs in record order, which follows the binning's atomics. */
size_t dbsr_warp_backward_gather_workspace_bytes(int n, int h, int w);
int dbsr_warp_backward_gather(int n, int h, int w, int c, dbsr_tensor dout, const float* flow,
                              long long flow_img_stride, dbsr_tensor gate, dbsr_tensor dfeat, void* workspace,
                              size_t workspace_bytes, void* stream);
/* out = [gate > 0] * in over n NHWC images of c channels (c, ld, c0 multiples of 8). */
int dbsr_gate_copy(int n, int hw, int c, dbsr_tensor in, dbsr_tensor gate, dbsr_tensor out, void* stream);
/* torch.optim.Adam step (weight_decay 0) on flat fp32 buffers; grad is scaled by grad_scale first. */
int dbsr_adam_step(long long n, float* param, const float* grad, float* exp_avg, float* exp_avg_sq, float lr,
                   float beta1, float beta2, float eps, int step, float grad_scale, void* stream);
/* wt[ci][co][ky][kx] = w[co][ci][kh-1-ky][kw-1-kx] (fp32): the dgrad conv's weights, to pack with
 * dbsr_conv_pack_weights(cout = cin, cin = cout). */
int dbsr_dgrad_weights(const float* w, int cout, int cin, int kh, int kw, float* wt, void* stream);

/* n NHWC images (c channels from in.c0, any dtype) -> fp32 NCHW out [n][c][hw]: the fusion weights in the
 * reference's [B,N,C,H,W] fp32 layout (merging.py:117-126), materialised when a caller reads them. */
int dbsr_nhwc_to_nchw_f32(int n, int hw, int c, dbsr_tensor in, float* out, void* stream);

/* Fill an NHWC slice with zeros (used for channel padding of persistent buffers). */
int dbsr_zero(void* ptr, size_t bytes, void* stream);

const char* dbsr_last_error(void);
int dbsr_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif
