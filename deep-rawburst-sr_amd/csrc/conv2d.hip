// Implicit-GEMM 2-D convolution on gfx950 MFMA, NHWC activations.
//
// GEMM view: D[cout][pixel] = sum_k W[cout][k] * X[k][pixel], k = (tap, input channel).
// One MFMA 16x16x32 k-step covers four "k-groups" of 8 consecutive channels of one tap each;
// lane l supplies k-group (l>>4) for row/column (l&15):
//   A (weights):  8 contiguous packed values of cout row (l&15)      -> one 16-B (bf16) load
//   B (pixels):   8 contiguous channels of pixel (l&15) at that tap  -> one 16-B (bf16) load
// and the accumulator gives lane l four consecutive output channels of one pixel, which the
// epilogue stores as one 8-B (bf16) / 16-B (fp32) NHWC store.  fp32 mode runs the same data flow on
// v_mfma_f32_16x16x4_f32 (8 MFMAs per k-step, element j of each lane's 8-vector in MFMA j), which
// is an exact fp32 FMA chain (cdna_hip_programming.md §3 'FP32-input MFMA').
//
// Block = 4 waves; every wave owns all MT*16 output channels of the block and NT*16 pixels, so the
// block shares its weight rows (L1-resident) and each wave gathers its own pixels.  Arbitrary
// stride / dilation / padding / Cin (multiple-of-8 pixel stride) are handled per lane, so the one
// kernel serves every conv of the path: ResNet 3x3, 1x1 projections, strided PWC extractor,
// dilated refiner, the DenseNet decoder (channel-slice reads/writes into one buffer: no cat), the
// ResBlock residual (+ReLU) and the PixelShuffle epilogue of the decoder upsampler.
#include "common.hpp"

using namespace dbsr;

namespace {

struct ConvK {
    const void* x; long long x_is; int x_ld; dbsr_frame_map xm; int in_h, in_w;
    const void* w; const float* bias; int Kp, KG, KGp, CG, kw, stride, pad, dil, cout;
    void* y; int y_f32; long long y_is; int y_ld, y_c0; dbsr_frame_map ym; int out_h, out_w;
    int act;
    const void* r; long long r_is; int r_ld, r_c0; dbsr_frame_map rm; int post_act;
    int out_mode, shuffle, cps;
    int npix;
    int vec_store;
};

template <typename T> struct Frag;
template <> struct Frag<bf16_t> {
    bf16x8_t v;
    __device__ __forceinline__ void load(const bf16_t* p) { v = *(const bf16x8_t*)p; }
    __device__ __forceinline__ void zero() { v = bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0}; }
};
template <> struct Frag<float> {
    float4 a, b;
    __device__ __forceinline__ void load(const float* p) { a = *(const float4*)p; b = *(const float4*)(p + 4); }
    __device__ __forceinline__ void zero() { a = make_float4(0, 0, 0, 0); b = a; }
};

__device__ __forceinline__ f32x4_t mma(const Frag<bf16_t>& A, const Frag<bf16_t>& B, f32x4_t c) {
    typedef __attribute__((ext_vector_type(8))) __bf16 bfv;
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bfv, A.v), __builtin_bit_cast(bfv, B.v), c,
                                                   0, 0, 0);
}
__device__ __forceinline__ f32x4_t mma(const Frag<float>& A, const Frag<float>& B, f32x4_t c) {
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(A.a.x, B.a.x, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(A.a.y, B.a.y, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(A.a.z, B.a.z, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(A.a.w, B.a.w, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(A.b.x, B.b.x, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(A.b.y, B.b.y, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(A.b.z, B.b.z, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(A.b.w, B.b.w, c, 0, 0, 0);
    return c;
}

template <typename T>
__device__ __forceinline__ void store4(const ConvK& k, long long off, const float (&v)[4], int nvalid) {
    if (k.y_f32) {
        float* y = (float*)k.y + off;
        if (nvalid == 4 && k.vec_store) {
            *(float4*)y = make_float4(v[0], v[1], v[2], v[3]);
        } else {
            for (int r = 0; r < nvalid; ++r) y[r] = v[r];
        }
    } else {
        T* y = (T*)k.y + off;
        if (nvalid == 4 && k.vec_store) {
            if constexpr (sizeof(T) == 2) {
                uint2 q;
                q.x = (unsigned)f2bf(v[0]) | ((unsigned)f2bf(v[1]) << 16);
                q.y = (unsigned)f2bf(v[2]) | ((unsigned)f2bf(v[3]) << 16);
                *(uint2*)y = q;
            } else {
                *(float4*)y = make_float4(v[0], v[1], v[2], v[3]);
            }
        } else {
            for (int r = 0; r < nvalid; ++r) elem<T>::st(y + r, v[r]);
        }
    }
}

template <typename T, int MT, int NT>
__global__ __launch_bounds__(256) void conv2d_kernel(ConvK k) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int kgl = lane >> 4, col = lane & 15;
    const int hw = k.out_h * k.out_w;
    const int p_base = blockIdx.x * (4 * NT * 16) + wave * (NT * 16);
    const int c_base = blockIdx.y * (MT * 16);

    const T* xb[NT];
    int iy0[NT], ix0[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const int p = p_base + j * 16 + col;
        if (p < k.npix) {
            const int f = p / hw, rr = p - f * hw;
            const int oy = rr / k.out_w, ox = rr - oy * k.out_w;
            xb[j] = (const T*)k.x + map_frame(k.xm, f) * k.x_is;
            iy0[j] = oy * k.stride - k.pad;
            ix0[j] = ox * k.stride - k.pad;
        } else {
            xb[j] = (const T*)k.x;
            iy0[j] = -(1 << 28);
            ix0[j] = 0;
        }
    }
    const T* wr[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) wr[i] = (const T*)k.w + (long long)(c_base + i * 16 + col) * k.Kp + kgl * 8;

    f32x4_t acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    // k-group decode for this lane, advanced incrementally by 4 per k-step
    int tap = kgl / k.CG;
    int cg = kgl - tap * k.CG;
    int ky = tap / k.kw, kx = tap - (tap / k.kw) * k.kw;
    const int nks = k.KGp >> 2;
    for (int ks = 0; ks < nks; ++ks) {
        const bool kval = ks * 4 + kgl < k.KG;
        Frag<T> a[MT], b[NT];
#pragma unroll
        for (int i = 0; i < MT; ++i) a[i].load(wr[i] + ks * 32);
        const int dy = ky * k.dil, dx = kx * k.dil;
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            const int iy = iy0[j] + dy, ix = ix0[j] + dx;
            if (kval && (unsigned)iy < (unsigned)k.in_h && (unsigned)ix < (unsigned)k.in_w)
                b[j].load(xb[j] + ((long long)iy * k.in_w + ix) * k.x_ld + cg * 8);
            else
                b[j].zero();
        }
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int j = 0; j < NT; ++j) acc[i][j] = mma(a[i], b[j], acc[i][j]);
        cg += 4;
        while (cg >= k.CG) {
            cg -= k.CG;
            if (++kx == k.kw) { kx = 0; ++ky; }
        }
    }

    // epilogue: bias, activation, residual, post-activation, store
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const int p = p_base + j * 16 + col;
        if (p >= k.npix) continue;
        const int f = p / hw, rr = p - f * hw;
        const int oy = rr / k.out_w, ox = rr - oy * k.out_w;
#pragma unroll
        for (int i = 0; i < MT; ++i) {
            const int co = c_base + i * 16 + kgl * 4;
            if (co >= k.cout) continue;
            const int nvalid = min(4, k.cout - co);
            float v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float t = acc[i][j][r];
                if (k.bias && r < nvalid) t += k.bias[co + r];
                v[r] = apply_act(t, k.act);
            }
            if (k.out_mode == DBSR_OUT_NHWC) {
                if (k.r) {
                    const long long roff = map_frame(k.rm, f) * k.r_is + (long long)rr * k.r_ld + k.r_c0 + co;
                    if (k.y_f32) {
                        const float* rp = (const float*)k.r + roff;
                        for (int r = 0; r < nvalid; ++r) v[r] = apply_act(v[r] + rp[r], k.post_act);
                    } else {
                        const T* rp = (const T*)k.r + roff;
                        for (int r = 0; r < nvalid; ++r) v[r] = apply_act(v[r] + elem<T>::ld(rp + r), k.post_act);
                    }
                }
                store4<T>(k, map_frame(k.ym, f) * k.y_is + (long long)rr * k.y_ld + k.y_c0 + co, v, nvalid);
            } else if (k.out_mode == DBSR_OUT_SHUFFLE) {
                const int s = k.shuffle, sub = co / k.cps, c = co - sub * k.cps;
                const int Y = oy * s + sub / s, X = ox * s + sub % s;
                const long long off = map_frame(k.ym, f) * k.y_is +
                                      ((long long)Y * (k.out_w * s) + X) * k.y_ld + k.y_c0 + c;
                store4<T>(k, off, v, nvalid);
            } else {   // NCHW fp32
                float* y = (float*)k.y + map_frame(k.ym, f) * k.y_is + (long long)co * hw + rr;
                for (int r = 0; r < nvalid; ++r) y[(long long)r * hw] = v[r];
            }
        }
    }
}

__global__ void pack_weights_kernel(const float* __restrict__ w, const float* __restrict__ bias, int cout, int cin,
                                    int kh, int kw, int CG, int KG, int Kp, int cout_pad, int shuffle, int is_bf16,
                                    void* __restrict__ out, float* __restrict__ bias_out) {
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long total = (long long)cout_pad * Kp;
    if (idx >= total) return;
    const int co = (int)(idx / Kp), kk = (int)(idx - (long long)co * Kp);
    int co_src = co;
    if (shuffle > 1 && co < cout) {
        const int s2 = shuffle * shuffle, cps = cout / s2;
        const int sub = co / cps, c = co - sub * cps;
        co_src = c * s2 + sub;
    }
    const int kg = kk >> 3, jj = kk & 7;
    float v = 0.f;
    if (co < cout && kg < KG) {
        const int tap = kg / CG, c = (kg - tap * CG) * 8 + jj;
        if (c < cin) {
            const int ky = tap / kw, kx = tap - ky * kw;
            v = w[(((long long)co_src * cin + c) * kh + ky) * kw + kx];
        }
    }
    if (is_bf16)
        ((bf16_t*)out)[idx] = f2bf(v);
    else
        ((float*)out)[idx] = v;
    if (bias_out && kk == 0 && co < cout) bias_out[co] = bias ? bias[co_src] : 0.f;
}

template <typename T, int MT, int NT>
int launch_conv(const ConvK& k, hipStream_t s) {
    dim3 grid((k.npix + 4 * NT * 16 - 1) / (4 * NT * 16), (k.cout + MT * 16 - 1) / (MT * 16));
    hipLaunchKernelGGL((conv2d_kernel<T, MT, NT>), grid, dim3(256), 0, s, k);
    DBSR_LAUNCH_CHECK();
    return 0;
}

template <typename T>
int dispatch_conv(const ConvK& k, hipStream_t s) {
    const int tiles4 = (k.npix + 255) / 256;
    const bool small = tiles4 * ((k.cout + 63) / 64) < 512;   // too few blocks to fill 256 CUs
    if (k.cout <= 16) return small ? launch_conv<T, 1, 2>(k, s) : launch_conv<T, 1, 4>(k, s);
    if (k.cout <= 32) return small ? launch_conv<T, 2, 2>(k, s) : launch_conv<T, 2, 4>(k, s);
    return small ? launch_conv<T, 4, 2>(k, s) : launch_conv<T, 4, 4>(k, s);
}

inline int round_up(int a, int b) { return (a + b - 1) / b * b; }

}  // namespace

extern "C" size_t dbsr_conv_packed_elems(int cout, int cin, int kh, int kw) {
    const int cin8 = round_up(cin, 8);
    const int KGp = round_up(kh * kw * (cin8 / 8), 4);
    return (size_t)round_up(cout, 64) * KGp * 8;
}

extern "C" int dbsr_conv_pack_weights(const float* w_f32, const float* bias_f32, int cout, int cin, int kh, int kw,
                                      int dtype, int shuffle, void* w_packed, float* bias_out, void* stream) {
    DBSR_CHECK_ARG(w_f32 && w_packed, "pack_weights: null pointer");
    DBSR_CHECK_ARG(cout > 0 && cin > 0 && kh > 0 && kw > 0, "pack_weights: bad shape");
    DBSR_CHECK_ARG(dtype == DBSR_F32 || dtype == DBSR_BF16, "pack_weights: bad dtype");
    if (shuffle > 1)
        DBSR_CHECK_ARG(cout % (shuffle * shuffle) == 0 && (cout / (shuffle * shuffle)) % 4 == 0,
                       "pack_weights: cout %d not divisible for shuffle %d", cout, shuffle);
    const int CG = round_up(cin, 8) / 8, KG = kh * kw * CG, KGp = round_up(KG, 4), Kp = KGp * 8;
    const int cout_pad = round_up(cout, 64);
    const long long total = (long long)cout_pad * Kp;
    hipLaunchKernelGGL(pack_weights_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       w_f32, bias_f32, cout, cin, kh, kw, CG, KG, Kp, cout_pad, shuffle, dtype == DBSR_BF16 ? 1 : 0,
                       w_packed, bias_out);
    DBSR_LAUNCH_CHECK();
    return 0;
}

extern "C" int dbsr_conv2d(const dbsr_conv_desc* d, void* stream) {
    DBSR_CHECK_ARG(d, "conv2d: null desc");
    DBSR_CHECK_ARG(d->x.ptr && d->w && d->y.ptr, "conv2d: null pointer");
    DBSR_CHECK_ARG(d->x.dtype == DBSR_F32 || d->x.dtype == DBSR_BF16, "conv2d: bad input dtype");
    DBSR_CHECK_ARG(d->y.dtype == DBSR_F32 || d->y.dtype == d->x.dtype, "conv2d: output dtype must be f32 or input dtype");
    DBSR_CHECK_ARG(d->n_frames > 0 && d->in_h > 0 && d->in_w > 0 && d->out_h > 0 && d->out_w > 0, "conv2d: bad sizes");
    DBSR_CHECK_ARG(d->cin > 0 && d->cout > 0 && d->kh > 0 && d->kw > 0 && d->stride > 0 && d->dil > 0, "conv2d: bad shape");
    DBSR_CHECK_ARG(d->x.ld % 8 == 0 && d->x.c0 % 8 == 0, "conv2d: input ld/c0 must be multiples of 8 (got %d/%d)",
                   d->x.ld, d->x.c0);
    DBSR_CHECK_ARG(d->x.c0 + round_up(d->cin, 8) <= d->x.ld, "conv2d: input channel slice exceeds ld");
    DBSR_CHECK_ARG(d->x.map.fpg > 0 && d->y.map.fpg > 0, "conv2d: frame map fpg must be > 0");
    DBSR_CHECK_ARG(d->out_h == (d->in_h + 2 * d->pad - d->dil * (d->kh - 1) - 1) / d->stride + 1 &&
                   d->out_w == (d->in_w + 2 * d->pad - d->dil * (d->kw - 1) - 1) / d->stride + 1,
                   "conv2d: output size inconsistent with conv geometry");
    DBSR_CHECK_ARG(d->out_mode >= 0 && d->out_mode <= 2, "conv2d: bad out_mode");
    if (d->out_mode == DBSR_OUT_SHUFFLE) {
        const int s2 = d->shuffle * d->shuffle;
        DBSR_CHECK_ARG(d->shuffle > 1 && d->cout % s2 == 0 && (d->cout / s2) % 4 == 0, "conv2d: bad shuffle");
        DBSR_CHECK_ARG(d->res.ptr == nullptr, "conv2d: residual not supported with shuffle output");
    }
    if (d->out_mode == DBSR_OUT_NHWC) DBSR_CHECK_ARG(d->y.c0 + d->cout <= d->y.ld, "conv2d: output slice exceeds ld");
    if (d->out_mode == DBSR_OUT_NCHW_F32) DBSR_CHECK_ARG(d->y.dtype == DBSR_F32 && !d->res.ptr, "conv2d: NCHW out is f32, no residual");
    if (d->res.ptr) DBSR_CHECK_ARG(d->res.dtype == d->y.dtype && d->res.map.fpg > 0, "conv2d: residual dtype must equal output dtype");
    const long long npix = (long long)d->n_frames * d->out_h * d->out_w;
    DBSR_CHECK_ARG(npix < (1LL << 31), "conv2d: too many pixels");

    ConvK k;
    k.x = d->x.ptr; k.x_is = d->x.img_stride; k.x_ld = d->x.ld; k.xm = d->x.map; k.in_h = d->in_h; k.in_w = d->in_w;
    // the channel offset is folded into the base pointer (x.c0 is a multiple of 8)
    const int esz = d->x.dtype == DBSR_BF16 ? 2 : 4;
    k.x = (const char*)d->x.ptr + (long long)d->x.c0 * esz;
    const int CG = round_up(d->cin, 8) / 8;
    k.CG = CG; k.KG = d->kh * d->kw * CG; k.KGp = round_up(k.KG, 4); k.Kp = k.KGp * 8;
    k.w = d->w; k.bias = d->bias; k.kw = d->kw; k.stride = d->stride; k.pad = d->pad; k.dil = d->dil; k.cout = d->cout;
    k.y = d->y.ptr; k.y_f32 = d->y.dtype == DBSR_F32; k.y_is = d->y.img_stride; k.y_ld = d->y.ld; k.y_c0 = d->y.c0;
    k.ym = d->y.map; k.out_h = d->out_h; k.out_w = d->out_w; k.act = d->act;
    k.r = d->res.ptr; k.r_is = d->res.img_stride; k.r_ld = d->res.ld; k.r_c0 = d->res.c0; k.rm = d->res.map;
    if (!k.r) k.rm = d->y.map;
    k.post_act = d->post_act; k.out_mode = d->out_mode; k.shuffle = d->shuffle;
    k.cps = d->out_mode == DBSR_OUT_SHUFFLE ? d->cout / (d->shuffle * d->shuffle) : 0;
    k.npix = (int)npix;
    k.vec_store = (d->out_mode != DBSR_OUT_NCHW_F32) && (d->y.ld % 4 == 0) && (d->y.c0 % 4 == 0);
    hipStream_t s = (hipStream_t)stream;
    return d->x.dtype == DBSR_BF16 ? dispatch_conv<bf16_t>(k, s) : dispatch_conv<float>(k, s);
}
