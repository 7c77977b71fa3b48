// DBSR merge-path kernels: flow-guided warp of the frame embeddings (HBM-bound), softmax-over-burst
// fusion (HBM-bound), merge input prep and the decoder's Gaussian blur.  NHWC activations.
#include <cstdlib>
#include <type_traits>
#include "common.hpp"

using namespace dbsr;

namespace {

// ------------------------------------------------------------------------------------------------
// warp (models/layers/warp.py:19-46): sample feat at grid = (x + 0.5 + fx, y + 0.5 + fy) normalised by
// 2g/W - 1 and unnormalised by grid_sample(align_corners=False): ((g+1)*W - 1)/2, i.e. x + fx; the
// float op sequence of the reference is kept so sample positions round identically.
// Thread = (pixel, 8-channel group): a wave covers 512 contiguous channels (1 KiB bf16) per tap.
// ------------------------------------------------------------------------------------------------
template <typename T, bool WAVE_PIX>
__global__ __launch_bounds__(256) void warp_kernel(int n, int h, int w, int groups, dbsr_tensor feat,
                                                   const float* __restrict__ flow, long long fis, dbsr_tensor out) {
    // contiguous pixel ranges per XCD: the bilinear taps of neighbouring pixels then share one L2
    // (measured: fetch 576 -> 243 MB per launch at cfg2, i.e. the compulsory bytes; speed-only remap)
    const unsigned b = blockIdx.x, nb = gridDim.x, xcd = b & 7, q8 = nb >> 3, r8 = nb & 7;
    const unsigned lb = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
    const int hw = h * w;
    int g, p, rr;
    if constexpr (WAVE_PIX) {
        // groups % 64 == 0: a wave covers channels of one pixel, so the pixel index is wave-uniform
        // and all index divisions run on the scalar unit
        const unsigned gw = __builtin_amdgcn_readfirstlane(lb * 4 + (threadIdx.x >> 6));
        const unsigned wpp = (unsigned)groups >> 6;
        const unsigned pix = gw / wpp;
        if (pix >= (unsigned)n * hw) return;
        g = (int)(gw - pix * wpp) * 64 + (threadIdx.x & 63);
        p = (int)(pix / hw);
        rr = (int)(pix - (unsigned)p * hw);
    } else {
        const long long idx = (long long)lb * blockDim.x + threadIdx.x;
        if (idx >= (long long)n * h * w * groups) return;
        g = (int)(idx % groups);
        const long long pix = idx / groups;
        p = (int)(pix / hw);
        rr = (int)(pix - (long long)p * hw);
    }
    const int y = rr / w, x = rr - y * w;
    const float* fl = flow + (long long)p * fis + rr;
    const float gx = ((float)x + 0.5f) + fl[0];
    const float gy = ((float)y + 0.5f) + fl[hw];
    const float gxn = 2.0f * gx / (float)w - 1.0f, gyn = 2.0f * gy / (float)h - 1.0f;
    const float ix = ((gxn + 1.f) * (float)w - 1.f) / 2.f;
    const float iy = ((gyn + 1.f) * (float)h - 1.f) / 2.f;
    const float fx0 = floorf(ix), fy0 = floorf(iy);
    const int x0 = (int)fx0, y0 = (int)fy0;
    const float wx1 = ix - fx0, wx0 = 1.f - wx1, wy1 = iy - fy0, wy0 = 1.f - wy1;
    const T* base = img_ptr<T>(feat, p) + g * 8;
    if constexpr (sizeof(T) == 2) {
        // packed fp32 math (v_pk_fma_f32): 4 two-wide FMAs per tap instead of 8
        f32x2_t acc[4] = {{0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int xx = x0 + (t & 1), yy = y0 + (t >> 1);
            const float wt = ((t & 1) ? wx1 : wx0) * ((t >> 1) ? wy1 : wy0);
            if ((unsigned)xx < (unsigned)w && (unsigned)yy < (unsigned)h) {
                const u32x4_t q = *(const u32x4_t*)(base + ((long long)yy * w + xx) * feat.ld);
                const f32x2_t w2 = {wt, wt};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const f32x2_t v = {H16<T>::lo(q[e]), H16<T>::hi(q[e])};
                    acc[e] = __builtin_elementwise_fma(w2, v, acc[e]);
                }
            }
        }
        u32x4_t o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = H16<T>::pack(acc[e][0], acc[e][1]);
        *(u32x4_t*)(img_ptr<T>(out, p) + (long long)rr * out.ld + g * 8) = o;
    } else {
        float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int xx = x0 + (t & 1), yy = y0 + (t >> 1);
            const float wt = ((t & 1) ? wx1 : wx0) * ((t >> 1) ? wy1 : wy0);
            if ((unsigned)xx < (unsigned)w && (unsigned)yy < (unsigned)h) {
                float v[8];
                load8(base + ((long long)yy * w + xx) * feat.ld, v);
#pragma unroll
                for (int j = 0; j < 8; ++j) acc[j] = fmaf(wt, v[j], acc[j]);
            }
        }
        store8(img_ptr<T>(out, p) + (long long)rr * out.ld + g * 8, acc);
    }
}

// C == 512 (64 lanes x 8 channels = one pixel per wave-row): each wave handles PPW consecutive
// pixels, issues all 4*PPW tap loads before consuming any (the per-pixel version had two dependent
// memory round trips and only 4 KiB in flight per wave: latency-bound), and reads the flow with
// wave-uniform (scalar) loads.
template <typename T, int PPW>
__global__ __launch_bounds__(256) void warp512_bf16_kernel(int n, int h, int w, dbsr_tensor feat,
                                                           const float* __restrict__ flow, long long fis,
                                                           dbsr_tensor out) {
    const unsigned b = blockIdx.x, nb = gridDim.x, xcd = b & 7, q8 = nb >> 3, r8 = nb & 7;
    const unsigned lb = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
    const unsigned gw = __builtin_amdgcn_readfirstlane(lb * 4 + (threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    const int hw = h * w;
    const unsigned total = (unsigned)n * hw;
    int tapoff[PPW][4];
    float tapw[PPW][4];
    const T* fbase[PPW];
    T* obase[PPW];
    bool live[PPW];
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
        const unsigned pix = gw * PPW + i;
        live[i] = pix < total;
        const unsigned pc = live[i] ? pix : 0;
        const int p = (int)(pc / hw), rr = (int)(pc - (unsigned)p * hw);
        const int y = rr / w, x = rr - y * w;
        const float* fl = flow + (long long)p * fis + rr;
        const float gx = ((float)x + 0.5f) + fl[0];
        const float gy = ((float)y + 0.5f) + fl[hw];
        const float gxn = 2.0f * gx / (float)w - 1.0f, gyn = 2.0f * gy / (float)h - 1.0f;
        const float ix = ((gxn + 1.f) * (float)w - 1.f) / 2.f;
        const float iy = ((gyn + 1.f) * (float)h - 1.f) / 2.f;
        const float fx0 = floorf(ix), fy0 = floorf(iy);
        const int x0 = (int)fx0, y0 = (int)fy0;
        const float wx1 = ix - fx0, wx0 = 1.f - wx1, wy1 = iy - fy0, wy0 = 1.f - wy1;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int xx = x0 + (t & 1), yy = y0 + (t >> 1);
            const bool ok = (unsigned)xx < (unsigned)w && (unsigned)yy < (unsigned)h;
            tapw[i][t] = ok ? ((t & 1) ? wx1 : wx0) * ((t >> 1) ? wy1 : wy0) : 0.f;
            tapoff[i][t] = ok ? (yy * w + xx) * feat.ld : 0;        // clamped: in-bounds address, weight 0
        }
        fbase[i] = img_ptr<T>(feat, p) + lane * 8;
        obase[i] = img_ptr<T>(out, p) + (long long)rr * out.ld + lane * 8;
    }
    u32x4_t v[PPW][4];
#pragma unroll
    for (int i = 0; i < PPW; ++i)
#pragma unroll
        for (int t = 0; t < 4; ++t) v[i][t] = *(const u32x4_t*)(fbase[i] + tapoff[i][t]);
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
        f32x2_t acc[4] = {{0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const f32x2_t w2 = {tapw[i][t], tapw[i][t]};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const f32x2_t x2 = {H16<T>::lo(v[i][t][e]), H16<T>::hi(v[i][t][e])};
                acc[e] = __builtin_elementwise_fma(w2, x2, acc[e]);
            }
        }
        u32x4_t o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = H16<T>::pack(acc[e][0], acc[e][1]);
        if (live[i]) *(u32x4_t*)obase[i] = o;
    }
}

// ------------------------------------------------------------------------------------------------
// Fusion (merging.py:116-126): w = softmax_n(logits[b,n]), fused[b] = sum_n feat[b,n] * w[b,n].
// Thread = (b, pixel, 4 channels); the N logits stay in registers (one read of each byte), fp32
// softmax, optional write of the normalised weights (the reference's aux 'fusion_weights').
// ------------------------------------------------------------------------------------------------
template <typename T> struct Vec4;
template <> struct Vec4<float> {
    static __device__ __forceinline__ void ld(const float* p, float (&v)[4]) {
        float4 q = *(const float4*)p;
        v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
    }
    static __device__ __forceinline__ void st(float* p, const float (&v)[4]) {
        *(float4*)p = make_float4(v[0], v[1], v[2], v[3]);
    }
};
template <typename T> struct Vec4 {          // 16-bit storage (bf16 / fp16)
    static __device__ __forceinline__ void ld(const T* p, float (&v)[4]) {
        uint2 q = *(const uint2*)p;
        v[0] = H16<T>::lo(q.x); v[1] = H16<T>::hi(q.x);
        v[2] = H16<T>::lo(q.y); v[3] = H16<T>::hi(q.y);
    }
    static __device__ __forceinline__ void st(T* p, const float (&v)[4]) {
        uint2 q;
        q.x = H16<T>::pack(v[0], v[1]);
        q.y = H16<T>::pack(v[2], v[3]);
        *(uint2*)p = q;
    }
};

template <typename T, int NMAX, bool WAVE_PIX>
__global__ __launch_bounds__(256) void fuse_softmax_kernel(int B, int N, int hw, int groups, dbsr_tensor logits,
                                                           dbsr_tensor ref, dbsr_tensor oth, dbsr_tensor fused,
                                                           dbsr_tensor weights) {
    int g, b, rr;
    if constexpr (WAVE_PIX) {            // groups % 64 == 0: wave-uniform pixel, scalar index math
        const unsigned gw = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
        const unsigned wpp = (unsigned)groups >> 6;
        const unsigned pix = gw / wpp;
        if (pix >= (unsigned)B * hw) return;
        g = (int)(gw - pix * wpp) * 64 + (threadIdx.x & 63);
        b = (int)(pix / hw);
        rr = (int)(pix - (unsigned)b * hw);
    } else {
        const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
        if (idx >= (long long)B * hw * groups) return;
        g = (int)(idx % groups);
        const long long pix = idx / groups;
        b = (int)(pix / hw);
        rr = (int)(pix - (long long)b * hw);
    }
    const int c = g * 4;
    float l[NMAX][4], fv[NMAX][4];
    float m[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    // issue every logit and feature load up front (2N independent loads in flight per thread)
#pragma unroll
    for (int n = 0; n < NMAX; ++n) {
        if (n < N) {
            Vec4<T>::ld(img_ptr<T>(logits, b * N + n) + (long long)rr * logits.ld + c, l[n]);
            const T* fp = n == 0 ? img_ptr<T>(ref, b) + (long long)rr * ref.ld
                                 : img_ptr<T>(oth, b * (N - 1) + n - 1) + (long long)rr * oth.ld;
            Vec4<T>::ld(fp + c, fv[n]);
        }
    }
#pragma unroll
    for (int n = 0; n < NMAX; ++n) {
        if (n < N) {
#pragma unroll
            for (int j = 0; j < 4; ++j) m[j] = fmaxf(m[j], l[n][j]);
        }
    }
    float s[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int n = 0; n < NMAX; ++n) {
        if (n < N) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                l[n][j] = __expf(l[n][j] - m[j]);
                s[j] += l[n][j];
            }
        }
    }
    float inv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) inv[j] = 1.0f / s[j];
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int n = 0; n < NMAX; ++n) {
        if (n < N) {
            float wn[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                wn[j] = l[n][j] * inv[j];
                acc[j] = fmaf(fv[n][j], wn[j], acc[j]);
            }
            if (weights.ptr) {
                if (weights.dtype == DBSR_F32)
                    Vec4<float>::st(img_ptr<float>(weights, b * N + n) + (long long)rr * weights.ld + c, wn);
                else
                    Vec4<T>::st(img_ptr<T>(weights, b * N + n) + (long long)rr * weights.ld + c, wn);
            }
        }
    }
    Vec4<T>::st(img_ptr<T>(fused, b) + (long long)rr * fused.ld + c, acc);
}

// bf16, C == 512: one wave per pixel, 8 channels per lane, so every logit/feature/weight access is a
// 16-B-per-lane sweep of one 1-KiB pixel row (the 4-channel kernel above moves 8 B per lane and needs
// twice the memory instructions).  All 2N loads are issued before the first use; the logits are
// consumed once, so they are streamed with non-temporal loads, and the aux weights (written once,
// never re-read by the forward) with non-temporal stores, keeping L2 for the feature rows.
template <typename T, int NMAX>
__global__ __launch_bounds__(256, 2) void fuse512_bf16_kernel(int B, int N, int hw, dbsr_tensor logits, dbsr_tensor ref,
                                                           dbsr_tensor oth, dbsr_tensor fused, dbsr_tensor weights) {
    const unsigned pix = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
    if (pix >= (unsigned)B * hw) return;
    const int b = (int)(pix / hw), rr = (int)(pix - (unsigned)b * hw);
    const int c = (threadIdx.x & 63) * 8;
    u32x4_t lr[NMAX], fr[NMAX];
#pragma unroll
    for (int n = 0; n < NMAX; ++n) {
        if (n < N) {
            lr[n] = __builtin_nontemporal_load(
                (const u32x4_t*)(img_ptr<T>(logits, b * N + n) + (long long)rr * logits.ld + c));
            const T* fp = n == 0 ? img_ptr<T>(ref, b) + (long long)rr * ref.ld
                                 : img_ptr<T>(oth, b * (N - 1) + n - 1) + (long long)rr * oth.ld;
            fr[n] = *(const u32x4_t*)(fp + c);
        }
    }
    float m[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) m[j] = -INFINITY;
#pragma unroll
    for (int n = 0; n < NMAX; ++n) {
        if (n < N) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                m[2 * j] = fmaxf(m[2 * j], H16<T>::lo(lr[n][j]));
                m[2 * j + 1] = fmaxf(m[2 * j + 1], H16<T>::hi(lr[n][j]));
            }
        }
    }
    // the N x 8 exp() values stay live (recomputing them at 3 waves/SIMD spilled: +65 MB scratch traffic)
    float e[NMAX][8], s[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] = 0.f;
#pragma unroll
    for (int n = 0; n < NMAX; ++n) {
        if (n < N) {
            float en[8];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                en[2 * j] = __expf(H16<T>::lo(lr[n][j]) - m[2 * j]);
                en[2 * j + 1] = __expf(H16<T>::hi(lr[n][j]) - m[2 * j + 1]);
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                s[j] += en[j];
                e[n][j] = en[j];
            }
        }
    }
    float inv[8], acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        inv[j] = 1.0f / s[j];
        acc[j] = 0.f;
    }
#pragma unroll
    for (int n = 0; n < NMAX; ++n) {
        if (n < N) {
            float wn[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) wn[j] = e[n][j] * inv[j];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                acc[2 * j] = fmaf(H16<T>::lo(fr[n][j]), wn[2 * j], acc[2 * j]);
                acc[2 * j + 1] = fmaf(H16<T>::hi(fr[n][j]), wn[2 * j + 1], acc[2 * j + 1]);
            }
            if (weights.ptr) {
                u32x4_t o;
#pragma unroll
                for (int j = 0; j < 4; ++j) o[j] = H16<T>::pack(wn[2 * j], wn[2 * j + 1]);
                __builtin_nontemporal_store(o, (u32x4_t*)(img_ptr<T>(weights, b * N + n) + (long long)rr * weights.ld + c));
            }
        }
    }
    u32x4_t o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = H16<T>::pack(acc[2 * j], acc[2 * j + 1]);
    *(u32x4_t*)(img_ptr<T>(fused, b) + (long long)rr * fused.ld + c) = o;
}

// ------------------------------------------------------------------------------------------------
// Frame-sharded fusion (SURVEY §8e, configs[4]): the softmax over the burst (merging.py:116-124)
// split over ranks that each hold a subset of the frames.  Rank-local partial statistics per
// (b, pixel, channel): m = max_n l_n, s = sum_n exp(l_n - m), a = sum_n exp(l_n - m) * f_n over the
// local frames [first, N); then a log-sum-exp combine over the R ranks' statistics:
// fused = (sum_r a_r e^(m_r - M)) / (sum_r s_r e^(m_r - M)), M = max_r m_r.  Same value as
// sum_n f_n softmax(l)_n up to fp32 rounding order.  stats: fp32 [B][hw][3c] = (m | s | a).
// ------------------------------------------------------------------------------------------------
template <typename T, int NMAX>
__global__ __launch_bounds__(256) void fuse_partial_kernel(int B, int N, int hw, int groups, int first,
                                                           dbsr_tensor logits, dbsr_tensor ref, dbsr_tensor oth,
                                                           float* __restrict__ stats) {
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long long)B * hw * groups) return;
    const int g = (int)(idx % groups);
    const long long pix = idx / groups;
    const int b = (int)(pix / hw), rr = (int)(pix - (long long)b * hw);
    const int c = g * 4, C = groups * 4;
    float l[NMAX][4];
    float m[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY}, s[4] = {0.f, 0.f, 0.f, 0.f}, a[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int n = 0; n < NMAX; ++n) {
        if (n >= first && n < N) {
            Vec4<T>::ld(img_ptr<T>(logits, b * N + n) + (long long)rr * logits.ld + c, l[n]);
#pragma unroll
            for (int j = 0; j < 4; ++j) m[j] = fmaxf(m[j], l[n][j]);
        }
    }
#pragma unroll
    for (int n = 0; n < NMAX; ++n) {
        if (n >= first && n < N) {
            float fv[4];
            const T* fp = n == 0 ? img_ptr<T>(ref, b) + (long long)rr * ref.ld
                                 : img_ptr<T>(oth, b * (N - 1) + n - 1) + (long long)rr * oth.ld;
            Vec4<T>::ld(fp + c, fv);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float e = __expf(l[n][j] - m[j]);
                s[j] += e;
                a[j] = fmaf(fv[j], e, a[j]);
            }
        }
    }
    float* o = stats + pix * 3 * C + c;
    Vec4<float>::st(o, m);
    Vec4<float>::st(o + C, s);
    Vec4<float>::st(o + 2 * C, a);
}

// Any burst size (N > 16, beyond the register-resident kernels above): the same three passes over the
// frames (max, sum of exp, normalised weights x features), reloading the logits per pass instead of
// holding them in registers.  Same arithmetic and order as fuse_softmax_kernel.
template <typename T>
__global__ __launch_bounds__(256) void fuse_softmax_any_kernel(int B, int N, int hw, int groups, dbsr_tensor logits,
                                                               dbsr_tensor ref, dbsr_tensor oth, dbsr_tensor fused,
                                                               dbsr_tensor weights) {
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long long)B * hw * groups) return;
    const int g = (int)(idx % groups);
    const long long pix = idx / groups;
    const int b = (int)(pix / hw), rr = (int)(pix - (long long)b * hw);
    const int c = g * 4;
    auto lg = [&](int n, float (&v)[4]) { Vec4<T>::ld(img_ptr<T>(logits, b * N + n) + (long long)rr * logits.ld + c, v); };
    float m[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY}, s[4] = {0.f, 0.f, 0.f, 0.f};
    for (int n = 0; n < N; ++n) {
        float l[4];
        lg(n, l);
#pragma unroll
        for (int j = 0; j < 4; ++j) m[j] = fmaxf(m[j], l[j]);
    }
    for (int n = 0; n < N; ++n) {
        float l[4];
        lg(n, l);
#pragma unroll
        for (int j = 0; j < 4; ++j) s[j] += __expf(l[j] - m[j]);
    }
    float inv[4], acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 4; ++j) inv[j] = 1.0f / s[j];
    for (int n = 0; n < N; ++n) {
        float l[4], fv[4], wn[4];
        lg(n, l);
        const T* fp = n == 0 ? img_ptr<T>(ref, b) + (long long)rr * ref.ld
                             : img_ptr<T>(oth, b * (N - 1) + n - 1) + (long long)rr * oth.ld;
        Vec4<T>::ld(fp + c, fv);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            wn[j] = __expf(l[j] - m[j]) * inv[j];
            acc[j] = fmaf(fv[j], wn[j], acc[j]);
        }
        if (weights.ptr) {
            if (weights.dtype == DBSR_F32)
                Vec4<float>::st(img_ptr<float>(weights, b * N + n) + (long long)rr * weights.ld + c, wn);
            else
                Vec4<T>::st(img_ptr<T>(weights, b * N + n) + (long long)rr * weights.ld + c, wn);
        }
    }
    Vec4<T>::st(img_ptr<T>(fused, b) + (long long)rr * fused.ld + c, acc);
}

// frame-sharded statistics for any burst size (two passes over the local frames)
template <typename T>
__global__ __launch_bounds__(256) void fuse_partial_any_kernel(int B, int N, int hw, int groups, int first,
                                                               dbsr_tensor logits, dbsr_tensor ref, dbsr_tensor oth,
                                                               float* __restrict__ stats) {
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long long)B * hw * groups) return;
    const int g = (int)(idx % groups);
    const long long pix = idx / groups;
    const int b = (int)(pix / hw), rr = (int)(pix - (long long)b * hw);
    const int c = g * 4, C = groups * 4;
    float m[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY}, s[4] = {0.f, 0.f, 0.f, 0.f}, a[4] = {0.f, 0.f, 0.f, 0.f};
    for (int n = first; n < N; ++n) {
        float l[4];
        Vec4<T>::ld(img_ptr<T>(logits, b * N + n) + (long long)rr * logits.ld + c, l);
#pragma unroll
        for (int j = 0; j < 4; ++j) m[j] = fmaxf(m[j], l[j]);
    }
    for (int n = first; n < N; ++n) {
        float l[4], fv[4];
        Vec4<T>::ld(img_ptr<T>(logits, b * N + n) + (long long)rr * logits.ld + c, l);
        const T* fp = n == 0 ? img_ptr<T>(ref, b) + (long long)rr * ref.ld
                             : img_ptr<T>(oth, b * (N - 1) + n - 1) + (long long)rr * oth.ld;
        Vec4<T>::ld(fp + c, fv);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float e = __expf(l[j] - m[j]);
            s[j] += e;
            a[j] = fmaf(fv[j], e, a[j]);
        }
    }
    float* o = stats + pix * 3 * C + c;
    Vec4<float>::st(o, m);
    Vec4<float>::st(o + C, s);
    Vec4<float>::st(o + 2 * C, a);
}

template <typename T>
__global__ __launch_bounds__(256) void fuse_combine_kernel(int R, int B, int hw, int groups,
                                                           const float* __restrict__ stats, dbsr_tensor fused) {
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long total = (long long)B * hw * groups;
    if (idx >= total) return;
    const int g = (int)(idx % groups);
    const long long pix = idx / groups;
    const int b = (int)(pix / hw), rr = (int)(pix - (long long)b * hw);
    const int c = g * 4, C = groups * 4;
    const long long rank_stride = (long long)B * hw * 3 * C;
    float M[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    for (int r = 0; r < R; ++r) {
        float m[4];
        Vec4<float>::ld(stats + r * rank_stride + pix * 3 * C + c, m);
#pragma unroll
        for (int j = 0; j < 4; ++j) M[j] = fmaxf(M[j], m[j]);
    }
    float S[4] = {0.f, 0.f, 0.f, 0.f}, A[4] = {0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < R; ++r) {
        const float* p = stats + r * rank_stride + pix * 3 * C + c;
        float m[4], sv[4], av[4];
        Vec4<float>::ld(p, m);
        Vec4<float>::ld(p + C, sv);
        Vec4<float>::ld(p + 2 * C, av);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float k = m[j] == -INFINITY ? 0.f : __expf(m[j] - M[j]);   // a rank with no frames adds nothing
            S[j] = fmaf(sv[j], k, S[j]);
            A[j] = fmaf(av[j], k, A[j]);
        }
    }
    float out[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) out[j] = A[j] / S[j];
    Vec4<T>::st(img_ptr<T>(fused, b) + (long long)rr * fused.ld + c, out);
}

// ------------------------------------------------------------------------------------------------
// merge prep (merging.py:79-89): out = [proj[b,0] | proj[b,n] - proj[b,0]]
// ------------------------------------------------------------------------------------------------
template <typename T>
__global__ void merge_prep_kernel(int B, int N, int hw, int C, dbsr_tensor proj, dbsr_tensor out) {
    const int groups = C / 8;
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long long)B * N * hw * groups) return;
    const int g = (int)(idx % groups);
    const long long pix = idx / groups;
    const int f = (int)(pix / hw), rr = (int)(pix - (long long)f * hw);
    const int b = f / N;
    float base[8], cur[8];
    load8(img_ptr<T>(proj, b * N) + (long long)rr * proj.ld + g * 8, base);
    load8(img_ptr<T>(proj, f) + (long long)rr * proj.ld + g * 8, cur);
#pragma unroll
    for (int j = 0; j < 8; ++j) cur[j] -= base[j];
    T* o = img_ptr<T>(out, f) + (long long)rr * out.ld + g * 8;
    store8(o, base);
    store8(o + C, cur);
}

// ------------------------------------------------------------------------------------------------
// Gaussian blur (upsampling.py:59-65): per-channel 3x3 cross-correlation with zero padding.
// ------------------------------------------------------------------------------------------------
struct K9 {
    float k[9];
};
// Thread = (frame, 8-channel group, column, strip of BLUR_ROWS rows): it slides a 3-row window down
// its strip, loading each input row's 3 column neighbours once (3 16-B loads per output instead of 9);
// consecutive threads are consecutive (group, column), so every row load is a coalesced 16-B-per-lane
// sweep of one image row.
constexpr int BLUR_ROWS = 8;
template <typename T>
__global__ __launch_bounds__(256) void blur3_kernel(int n, int h, int w, int groups, dbsr_tensor in, K9 kk,
                                                    dbsr_tensor out) {
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const int strips = (h + BLUR_ROWS - 1) / BLUR_ROWS;
    if (idx >= (long long)n * strips * w * groups) return;
    const int g = (int)(idx % groups);
    long long r = idx / groups;
    const int x = (int)(r % w);
    r /= w;
    const int st = (int)(r % strips);
    const int f = (int)(r / strips);
    const T* base = img_ptr<T>(in, f) + g * 8;
    T* obase = img_ptr<T>(out, f) + g * 8;
    float win[3][3][8];                       // [row slot][column -1..+1][channel]
    auto load_row = [&](int yy, float (&dst)[3][8]) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const int xx = x + j - 1;
            if ((unsigned)yy < (unsigned)h && (unsigned)xx < (unsigned)w) {
                load8(base + ((long long)yy * w + xx) * in.ld, dst[j]);
            } else {
#pragma unroll
                for (int q = 0; q < 8; ++q) dst[j][q] = 0.f;
            }
        }
    };
    const int y0 = st * BLUR_ROWS;
    load_row(y0 - 1, win[0]);
    load_row(y0, win[1]);
#pragma unroll
    for (int t = 0; t < BLUR_ROWS; ++t) {
        const int y = y0 + t;
        if (y >= h) break;
        // rotating slots: rows y-1, y, y+1 sit in slots t%3, (t+1)%3, (t+2)%3 (unrolled: static indices)
        load_row(y + 1, win[(t + 2) % 3]);
        float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const float kv = kk.k[i * 3 + j];
#pragma unroll
                for (int q = 0; q < 8; ++q) acc[q] = fmaf(kv, win[(t + i) % 3][j][q], acc[q]);
            }
        store8(obase + ((long long)y * w + x) * out.ld, acc);
    }
}

// 16-bit variant: every row load of the strip (ROWS + 2 rows x 3 columns, raw 16-B, 120 VGPRs at 8 rows)
// is issued before the first FMA, so a thread waits one memory latency instead of one per row.  The Gaussian
// (separable: blur_separable) runs as blur_row + blur_col, the sums dbsr_conv_shuffle_blur uses (bitwise equal).
template <typename T, int ROWS>
__global__ __launch_bounds__(256) void blur3_h16_kernel(int n, int h, int w, int groups, dbsr_tensor in, Blur3 kb,
                                                        dbsr_tensor out) {
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const int strips = (h + ROWS - 1) / ROWS;
    if (idx >= (long long)n * strips * w * groups) return;
    const int g = (int)(idx % groups);
    long long r = idx / groups;
    const int x = (int)(r % w);
    r /= w;
    const int st = (int)(r % strips);
    const int f = (int)(r / strips);
    const T* base = img_ptr<T>(in, f) + g * 8;
    T* obase = img_ptr<T>(out, f) + g * 8;
    const int y0 = st * ROWS;
    u32x4_t raw[ROWS + 2][3];
#pragma unroll
    for (int i = 0; i < ROWS + 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const int yy = y0 + i - 1, xx = x + j - 1;
            raw[i][j] = u32x4_t{0u, 0u, 0u, 0u};
            if ((unsigned)yy < (unsigned)h && (unsigned)xx < (unsigned)w)
                raw[i][j] = *(const u32x4_t*)(base + ((long long)yy * w + xx) * in.ld);
        }
    float hr[3][8];
    blur_row<T>(kb, raw[0][0], raw[0][1], raw[0][2], hr[0]);
    blur_row<T>(kb, raw[1][0], raw[1][1], raw[1][2], hr[1]);
#pragma unroll
    for (int t = 0; t < ROWS; ++t) {
        const int y = y0 + t;
        blur_row<T>(kb, raw[t + 2][0], raw[t + 2][1], raw[t + 2][2], hr[(t + 2) % 3]);
        float acc[8];
        blur_col(kb, hr[t % 3], hr[(t + 1) % 3], hr[(t + 2) % 3], acc);
        if (y < h) store8(obase + ((long long)y * w + x) * out.ld, acc);
    }
}

// WeightedSum with softmax=False (merging.py:117-121): weights = relu(w) / (sum_n relu(w) + 1e-12), fused = sum_n
// weights * feat -- two passes over the burst's logits (sum, then normalise and fuse), 4 channels per thread;
// addressing as the softmax kernels
template <typename T>
__global__ __launch_bounds__(256) void fuse_relunorm_kernel(int B, int N, int hw, int groups, dbsr_tensor logits,
                                                            dbsr_tensor ref, dbsr_tensor oth, dbsr_tensor fused,
                                                            dbsr_tensor weights) {
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long long)B * hw * groups) return;
    const int g = (int)(idx % groups);
    const long long pix = idx / groups;
    const int b = (int)(pix / hw), rr = (int)(pix - (long long)b * hw);
    const int c = g * 4;
    auto lg = [&](int n, float (&v)[4]) { Vec4<T>::ld(img_ptr<T>(logits, b * N + n) + (long long)rr * logits.ld + c, v); };
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    for (int n = 0; n < N; ++n) {
        float l[4];
        lg(n, l);
#pragma unroll
        for (int j = 0; j < 4; ++j) s[j] += fmaxf(l[j], 0.f);
    }
    float den[4], acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 4; ++j) den[j] = s[j] + 1e-12f;
    for (int n = 0; n < N; ++n) {
        float l[4], fv[4], wn[4];
        lg(n, l);
        const T* fp = n == 0 ? img_ptr<T>(ref, b) + (long long)rr * ref.ld
                             : img_ptr<T>(oth, b * (N - 1) + n - 1) + (long long)rr * oth.ld;
        Vec4<T>::ld(fp + c, fv);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            wn[j] = fmaxf(l[j], 0.f) / den[j];
            acc[j] = fmaf(fv[j], wn[j], acc[j]);
        }
        if (weights.ptr) {
            if (weights.dtype == DBSR_F32)
                Vec4<float>::st(img_ptr<float>(weights, b * N + n) + (long long)rr * weights.ld + c, wn);
            else
                Vec4<T>::st(img_ptr<T>(weights, b * N + n) + (long long)rr * weights.ld + c, wn);
        }
    }
    Vec4<T>::st(img_ptr<T>(fused, b) + (long long)rr * fused.ld + c, acc);
}

// the burst mean of the projected embeddings (merging.py:81-82, use_base_frame=False): out[b] = (sum_n in[b*N+n]) / N
template <typename T>
__global__ __launch_bounds__(256) void burst_mean_kernel(int B, int N, int hw, int groups, dbsr_tensor in,
                                                         dbsr_tensor out) {
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long long)B * hw * groups) return;
    const int g = (int)(idx % groups);
    const long long pix = idx / groups;
    const int b = (int)(pix / hw), rr = (int)(pix - (long long)b * hw);
    const int c = g * 4;
    float a[4] = {0.f, 0.f, 0.f, 0.f};
    for (int n = 0; n < N; ++n) {
        float v[4];
        Vec4<T>::ld(img_ptr<T>(in, b * N + n) + (long long)rr * in.ld + c, v);
#pragma unroll
        for (int j = 0; j < 4; ++j) a[j] += v[j];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) a[j] /= (float)N;
    Vec4<T>::st(img_ptr<T>(out, b) + (long long)rr * out.ld + c, a);
}

inline unsigned nblocks(long long total, int bs) { return (unsigned)((total + bs - 1) / bs); }
bool map_ok(const dbsr_tensor& t) { return t.ptr && t.map.fpg > 0; }
bool vec_ok(const dbsr_tensor& t, int v) { return t.ld % v == 0 && t.c0 % v == 0; }

template <typename F>
int by_dtype(int dtype, F&& f) {
    if (dtype == DBSR_BF16) return f((bf16_t*)nullptr);
    if (dtype == DBSR_F16) return f((f16_t*)nullptr);
    if (dtype == DBSR_F32) return f((float*)nullptr);
    dbsr_set_error("unsupported dtype %d", dtype);
    return DBSR_E_ARG;
}

}  // namespace

extern "C" int dbsr_warp_bilinear(int n, int h, int w, int c, dbsr_tensor feat, const float* flow,
                                  long long flow_img_stride, dbsr_tensor out, void* stream) {
    DBSR_CHECK_ARG(map_ok(feat) && map_ok(out) && flow, "warp: bad tensor");
    DBSR_CHECK_ARG(feat.dtype == out.dtype, "warp: dtype mismatch");
    DBSR_CHECK_ARG(n > 0 && h > 0 && w > 0 && c > 0 && c % 8 == 0, "warp: c must be a multiple of 8");
    DBSR_CHECK_ARG(vec_ok(feat, 8) && vec_ok(out, 8), "warp: ld/c0 must be multiples of 8");
    const int groups = c / 8;
    return by_dtype(feat.dtype, [&](auto* tag) {
        using T = std::remove_pointer_t<decltype(tag)>;
        if (sizeof(T) == 2 && groups == 64) {
          if constexpr (sizeof(T) == 2) {
            // 4 pixels per wave (2: equal time, 8: occupancy-bound -- measured round 1)
            constexpr int PPW = 4;
            hipLaunchKernelGGL((warp512_bf16_kernel<T, PPW>), dim3(nblocks(((long long)n * h * w + PPW - 1) / PPW, 4)),
                               dim3(256), 0, (hipStream_t)stream, n, h, w, feat, flow, flow_img_stride, out);
          }
        } else if (groups % 64 == 0)
            hipLaunchKernelGGL((warp_kernel<T, true>), dim3(nblocks((long long)n * h * w * groups, 256)), dim3(256), 0,
                               (hipStream_t)stream, n, h, w, groups, feat, flow, flow_img_stride, out);
        else
            hipLaunchKernelGGL((warp_kernel<T, false>), dim3(nblocks((long long)n * h * w * groups, 256)), dim3(256),
                               0, (hipStream_t)stream, n, h, w, groups, feat, flow, flow_img_stride, out);
        DBSR_LAUNCH_CHECK();
        return 0;
    });
}

extern "C" int dbsr_fuse_softmax(int B, int N, int hw, int c, dbsr_tensor logits, dbsr_tensor ref, dbsr_tensor oth,
                                 dbsr_tensor fused, dbsr_tensor weights, void* stream) {
    DBSR_CHECK_ARG(map_ok(logits) && map_ok(ref) && map_ok(fused) && (N == 1 || map_ok(oth)), "fuse: bad tensor");
    DBSR_CHECK_ARG(logits.dtype == ref.dtype && fused.dtype == ref.dtype && (N == 1 || oth.dtype == ref.dtype),
                   "fuse: dtype mismatch");
    DBSR_CHECK_ARG(B > 0 && N > 0 && hw > 0 && c % 4 == 0, "fuse: B, N, hw > 0 and c a multiple of 4");
    DBSR_CHECK_ARG(vec_ok(logits, 4) && vec_ok(ref, 4) && vec_ok(fused, 4) && (N == 1 || vec_ok(oth, 4)),
                   "fuse: ld/c0 must be multiples of 4");
    if (weights.ptr) DBSR_CHECK_ARG(map_ok(weights) && vec_ok(weights, 4), "fuse: bad weights tensor");
    const int groups = c / 4;
    const long long total = (long long)B * hw * groups;
    return by_dtype(ref.dtype, [&](auto* tag) {
        using T = std::remove_pointer_t<decltype(tag)>;
        if (N > 16) {                   // any burst size: logits reloaded per pass
            hipLaunchKernelGGL(fuse_softmax_any_kernel<T>, dim3(nblocks(total, 256)), dim3(256), 0,
                               (hipStream_t)stream, B, N, hw, groups, logits, ref, oth, fused, weights);
            DBSR_LAUNCH_CHECK();
            return 0;
        }
        const bool wp = groups % 64 == 0;
        if constexpr (sizeof(T) == 2) {
            if (c == 512 && vec_ok(logits, 8) && vec_ok(ref, 8) && vec_ok(fused, 8) &&
                (N == 1 || vec_ok(oth, 8)) && (!weights.ptr || (weights.dtype == ref.dtype && vec_ok(weights, 8)))) {
                const long long waves = (long long)B * hw;
#define DBSR_FUSE512(NM)                                                                                       \
    hipLaunchKernelGGL((fuse512_bf16_kernel<T, NM>), dim3(nblocks(waves, 4)), dim3(256), 0, (hipStream_t)stream, B, \
                       N, hw, logits, ref, oth, fused, weights);
                if (N <= 4) {
                    DBSR_FUSE512(4)
                } else if (N <= 8) {
                    DBSR_FUSE512(8)
                } else if (N == 14) {
                    DBSR_FUSE512(14)
                } else {
                    DBSR_FUSE512(16)
                }
#undef DBSR_FUSE512
                DBSR_LAUNCH_CHECK();
                return 0;
            }
        }
#define DBSR_FUSE(NM)                                                                                         \
    if (wp)                                                                                                   \
        hipLaunchKernelGGL((fuse_softmax_kernel<T, NM, true>), dim3(nblocks(total, 256)), dim3(256), 0,       \
                           (hipStream_t)stream, B, N, hw, groups, logits, ref, oth, fused, weights);          \
    else                                                                                                      \
        hipLaunchKernelGGL((fuse_softmax_kernel<T, NM, false>), dim3(nblocks(total, 256)), dim3(256), 0,      \
                           (hipStream_t)stream, B, N, hw, groups, logits, ref, oth, fused, weights);
        if (N <= 4) {
            DBSR_FUSE(4)
        } else if (N <= 8) {
            DBSR_FUSE(8)
        } else if (N == 14) {
            DBSR_FUSE(14)
        } else {
            DBSR_FUSE(16)
        }
#undef DBSR_FUSE
        DBSR_LAUNCH_CHECK();
        return 0;
    });
}

extern "C" int dbsr_fuse_partial(int B, int N, int hw, int c, int first_frame, dbsr_tensor logits, dbsr_tensor ref,
                                 dbsr_tensor oth, float* stats, void* stream) {
    DBSR_CHECK_ARG(stats && map_ok(logits) && map_ok(ref) && (N == 1 || map_ok(oth)), "fuse_partial: bad tensor");
    DBSR_CHECK_ARG(logits.dtype == ref.dtype && (N == 1 || oth.dtype == ref.dtype), "fuse_partial: dtype mismatch");
    DBSR_CHECK_ARG(B > 0 && N > 0 && hw > 0 && c % 4 == 0 && first_frame >= 0 && first_frame <= N,
                   "fuse_partial: B, N, hw > 0, c multiple of 4, first_frame in [0,N]");
    DBSR_CHECK_ARG(vec_ok(logits, 4) && vec_ok(ref, 4) && (N == 1 || vec_ok(oth, 4)), "fuse_partial: ld/c0 % 4");
    const int groups = c / 4;
    const long long total = (long long)B * hw * groups;
    return by_dtype(ref.dtype, [&](auto* tag) {
        using T = std::remove_pointer_t<decltype(tag)>;
        if (N > 16)
            hipLaunchKernelGGL(fuse_partial_any_kernel<T>, dim3(nblocks(total, 256)), dim3(256), 0,
                               (hipStream_t)stream, B, N, hw, groups, first_frame, logits, ref, oth, stats);
        else if (N <= 8)
            hipLaunchKernelGGL((fuse_partial_kernel<T, 8>), dim3(nblocks(total, 256)), dim3(256), 0, (hipStream_t)stream,
                               B, N, hw, groups, first_frame, logits, ref, oth, stats);
        else
            hipLaunchKernelGGL((fuse_partial_kernel<T, 16>), dim3(nblocks(total, 256)), dim3(256), 0,
                               (hipStream_t)stream, B, N, hw, groups, first_frame, logits, ref, oth, stats);
        DBSR_LAUNCH_CHECK();
        return 0;
    });
}

extern "C" int dbsr_fuse_relu_norm(int B, int N, int hw, int c, dbsr_tensor logits, dbsr_tensor ref, dbsr_tensor oth,
                                   dbsr_tensor fused, dbsr_tensor weights, void* stream) {
    DBSR_CHECK_ARG(map_ok(logits) && map_ok(ref) && map_ok(fused) && (N == 1 || map_ok(oth)), "fuse_relu_norm: bad tensor");
    DBSR_CHECK_ARG(logits.dtype == ref.dtype && fused.dtype == ref.dtype && (N == 1 || oth.dtype == ref.dtype),
                   "fuse_relu_norm: dtype mismatch");
    DBSR_CHECK_ARG(B > 0 && N > 0 && hw > 0 && c % 4 == 0, "fuse_relu_norm: B, N, hw > 0 and c a multiple of 4");
    DBSR_CHECK_ARG(vec_ok(logits, 4) && vec_ok(ref, 4) && vec_ok(fused, 4) && (N == 1 || vec_ok(oth, 4)),
                   "fuse_relu_norm: ld/c0 must be multiples of 4");
    if (weights.ptr) DBSR_CHECK_ARG(map_ok(weights) && vec_ok(weights, 4), "fuse_relu_norm: bad weights tensor");
    const int groups = c / 4;
    const long long total = (long long)B * hw * groups;
    return by_dtype(ref.dtype, [&](auto* tag) {
        using T = std::remove_pointer_t<decltype(tag)>;
        hipLaunchKernelGGL(fuse_relunorm_kernel<T>, dim3(nblocks(total, 256)), dim3(256), 0, (hipStream_t)stream, B, N,
                           hw, groups, logits, ref, oth, fused, weights);
        DBSR_LAUNCH_CHECK();
        return 0;
    });
}

extern "C" int dbsr_burst_mean(int B, int N, int hw, int c, dbsr_tensor in, dbsr_tensor out, void* stream) {
    DBSR_CHECK_ARG(map_ok(in) && map_ok(out) && in.dtype == out.dtype, "burst_mean: bad tensors");
    DBSR_CHECK_ARG(B > 0 && N > 0 && hw > 0 && c % 4 == 0 && vec_ok(in, 4) && vec_ok(out, 4),
                   "burst_mean: B, N, hw > 0, c and ld/c0 multiples of 4");
    const int groups = c / 4;
    const long long total = (long long)B * hw * groups;
    return by_dtype(in.dtype, [&](auto* tag) {
        using T = std::remove_pointer_t<decltype(tag)>;
        hipLaunchKernelGGL(burst_mean_kernel<T>, dim3(nblocks(total, 256)), dim3(256), 0, (hipStream_t)stream, B, N, hw,
                           groups, in, out);
        DBSR_LAUNCH_CHECK();
        return 0;
    });
}

extern "C" int dbsr_fuse_combine(int R, int B, int hw, int c, const float* stats, dbsr_tensor fused, void* stream) {
    DBSR_CHECK_ARG(stats && map_ok(fused) && R > 0 && B > 0 && hw > 0 && c % 4 == 0 && vec_ok(fused, 4),
                   "fuse_combine: bad arguments");
    const int groups = c / 4;
    const long long total = (long long)B * hw * groups;
    return by_dtype(fused.dtype, [&](auto* tag) {
        using T = std::remove_pointer_t<decltype(tag)>;
        hipLaunchKernelGGL((fuse_combine_kernel<T>), dim3(nblocks(total, 256)), dim3(256), 0, (hipStream_t)stream, R,
                           B, hw, groups, stats, fused);
        DBSR_LAUNCH_CHECK();
        return 0;
    });
}

namespace {
// NHWC (16-bit or fp32) -> fp32 NCHW, per image: out[img][c][p] = in[img][p][c].  64 pixels x 64 channels per
// block through a padded LDS tile: both the reads (channels of a pixel) and the writes (pixels of a channel)
// are coalesced.  The aux fusion weights in the reference's layout (merging.py:117-126 returns the fp32
// softmax [B,N,C,H,W]), materialised only when a caller reads them.
template <typename T>
__global__ __launch_bounds__(256) void nhwc_to_nchw_kernel(int hw, int C, dbsr_tensor in, float* __restrict__ out) {
    __shared__ float tile[64][65];
    const int img = blockIdx.z, p0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
    const T* src = img_ptr<T>(in, img);
    for (int i = threadIdx.x; i < 64 * 64; i += 256) {
        const int pl = i / 64, cl = i % 64;
        const int p = p0 + pl, c = c0 + cl;
        tile[pl][cl] = (p < hw && c < C) ? elem<T>::ld(src + (long long)p * in.ld + c) : 0.f;
    }
    __syncthreads();
    float* dst = out + (long long)img * C * hw;
    for (int i = threadIdx.x; i < 64 * 64; i += 256) {
        const int cl = i / 64, pl = i % 64;
        const int p = p0 + pl, c = c0 + cl;
        if (p < hw && c < C) dst[(long long)c * hw + p] = tile[pl][cl];
    }
}
}  // namespace

extern "C" int dbsr_nhwc_to_nchw_f32(int n, int hw, int c, dbsr_tensor in, float* out, void* stream) {
    DBSR_CHECK_ARG(map_ok(in) && out && n > 0 && hw > 0 && c > 0 && in.c0 + c <= in.ld, "nhwc_to_nchw: bad tensor");
    return by_dtype(in.dtype, [&](auto* tag) {
        using T = std::remove_pointer_t<decltype(tag)>;
        hipLaunchKernelGGL(nhwc_to_nchw_kernel<T>, dim3((unsigned)((hw + 63) / 64), (unsigned)((c + 63) / 64), (unsigned)n),
                           dim3(256), 0, (hipStream_t)stream, hw, c, in, out);
        DBSR_LAUNCH_CHECK();
        return 0;
    });
}

extern "C" int dbsr_merge_prep(int B, int N, int hw, int c, dbsr_tensor proj, dbsr_tensor out, void* stream) {
    DBSR_CHECK_ARG(map_ok(proj) && map_ok(out) && proj.dtype == out.dtype, "merge_prep: bad tensor");
    DBSR_CHECK_ARG(c % 8 == 0 && vec_ok(proj, 8) && vec_ok(out, 8) && out.c0 + 2 * c <= out.ld, "merge_prep: layout");
    const long long total = (long long)B * N * hw * (c / 8);
    return by_dtype(out.dtype, [&](auto* tag) {
        using T = std::remove_pointer_t<decltype(tag)>;
        hipLaunchKernelGGL(merge_prep_kernel<T>, dim3(nblocks(total, 256)), dim3(256), 0, (hipStream_t)stream, B, N,
                           hw, c, proj, out);
        DBSR_LAUNCH_CHECK();
        return 0;
    });
}

extern "C" int dbsr_gauss_blur3(int n, int h, int w, int c, dbsr_tensor in, const float* k_host, dbsr_tensor out,
                                void* stream) {
    DBSR_CHECK_ARG(map_ok(in) && map_ok(out) && k_host && in.dtype == out.dtype, "blur: bad tensor");
    DBSR_CHECK_ARG(c % 8 == 0 && vec_ok(in, 8) && vec_ok(out, 8), "blur: layout");
    K9 kk;
    for (int i = 0; i < 9; ++i) kk.k[i] = k_host[i];
    Blur3 kb;
    const bool sep = blur_separable(k_host, kb);
    const long long total = (long long)n * ((h + BLUR_ROWS - 1) / BLUR_ROWS) * w * (c / 8);
    return by_dtype(in.dtype, [&](auto* tag) {
        using T = std::remove_pointer_t<decltype(tag)>;
        // 16-bit, separable: load-first strips of 8 rows (dec.blur 38.0 -> 31.4 us; strips of 4 rows: 32.5 us)
        if constexpr (sizeof(T) == 2) {
            if (!sep) {
                hipLaunchKernelGGL(blur3_kernel<T>, dim3(nblocks(total, 256)), dim3(256), 0, (hipStream_t)stream, n,
                                   h, w, c / 8, in, kk, out);
                DBSR_LAUNCH_CHECK();
                return 0;
            }
            hipLaunchKernelGGL((blur3_h16_kernel<T, BLUR_ROWS>), dim3(nblocks(total, 256)), dim3(256), 0,
                               (hipStream_t)stream, n, h, w, c / 8, in, kb, out);
        } else
            hipLaunchKernelGGL(blur3_kernel<T>, dim3(nblocks(total, 256)), dim3(256), 0, (hipStream_t)stream, n, h,
                               w, c / 8, in, kk, out);
        DBSR_LAUNCH_CHECK();
        return 0;
    });
}
