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
#include "conv_core.hpp"

#include <algorithm>
#include <type_traits>
#include <cstdlib>
#include <cstring>
#include <vector>

using namespace dbsr;

namespace {

int g_tiled_enabled = 1;

// The geometry every dispatch decision is taken on: `d` itself, or (d->plan_h > 0) `d` as if its image were
// plan_h output rows tall -- a frame-sharded rank's decoder slab then takes the whole image's kernels, tiles
// and K split, so each of its output pixels is summed in the whole image's order (dbsr_hip.h: plan_h)
const dbsr_conv_desc* sel_view(const dbsr_conv_desc* d, dbsr_conv_desc& v) {
    if (d->plan_h <= 0 || d->plan_h == d->out_h) return d;
    v = *d;
    v.in_h = d->in_h + (d->plan_h - d->out_h) * d->stride;
    v.out_h = d->plan_h;
    return &v;
}

// The channel a lane's 16-B run of a residual / gate load starts at, for a cout tile whose lanes may lie past
// cout (a partial tile): such lanes read the tile's first run instead (their values are never stored).  The
// kernels address through these functions and the host reach model (conv_lane_reach, dbsr_conv_lane_reach)
// enumerates the same lanes through them, so what the model checks is what the kernels load.
// pipelined kernel: lane (h, g) of the cout tile at cb holds couts cb + 32h + 8g .. +7
__host__ __device__ __forceinline__ int pipe_lane_ch(int cb, int h, int g, int cout) {
    const int c = cb + 32 * h + 8 * g;
    return c < cout ? c : cb;
}
// weight-stationary kernel: wave wc, lane group g of the cout tile at ctb holds couts ctb + 32wc + 8g .. +7
__host__ __device__ __forceinline__ int ws_lane_ch(int ctb, int wc, int g, int cout) {
    const int c = ctb + 32 * wc + 8 * g;
    return c < cout ? c : ctb;
}

// bias of output channels co..co+3, loaded unconditionally from clamped indices (a per-element
// conditional load makes hipcc branch and wait vmcnt(0) per element); 0 past cout or without bias
__device__ __forceinline__ f32x4_t load_bias4(const ConvK& k, int co) {
    f32x4_t b = {0.f, 0.f, 0.f, 0.f};
    if (k.bias) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float v = k.bias[min(co + r, k.cout - 1)];
            b[r] = co + r < k.cout ? v : 0.f;
        }
    }
    return b;
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
                q.x = H16<T>::pack(v[0], v[1]);
                q.y = H16<T>::pack(v[2], v[3]);
                *(uint2*)y = q;
            } else {
                *(float4*)y = make_float4(v[0], v[1], v[2], v[3]);
            }
        } else {
            for (int r = 0; r < nvalid; ++r) elem<T>::st(y + r, v[r]);
        }
    }
}

// bias + act (+ residual + post-act) of one pixel's 4 consecutive output channels, stored per out_mode
template <typename T>
__device__ __forceinline__ void epilogue_px(const ConvK& k, int p, int co, const f32x4_t& a, const f32x4_t& b) {
    const int hw = k.out_h * k.out_w;
    const int f = p / hw, rr = p - f * hw;
    const int oy = rr / k.out_w, ox = rr - oy * k.out_w;
    const int nvalid = min(4, k.cout - co);
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = apply_act(a[r] + b[r], k.act);
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
        if (k.gt) {
            const long long goff = map_frame(k.gm, f) * k.g_is + (long long)rr * k.g_ld + k.g_c0 + co;
            for (int r = 0; r < nvalid; ++r) {
                const float gv = k.y_f32 ? ((const float*)k.gt)[goff + r] : elem<T>::ld((const T*)k.gt + goff + r);
                v[r] = gv > 0.f ? v[r] : 0.f;
            }
        }
        store4<T>(k, map_frame(k.ym, f) * k.y_is + (long long)rr * k.y_ld + k.y_c0 + co, v, nvalid);
    } else if (k.out_mode == DBSR_OUT_SHUFFLE) {
        const int s = k.shuffle, sub = co / k.cps, c = co - sub * k.cps;
        const int Y = oy * s + sub / s, X = ox * s + sub % s;
        const long long off = map_frame(k.ym, f) * k.y_is + ((long long)Y * (k.out_w * s) + X) * k.y_ld + k.y_c0 + c;
        store4<T>(k, off, v, nvalid);
    } else {   // NCHW fp32
        float* y = (float*)k.y + map_frame(k.ym, f) * k.y_is + (long long)co * hw + rr;
        for (int r = 0; r < nvalid; ++r) y[(long long)r * hw] = v[r];
    }
}

template <typename T, int MT, int NT, typename XT = T>
__global__ __launch_bounds__(256) void conv2d_kernel(ConvK k) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int kgl = lane >> 4, col = lane & 15;
    const int hw = k.out_h * k.out_w;
    const int p_base = blockIdx.x * (4 * NT * 16) + wave * (NT * 16);
    const int c_base = blockIdx.y * (MT * 16);

    const XT* xb[NT];
    int iy0[NT], ix0[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const int p = p_base + j * 16 + col;
        if (p < k.npix) {
            const int f = p / hw, rr = p - f * hw;
            const int oy = rr / k.out_w, ox = rr - oy * k.out_w;
            xb[j] = (const XT*)k.x + map_frame(k.xm, f) * k.x_is;
            iy0[j] = oy * k.stride - k.pad;
            ix0[j] = ox * k.stride - k.pad;
        } else {
            xb[j] = (const XT*)k.x;
            iy0[j] = -(1 << 28);
            ix0[j] = 0;
        }
    }
    const T* wr[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) wr[i] = (const T*)k.w + (long long)(c_base + i * 16 + col) * k.Kp + kgl * 8;
    f32x4_t bias[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) bias[i] = load_bias4(k, c_base + i * 16 + kgl * 4);

    f32x4_t acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    // this block's K slice [ks0, ks1) (whole K without split)
    const int nks_all = k.KGp >> 2;
    const int ks0 = (int)((long long)nks_all * blockIdx.z / k.ksplit);
    const int ks1 = (int)((long long)nks_all * (blockIdx.z + 1) / k.ksplit);
    // k-group decode of the next k-step to load, advanced incrementally by 4 per k-step
    int tap = (ks0 * 4 + kgl) / k.CG;
    int cg = (ks0 * 4 + kgl) - tap * k.CG;
    int ky = tap / k.kw, kx = tap - (tap / k.kw) * k.kw;
    auto load = [&](int ks, Frag<T> (&a)[MT], Frag<T> (&b)[NT]) {
        const bool kval = ks * 4 + kgl < k.KG;
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
        cg += 4;
        while (cg >= k.CG) {
            cg -= k.CG;
            if (++kx == k.kw) { kx = 0; ++ky; }
        }
    };
    auto compute = [&](const Frag<T> (&a)[MT], const Frag<T> (&b)[NT]) {
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int j = 0; j < NT; ++j) acc[i][j] = mma(a[i], b[j], acc[i][j]);
    };
    // (a one-k-step register prefetch was measured slower here: it cost occupancy on the large 1x1
    // convs without helping the latency-bound tiny ones)
    for (int ks = ks0; ks < ks1; ++ks) {
        Frag<T> a0[MT], b0[NT];
        load(ks, a0, b0);
        compute(a0, b0);
    }

    // staged epilogue (bf16, plain NHWC, cout % 8 == 0): bias + act into a per-wave LDS tile, then each
    // lane stores 16 B of a pixel row (MT*32 B per pixel), so a store instruction covers whole rows
    // instead of the per-lane path's 8-B pieces scattered over 16 pixel rows (that path ran the Cin<=8
    // input convs at ~1 TB/s)
    if constexpr (sizeof(T) == 2 && sizeof(XT) == 2 && MT * NT >= 2) {
        if (k.stage_epi) {
            constexpr int PITCH = MT * 16 + 8;                     // bf16 per LDS row (+16 B: spreads banks)
            constexpr int LPR = MT * 2;                            // lanes per pixel row (16 B each)
            constexpr int RPI = 64 / LPR;                          // rows per store instruction
            __shared__ __attribute__((aligned(16))) uint16_t stile[4][NT * 16 * PITCH];
            uint16_t* st = stile[wave];
#pragma unroll
            for (int j = 0; j < NT; ++j)
#pragma unroll
                for (int i = 0; i < MT; ++i) {
                    uint2 q;
                    q.x = H16<T>::pack(apply_act(acc[i][j][0] + bias[i][0], k.act), apply_act(acc[i][j][1] + bias[i][1], k.act));
                    q.y = H16<T>::pack(apply_act(acc[i][j][2] + bias[i][2], k.act), apply_act(acc[i][j][3] + bias[i][3], k.act));
                    *(uint2*)(st + (j * 16 + col) * PITCH + i * 16 + kgl * 4) = q;
                }
            __syncthreads();
            const int hw2 = k.out_h * k.out_w;
            const int ch = (lane % LPR) * 8;
#pragma unroll
            for (int it = 0; it < NT * 16 / RPI; ++it) {
                const int r = it * RPI + lane / LPR;
                const int p = p_base + r;
                if (p < k.npix && c_base + ch < k.cout) {
                    const int f = p / hw2, rr = p - f * hw2;
                    *(u32x4_t*)((T*)k.y + map_frame(k.ym, f) * k.y_is + (long long)rr * k.y_ld + k.y_c0 + c_base + ch) =
                        *(const u32x4_t*)(st + r * PITCH + ch);
                }
            }
            return;
        }
    }
    // epilogue: bias, activation, residual, post-activation, store (or fp32 partials under split-K)
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const int p = p_base + j * 16 + col;
        if (p >= k.npix) continue;
#pragma unroll
        for (int i = 0; i < MT; ++i) {
            const int co = c_base + i * 16 + kgl * 4;
            if (co >= k.cout) continue;
            if (k.ksplit > 1)
                *(f32x4_t*)(k.ws + ((long long)blockIdx.z * k.npix + p) * k.cw + co) = acc[i][j];
            else
                epilogue_px<T>(k, p, co, acc[i][j], bias[i]);
        }
    }
}

// split-K finalize: sum the K-slice partials in slice order (deterministic), then the normal epilogue
template <typename T>
__global__ __launch_bounds__(256) void conv_splitk_finalize(ConvK k) {
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const int groups = k.cw / 4;
    if (idx >= (long long)k.npix * groups) return;
    const int p = (int)(idx / groups), co = (int)(idx % groups) * 4;
    if (co >= k.cout) return;
    f32x4_t a = {0.f, 0.f, 0.f, 0.f};
    for (int z = 0; z < k.ksplit; ++z) a += *(const f32x4_t*)(k.ws + ((long long)z * k.npix + p) * k.cw + co);
    epilogue_px<T>(k, p, co, a, load_bias4(k, co));
}

// ------------------------------------------------------------------------------------------------
// Narrow-output 3x3 conv over a long K, 16-bit, cout <= 4 (PWC-Net's 2-channel flow head, pwcnet.py:156
// netFlow: K = 9 x 565 at level 2).  The tiled kernel runs it on 32-cout tiles in 32-channel chunks
// behind two barriers each: 27 us for 0.5 GFLOP.  Block = 4 waves on a 16 x 4-pixel tile (wave w: tile
// row w, one 16x16x32 MFMA per (tap, 32 channels); A rows >= cout are the packer's zero padding).  K moves
// in 64-channel chunks: the chunk's (6 x 18)-pixel halo (whole 128-B pixel pieces) and its 4 weight rows
// go global -> registers -> one of two LDS buffers, the next chunk's loads in flight while the current
// one is multiplied: 19.6 us.
// Measured and not kept: an MFMA wave streaming its K straight from L2 (16 pixels x 64 B per load,
// 62 us); lanes over the input channels with v_dot2 (26 us); a block per 16-pixel row with K split over
// its 4 waves, each staging its own chunks (23.6 us; the refiner's 32-channel output conv 12.5 us
// against 5.3 us tiled, so convs with cin < 256 stay on the tiled kernel); two chunks in flight here
// (two register sets) 21.2 us.
// ------------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void conv3x3_narrow_kernel(ConvK k, int tiles_x, int tiles_y) {
    constexpr int TW = 16, TH = 4, HX = TW + 2, NQ = HX * (TH + 2);     // 108 halo pixels
    constexpr int GPC = 8;                                               // 8-channel groups per chunk
    constexpr int NCO = 4;                                               // weight rows staged
    constexpr int HALO_ITEMS = NQ * GPC, W_ITEMS = NCO * 9 * GPC, ITEMS = HALO_ITEMS + W_ITEMS;
    constexpr int PER = (ITEMS + 255) / 256;
    constexpr int PITCH = GPC + 1;                                       // 16-B slots per halo pixel (+1: banks)
    constexpr int BUF = NQ * PITCH + W_ITEMS;                            // 16-B slots per buffer
    __shared__ __attribute__((aligned(16))) u32x4_t lds[2][BUF];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int col = lane & 15, kgl = lane >> 4;
    int b = blockIdx.x;
    const int tx = b % tiles_x; b /= tiles_x;
    const int ty = b % tiles_y;
    const int f = b / tiles_y;
    const T* xb = (const T*)k.x + map_frame(k.xm, f) * k.x_is;
    const int y0 = ty * TH - 1, x0 = tx * TW - 1;
    const int nchunk = (k.CG + GPC - 1) / GPC;

    u32x4_t r[PER];
    auto load = [&](int c) {
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int it = tid + 256 * i;
            u32x4_t v = {0u, 0u, 0u, 0u};
            if (it < HALO_ITEMS) {
                const int q = it / GPC, gg = it - q * GPC;
                const int hy = q / HX, hx = q - hy * HX;
                const int iy = y0 + hy, ix = x0 + hx, g = c * GPC + gg;
                if (g < k.CG && (unsigned)iy < (unsigned)k.in_h && (unsigned)ix < (unsigned)k.in_w)
                    v = *(const u32x4_t*)(xb + ((long long)iy * k.in_w + ix) * k.x_ld + g * 8);
            } else if (it < ITEMS) {
                const int wi = it - HALO_ITEMS;
                const int co = wi / (9 * GPC), rest = wi - co * (9 * GPC);
                const int tap = rest / GPC, gg = rest - tap * GPC, g = c * GPC + gg;
                if (g < k.CG) v = *(const u32x4_t*)((const T*)k.w + (long long)co * k.Kp + (tap * k.CG + g) * 8);
            }
            r[i] = v;
        }
    };
    auto put = [&](int buf) {
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int it = tid + 256 * i;
            if (it < HALO_ITEMS) {
                const int q = it / GPC, gg = it - q * GPC;
                lds[buf][q * PITCH + gg] = r[i];
            } else if (it < ITEMS) {
                lds[buf][NQ * PITCH + (it - HALO_ITEMS)] = r[i];
            }
        }
    };
    f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
    load(0);
    put(0);
    __syncthreads();
    for (int c = 0; c < nchunk; ++c) {
        if (c + 1 < nchunk) load(c + 1);
        const u32x4_t* L = lds[c & 1];
        const int gcount = min(GPC, k.CG - c * GPC);                     // 8, or 4 in a 32-channel tail chunk
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
            const int ky = tap / 3, kx = tap % 3;
            const int q = (wave + ky) * HX + col + kx;
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                if (s * 4 >= gcount) break;
                Frag<T> A, B;
                B.v = __builtin_bit_cast(bf16x8_t, L[q * PITCH + s * 4 + kgl]);
                if (col < NCO) A.v = __builtin_bit_cast(bf16x8_t, L[NQ * PITCH + (col * 9 + tap) * GPC + s * 4 + kgl]);
                else A.zero();
                acc = mma(A, B, acc);
            }
        }
        if (c + 1 < nchunk) put((c + 1) & 1);
        __syncthreads();
    }
    const int oy = ty * TH + wave, ox = tx * TW + col;
    if (kgl != 0 || oy >= k.out_h || ox >= k.out_w) return;
    epilogue_px<T>(k, (f * k.out_h + oy) * k.out_w + ox, 0, acc, load_bias4(k, 0));
}

// row layout [cout_pad][Kp] -> chunk-major pieces [cout_pad/16][chunk][tap][g][16 co][8] (3x3, cin > 16);
// within each tile of P = (cout <= 32 ? 32 : 64) couts, row col of 16-cout block blk holds physical cout
// pipe_cout_perm(blk, col) (the pipelined kernel's 8-consecutive-couts-per-lane epilogue order)
__host__ __device__ __forceinline__ int pipe_cout_perm(int i, int m) {
    return 32 * (i >> 1) + 8 * (m >> 2) + 4 * (i & 1) + (m & 3);
}
__global__ void pack_weights_pipe_kernel(const bf16_t* __restrict__ rows, int CG, int Kp, int P, long long total,
                                         bf16_t* __restrict__ out) {
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= total) return;
    const int e = (int)(idx & 7), col = (int)((idx >> 3) & 15), g = (int)((idx >> 7) & 3);
    long long piece = idx >> 9;
    const int tap = (int)(piece % 9); piece /= 9;
    const int nch = CG / 4;
    const int c = (int)(piece % nch);
    const long long cb16 = piece / nch;
    const int bpt = P / 16;                                   // 16-cout blocks per tile
    const long long co = (cb16 / bpt) * P + pipe_cout_perm((int)(cb16 % bpt), col);
    out[idx] = rows[co * Kp + (tap * CG + c * 4 + g) * 8 + e];
}

__global__ void pack_weights_kernel(const float* __restrict__ w, const float* __restrict__ bias, int cout, int cin,
                                    int kh, int kw, int CG, int KG, int Kp, int cout_pad, int shuffle, int dtype,
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
    if (dtype == DBSR_BF16)
        ((bf16_t*)out)[idx] = f2bf(v);
    else if (dtype == DBSR_F16)
        ((f16_t*)out)[idx] = (f16_t)v;
    else
        ((float*)out)[idx] = v;
    if (bias_out && kk == 0 && co < cout) bias_out[co] = bias ? bias[co_src] : 0.f;
}

// ------------------------------------------------------------------------------------------------
// Batched repack (dbsr_conv_pack_weights_batch): one launch over every job's packed elements, block b -> the job
// whose [blk0, next blk0) holds b.  Each element is computed from the fp32 source exactly as pack_weights_kernel
// (the row layout) and pack_weights_pipe_kernel (the chunk-major copy, which reads the row layout's element back)
// compute it, so the result is bitwise theirs; a transposed job reads the dgrad conv's weight straight from the
// source conv (dgrad_weights_kernel's transpose + flip, then rows [lo, lo + cout) of it).
// ------------------------------------------------------------------------------------------------
struct PackGeom { int CG, KG, Kp, cout_pad; long long rows; bool pipe; };
__host__ __device__ inline PackGeom pack_geom(const dbsr_pack_job& j) {
    PackGeom g;
    g.CG = (j.cin <= 16 ? (j.cin + 7) / 8 * 8 : (j.cin + 31) / 32 * 32) / 8;
    g.KG = j.kh * j.kw * g.CG;
    g.Kp = (g.KG + 3) / 4 * 4 * 8;
    g.cout_pad = (j.cout + 63) / 64 * 64;
    g.rows = (long long)g.cout_pad * g.Kp;
    g.pipe = j.kh == 3 && j.kw == 3 && j.cin > 16 && (j.dtype == DBSR_BF16 || j.dtype == DBSR_F16);
    return g;
}

__device__ inline float pack_row_value(const dbsr_pack_job& j, const PackGeom& g, int co, int kk, int* co_src_out) {
    int co_src = co;
    if (j.shuffle > 1 && co < j.cout) {
        const int s2 = j.shuffle * j.shuffle, cps = j.cout / s2;
        const int sub = co / cps, c = co - sub * cps;
        co_src = c * s2 + sub;
    }
    *co_src_out = co_src;
    const int kg = kk >> 3, jj = kk & 7;
    if (co < j.cout && kg < g.KG) {
        const int tap = kg / g.CG, c = (kg - tap * g.CG) * 8 + jj;
        if (c < j.cin) {
            const int ky = tap / j.kw, kx = tap - ky * j.kw;
            if (j.transposed)       // dgrad conv: out channel o = source input channel lo + o, taps flipped
                return j.w[(((long long)c * j.src_cin + j.lo + co_src) * j.kh + (j.kh - 1 - ky)) * j.kw +
                           (j.kw - 1 - kx)];
            return j.w[(((long long)co_src * j.cin + c) * j.kh + ky) * j.kw + kx];
        }
    }
    return 0.f;
}

__global__ __launch_bounds__(256) void pack_weights_batch_kernel(const dbsr_pack_job* __restrict__ jobs, int n) {
    const long long b = blockIdx.x;
    int lo = 0, hi = n - 1;             // the last job with blk0 <= b
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (jobs[mid].blk0 <= b) lo = mid;
        else hi = mid - 1;
    }
    const dbsr_pack_job j = jobs[lo];
    const PackGeom g = pack_geom(j);
    const long long idx = (b - j.blk0) * 256 + threadIdx.x;
    int co, kk;
    if (idx < g.rows) {
        co = (int)(idx / g.Kp); kk = (int)(idx - (long long)co * g.Kp);
    } else if (g.pipe && idx < 2 * g.rows) {
        const long long p = idx - g.rows;
        const int e = (int)(p & 7), col = (int)((p >> 3) & 15), gg = (int)((p >> 7) & 3);
        long long piece = p >> 9;
        const int tap = (int)(piece % 9); piece /= 9;
        const int nch = g.CG / 4;
        const int c = (int)(piece % nch);
        const long long cb16 = piece / nch;
        const int P = j.cout <= 32 ? 32 : 64, bpt = P / 16;
        co = (int)((cb16 / bpt) * P + pipe_cout_perm((int)(cb16 % bpt), col));
        kk = (tap * g.CG + c * 4 + gg) * 8 + e;
    } else {
        return;
    }
    int co_src;
    const float v = pack_row_value(j, g, co, kk, &co_src);
    if (j.dtype == DBSR_BF16)
        ((bf16_t*)j.w_packed)[idx] = f2bf(v);
    else if (j.dtype == DBSR_F16)
        ((f16_t*)j.w_packed)[idx] = (f16_t)v;
    else
        ((float*)j.w_packed)[idx] = v;
    if (idx < g.rows && j.bias_out && kk == 0 && co < j.cout)
        j.bias_out[co] = (j.bias && !j.transposed) ? j.bias[co_src] : 0.f;
}

// ------------------------------------------------------------------------------------------------
// LDS-tiled 3x3 / stride 1 / pad 1 convolution for Cin % 32 == 0 (the ResNet trunks: encoder,
// weight predictor, decoder; ~2/3 of the forward's FLOPs).
//
// Block = 4 waves = WM output channels x a spatial tile of TH x 16 pixels of one frame (each wave
// owns WN = 4*16*(TH/4) ... i.e. TH/4 rows of 16 pixels).  Per 32-channel input chunk the block
// stages into LDS (a) the (TH+2) x 18 halo tile and (b) the chunk's weights for all 9 taps, then
// every wave runs 9 taps x (WM/16) x (WN/16) MFMAs reading both operands with ds_read_b128.
// The next chunk's global loads are issued into registers before the current chunk's MFMAs and
// written to LDS after them (async-stage split), with one LDS buffer and two barriers per chunk
// (two blocks per CU overlap each other's barriers).
//
// LDS images are [k-group plane][row][16 B] with each plane a multiple of 256 B: any 16
// consecutive pixels (or output channels) of one plane then cover all 64 banks, for every tap
// shift, under ds_read_b128's lane groups ({0-3,12-15,20-27}, ...), because lane l reads row
// (l&15) of plane (l>>4) -- conflict-free by construction (conv tiling).
// Blocks are ordered so each XCD gets a contiguous range of (tile, cout-tile) pairs: the 8 cout
// tiles of a spatial tile and neighbouring tiles (shared halos) hit the same L2.
// ------------------------------------------------------------------------------------------------
template <typename T, int WM, int WN, int D>
struct TileCfg {
    static constexpr int TW = 16, TH = 4 * WN / 16, HWD = TW + 2 * D, HHT = TH + 2 * D;
    static constexpr int NQ = HHT * HWD;                      // halo pixels
    static constexpr int NQP = (NQ + 63) / 64 * 64;           // plane length (pixels): whole 1-KiB pieces
    static constexpr int HALVES = sizeof(T) / 2;              // 16-B halves per k-group (bf16 1, f32 2)
    static constexpr int PLANES = 4 * HALVES;                 // (k-group, half)
    static constexpr int IN_ITEMS = PLANES * (NQP / 64);      // 1-KiB LDS-DMA pieces of the halo tile
    static constexpr int W_ITEMS = 9 * (WM / 16) * HALVES;    // 1-KiB pieces: (tap, 16-cout block, half)
    static constexpr int IN_U4 = PLANES * NQP, W_U4 = W_ITEMS * 64;
    static constexpr int NPIX = 4 * WN;                       // output pixels per tile
    static constexpr int OSTR = WM * (int)sizeof(T) + 16;     // staged-output pixel stride (bytes)
};

// zero page for halo pixels outside the frame (LDS-DMA cannot write zeros itself); those lanes' source
// pointers advance by the chunk offset like every other lane, so the page covers 32 KiB of chunks
constexpr int ZERO_PAGE_BYTES = 32768;
__device__ __attribute__((aligned(16))) u32x4_t g_dbsr_zero16[ZERO_PAGE_BYTES / 16];

__device__ __forceinline__ void glds16(const void* src, u32x4_t* lds_piece) {
    __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_piece, 16, 0, 0);
}

// buffer-resource LDS-DMA helpers (BUF_OOB, buf_rsrc, blds16): common.hpp

template <typename T, int WM, int WN, int D>
__global__ __launch_bounds__(256, 2) void conv3x3_tiled_kernel(ConvK k, int tiles_x, int tiles_y, int nct,
                                                               int nblocks) {
    using C = TileCfg<T, WM, WN, D>;
    DBSR_OWN_SIMDS();
    // the configurations that need more than 256 registers (accumulation registers: fp32 tiles, bf16
    // dilation 8) run one wave per SIMD; they take the whole file too (test_capi checks every
    // pipelined / tiled kernel's allocation)
    if constexpr ((sizeof(T) == 4 && (WM == 64 || WN >= 64)) || (D == 8 && WN >= 64)) asm volatile("" ::: "a255");
    static_assert((C::IN_U4 + C::W_U4) * 16 <= 160 * 1024, "LDS tile exceeds 160 KiB");
    static_assert(C::NPIX * C::OSTR <= (C::IN_U4 + C::W_U4) * 16, "output staging must fit the LDS tile");
    // One LDS array (a second __shared__ object can de-pipeline LDS-DMA: cdna_hip_programming.md §5 item 4a)
    __shared__ __attribute__((aligned(16))) u32x4_t lds[C::IN_U4 + C::W_U4];
    u32x4_t* lin = lds;                 // [k-group][half][NQP halo pixels] x 16 B  (planar)
    u32x4_t* lw = lds + C::IN_U4;       // [tap][cout block][half][k-group][16 co] x 16 B

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane >> 4, col = lane & 15;

    // XCD-grouped block order (bijective; cdna_hip_programming.md §5 'XCD swizzle')
    const int bid = blockIdx.x;
    const int xcd = bid & 7, q8 = nblocks >> 3, r8 = nblocks & 7;
    const int lin_id = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    const int ct = lin_id % nct;
    int tile = lin_id / nct;
    const int tx = tile % tiles_x; tile /= tiles_x;
    const int ty = tile % tiles_y;
    const int f = tile / tiles_y;
    const int y0 = ty * C::TH, x0 = tx * C::TW;
    const int c_base = ct * WM;

    const T* xf = (const T*)k.x + map_frame(k.xm, f) * k.x_is;
    const int nchunks = k.CG / 4;
    f32x4_t bias[WM / 16];
#pragma unroll
    for (int i = 0; i < WM / 16; ++i) bias[i] = load_bias4(k, c_base + i * 16 + g * 4);

    // Stage one 32-channel chunk by LDS-DMA (16 B per lane, lane-linear destination):
    //  halo: one piece = 64 consecutive pixels of one (k-group, half) plane; pixels outside the frame
    //        read the zero page.  Planes are 1-KiB multiples, so the 16 pixels a ds_read_b128 lane group
    //        reads are 16 distinct bank slots for every tap shift (conflict-free), and a pixel's
    //        address is linear in the tap shift (immediate-offset reads).
    //  weights: one piece = 16 output channels x 4 k-groups of one tap (16 x 64 contiguous bytes).
    // Per-lane source pointers of every piece this wave stages, computed once per block: a chunk only
    // adds chunk * 32 elements (the address math is otherwise VALU work on every chunk).
    constexpr int IN_PER = (C::IN_ITEMS + 3) / 4, W_PER = (C::W_ITEMS + 3) / 4;
    const char* in_src[IN_PER];
    const char* w_src[W_PER];
#pragma unroll
    for (int it = 0; it < IN_PER; ++it) {
        const int item = wave + 4 * it;
        const int plane = item / (C::NQP / 64), seg = item % (C::NQP / 64);
        const int gg = plane / C::HALVES, h = plane % C::HALVES;
        const int q = seg * 64 + lane;
        const char* src = (const char*)g_dbsr_zero16;
        if (item < C::IN_ITEMS && q < C::NQ) {
            const int iy = y0 - D + q / C::HWD, ix = x0 - D + q % C::HWD;
            if ((unsigned)iy < (unsigned)k.in_h && (unsigned)ix < (unsigned)k.in_w)
                src = (const char*)(xf + ((long long)iy * k.in_w + ix) * k.x_ld + gg * 8 + h * 4);
        }
        in_src[it] = src;
    }
#pragma unroll
    for (int it = 0; it < W_PER; ++it) {
        const int item = wave + 4 * it;
        const int h = item % C::HALVES, rest = item / C::HALVES;
        const int cb = rest % (WM / 16), tap = rest / (WM / 16);
        const int co = c_base + cb * 16 + col;
        w_src[it] = (const char*)((const T*)k.w + (long long)co * k.Kp + (tap * k.CG + g) * 8 + h * 4);
    }
    // Stage one 32-channel chunk by LDS-DMA (16 B per lane, lane-linear destination):
    //  halo: one piece = 64 consecutive pixels of one (k-group, half) plane; pixels outside the frame
    //        read the zero page.  Planes are 1-KiB multiples, so the 16 pixels a ds_read_b128 lane group
    //        reads are 16 distinct bank slots for every tap shift (conflict-free), and a pixel's
    //        address is linear in the tap shift (immediate-offset reads).
    //  weights: one piece = 16 output channels x 4 k-groups of one tap (16 x 64 contiguous bytes).
    auto issue = [&](int chunk) {
        const int off = chunk * 32 * (int)sizeof(T);
#pragma unroll
        for (int it = 0; it < IN_PER; ++it)
            if (wave + 4 * it < C::IN_ITEMS) glds16(in_src[it] + off, lin + (wave + 4 * it) * 64);
#pragma unroll
        for (int it = 0; it < W_PER; ++it)
            if (wave + 4 * it < C::W_ITEMS) glds16(w_src[it] + off, lw + (wave + 4 * it) * 64);
    };

    f32x4_t acc[WM / 16][WN / 16];
#pragma unroll
    for (int i = 0; i < WM / 16; ++i)
#pragma unroll
        for (int j = 0; j < WN / 16; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    const int row0 = wave * (WN / 16);
    // lane-dependent LDS bases; every tap/fragment offset below is a compile-time immediate
    const u32x4_t* lb_in = lin + (g * C::HALVES) * C::NQP + row0 * C::HWD + col;
    const u32x4_t* lb_w = lw + g * 16 + col;
    auto read_frags = [&](int tap, Frag<T> (&a)[WM / 16], Frag<T> (&b)[WN / 16]) {
        const int ky = tap / 3, kx = tap % 3;
#pragma unroll
        for (int i = 0; i < WM / 16; ++i) {
            const u32x4_t* p = lb_w + ((tap * (WM / 16) + i) * C::HALVES) * 64;
            if constexpr (sizeof(T) == 2) {
                a[i].v = __builtin_bit_cast(bf16x8_t, p[0]);
            } else {
                a[i].a = __builtin_bit_cast(float4, p[0]);
                a[i].b = __builtin_bit_cast(float4, p[64]);
            }
        }
#pragma unroll
        for (int j = 0; j < WN / 16; ++j) {
            const u32x4_t* p = lb_in + (j + ky * D) * C::HWD + kx * D;
            if constexpr (sizeof(T) == 2) {
                b[j].v = __builtin_bit_cast(bf16x8_t, p[0]);
            } else {
                b[j].a = __builtin_bit_cast(float4, p[0]);
                b[j].b = __builtin_bit_cast(float4, p[C::NQP]);
            }
        }
    };
    auto mfmas = [&](const Frag<T> (&a)[WM / 16], const Frag<T> (&b)[WN / 16]) {
#pragma unroll
        for (int i = 0; i < WM / 16; ++i)
#pragma unroll
            for (int j = 0; j < WN / 16; ++j) acc[i][j] = mma(a[i], b[j], acc[i][j]);
    };

    // split-K (launch_tiled with k.ksplit > 1: blockIdx.y = the K slice): this block's whole 32-channel chunks
    const int ksl = (int)gridDim.y, kz = (int)blockIdx.y;
    const int ch0 = nchunks * kz / ksl, ch1 = nchunks * (kz + 1) / ksl;
    for (int chunk = ch0; chunk < ch1; ++chunk) {
        issue(chunk);
        dma_barrier();                   // vmcnt(0) for the LDS-DMA + barrier
        // taps software-pipelined through two fragment sets: tap t+1's ds_reads are in flight during
        // tap t's MFMAs
        Frag<T> a0[WM / 16], b0[WN / 16], a1[WM / 16], b1[WN / 16];
        read_frags(0, a0, b0);
#pragma unroll
        for (int tap = 0; tap < 9; tap += 2) {
            if (tap + 1 < 9) read_frags(tap + 1, a1, b1);
            mfmas(a0, b0);
            if (tap + 1 < 9) {
                if (tap + 2 < 9) read_frags(tap + 2, a0, b0);
                mfmas(a1, b1);
            }
        }
        __syncthreads();                 // all waves done reading before the next chunk lands
    }

    if (ksl > 1) {
        // the slice's fp32 partial sums, [slice][pixel][cw], summed in slice order (then bias, act, residual, gate)
        // by conv_splitk_finalize
#pragma unroll
        for (int j = 0; j < WN / 16; ++j) {
            const int oy = y0 + row0 + j, ox = x0 + col;
            if (oy >= k.out_h || ox >= k.out_w) continue;
            const long long p = ((long long)f * k.out_h + oy) * k.out_w + ox;
#pragma unroll
            for (int i = 0; i < WM / 16; ++i) {
                const int co = c_base + i * 16 + g * 4;
                if (co < k.cout) *(f32x4_t*)(k.ws + ((long long)kz * k.npix + p) * k.cw + co) = acc[i][j];
            }
        }
        return;
    }
    // ---- epilogue: bias + act into an LDS [pixel][cout] tile, then whole 16-B rows per lane ----
    const bool staged = !k.y_f32 && k.y_ld % 8 == 0 && k.y_c0 % 8 == 0 && k.cout % 8 == 0 &&
                        (!k.r || (k.r_ld % 8 == 0 && k.r_c0 % 8 == 0)) && (!k.gt || (k.g_ld % 8 == 0 && k.g_c0 % 8 == 0));
    if (staged) {
        char* ob = (char*)lds;
#pragma unroll
        for (int j = 0; j < WN / 16; ++j) {
            const int pix = (row0 + j) * C::TW + col;
#pragma unroll
            for (int i = 0; i < WM / 16; ++i) {
                const int co = i * 16 + g * 4;
                float v[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = apply_act(acc[i][j][r] + bias[i][r], k.act);
                if constexpr (sizeof(T) == 2) {
                    uint2 q;
                    q.x = H16<T>::pack(v[0], v[1]);
                    q.y = H16<T>::pack(v[2], v[3]);
                    *(uint2*)(ob + pix * C::OSTR + co * 2) = q;
                } else {
                    *(float4*)(ob + pix * C::OSTR + co * 4) = make_float4(v[0], v[1], v[2], v[3]);
                }
            }
        }
        __syncthreads();
        constexpr int EPC = 16 / (int)sizeof(T);                 // elements per 16-B chunk
        constexpr int CPP = WM / EPC;                            // chunks per pixel
        constexpr int NCH = C::NPIX * CPP;
        constexpr int PER = (NCH + 255) / 256;
        const int cvalid = min(WM, k.cout - c_base);
        const T* rbase = k.r ? (const T*)k.r + map_frame(k.rm, f) * k.r_is + k.r_c0 + c_base : nullptr;
        const T* gbase = k.gt ? (const T*)k.gt + map_frame(k.gm, f) * k.g_is + k.g_c0 + c_base : nullptr;
        T* ybase = (T*)k.y + map_frame(k.ym, f) * k.y_is + k.y_c0 + c_base;
        u32x4_t rv[PER];
        long long off[PER];
        bool ok[PER];
#pragma unroll
        for (int e = 0; e < PER; ++e) {
            const int c = threadIdx.x + e * 256;
            const int pix = c / CPP, sc = c % CPP;
            const int oy = y0 + pix / C::TW, ox = x0 + pix % C::TW;
            ok[e] = c < NCH && oy < k.out_h && ox < k.out_w && sc * EPC < cvalid;
            off[e] = ok[e] ? ((long long)oy * k.out_w + ox) : 0;
        }
        if (rbase) {        // uniform; every residual load issued back to back (clamped address, no branches)
#pragma unroll
            for (int e = 0; e < PER; ++e) {
                const int sc = (threadIdx.x + e * 256) % CPP;
                rv[e] = *(const u32x4_t*)(rbase + off[e] * k.r_ld + (ok[e] ? sc * EPC : 0));
            }
        }
#pragma unroll
        for (int e = 0; e < PER; ++e) {
            if (!ok[e]) continue;
            const int c = threadIdx.x + e * 256;
            const int pix = c / CPP, sc = c % CPP;
            u32x4_t val = *(const u32x4_t*)(ob + pix * C::OSTR + sc * 16);
            if (rbase) {
                if constexpr (sizeof(T) == 2) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const float lo = H16<T>::lo(val[q]) + H16<T>::lo(rv[e][q]);
                        const float hi = H16<T>::hi(val[q]) + H16<T>::hi(rv[e][q]);
                        val[q] = H16<T>::pack(apply_act(lo, k.post_act), apply_act(hi, k.post_act));
                    }
                } else {
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        val[q] = __float_as_uint(apply_act(__uint_as_float(val[q]) + __uint_as_float(rv[e][q]),
                                                           k.post_act));
                }
            }
            if (gbase) {
                const u32x4_t gv = *(const u32x4_t*)(gbase + off[e] * k.g_ld + sc * EPC);
                if constexpr (sizeof(T) == 2) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const unsigned keep = (H16<T>::lo(gv[q]) > 0.f ? 0x0000ffffu : 0u) |
                                              (H16<T>::hi(gv[q]) > 0.f ? 0xffff0000u : 0u);
                        val[q] &= keep;
                    }
                } else {
#pragma unroll
                    for (int q = 0; q < 4; ++q) val[q] = __uint_as_float(gv[q]) > 0.f ? val[q] : 0u;
                }
            }
            *(u32x4_t*)(ybase + off[e] * k.y_ld + sc * EPC) = val;
        }
        return;
    }
    // generic epilogue (fp32 output of a bf16 conv, unaligned slices): per-lane fragments
#pragma unroll
    for (int j = 0; j < WN / 16; ++j) {
        const int oy = y0 + row0 + j, ox = x0 + col;
        if (oy >= k.out_h || ox >= k.out_w) continue;
        const int rr = oy * k.out_w + ox;
#pragma unroll
        for (int i = 0; i < WM / 16; ++i) {
            const int co = c_base + i * 16 + g * 4;
            if (co >= k.cout) continue;
            const int nvalid = min(4, k.cout - co);
            float v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = apply_act(acc[i][j][r] + bias[i][r], k.act);
            if (k.r) {
                const long long roff = map_frame(k.rm, f) * k.r_is + (long long)rr * k.r_ld + k.r_c0 + co;
                for (int r = 0; r < nvalid; ++r)
                    v[r] = apply_act(v[r] + (k.y_f32 ? ((const float*)k.r)[roff + r] : elem<T>::ld((const T*)k.r + roff + r)),
                                     k.post_act);
            }
            if (k.gt) {
                const long long goff = map_frame(k.gm, f) * k.g_is + (long long)rr * k.g_ld + k.g_c0 + co;
                for (int r = 0; r < nvalid; ++r) {
                    const float gv = k.y_f32 ? ((const float*)k.gt)[goff + r] : elem<T>::ld((const T*)k.gt + goff + r);
                    v[r] = gv > 0.f ? v[r] : 0.f;
                }
            }
            store4<T>(k, map_frame(k.ym, f) * k.y_is + (long long)rr * k.y_ld + k.y_c0 + co, v, nvalid);
        }
    }
}

template <typename T, int WM, int WN, int D>
int launch_tiled(const ConvK& k, int n_frames, hipStream_t s) {
    using C = TileCfg<T, WM, WN, D>;
    const int tiles_x = (k.out_w + C::TW - 1) / C::TW, tiles_y = (k.out_h + C::TH - 1) / C::TH;
    const int nct = (k.cout + WM - 1) / WM;
    const long long nb = (long long)n_frames * tiles_x * tiles_y * nct;
    if (nb >= (1LL << 31)) {
        dbsr_set_error("conv2d: grid too large");
        return DBSR_E_ARG;
    }
    hipLaunchKernelGGL((conv3x3_tiled_kernel<T, WM, WN, D>), dim3((unsigned)nb, (unsigned)k.ksplit), dim3(256), 0, s, k,
                       tiles_x, tiles_y, nct, (int)nb);
    DBSR_LAUNCH_CHECK();
    if (k.ksplit > 1) {
        const long long n = (long long)k.npix * (k.cw / 4);
        hipLaunchKernelGGL((conv_splitk_finalize<T>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, k);
        DBSR_LAUNCH_CHECK();
    }
    return 0;
}

// ------------------------------------------------------------------------------------------------
// Pipelined LDS-tiled 3x3 conv (bf16, stride 1, pad 1, dilation 1) for the large trunk convs: the
// encoder and weight-predictor ResNets at 48x48 and the decoder's 384x384 ResBlocks.
//
// One 512-thread block per CU, persistent over output tiles (WM couts x TH rows x TW pixels of one
// frame).  The work of a block is a sequence of stages, one per (tile, 32-channel chunk); a stage
// image (halo + the chunk's weights for all 9 taps) is staged by LDS-DMA into one of two LDS
// buffers.  Stage s+1's DMA is issued while stage s's 9 taps of MFMAs run -- one or two 1-KiB pieces
// per tap, never in a burst: s_memtime stamps of a burst-issue version showed every wave parked ~2k
// cycles per stage in the vector-memory issue queue (72 pieces per CU at ~28 cycles each through the
// texture-address path) before its first MFMA.  The tile epilogue works from registers: its residual
// loads and its (deferred, one stage later) output stores are spread over the taps the same way, so
// the only exposed wait per stage is one barrier.
// 8 waves = the TH rows of the tile: wave w owns row w (TW/16 groups of 16 pixels) x all WM couts.
// Per stage: weights 9*WM*64 B + halo (TH+2)(TW+2)*64 B for 2*WM*TW*TH*288 FLOP, i.e. 203 FLOP/B at
// (WM, TW, TH) = (64, 48, 8) against 153 for the 64 x 16x16 tile of the two-barrier kernel.
//
// Cout order inside a WM tile (weights and bias permuted by the packer, pipe_cout_perm): MFMA row m of
// 16-cout block i is physical cout 32(i>>1) + 8(m>>2) + 4(i&1) + (m&3), so the accumulators of blocks
// 2h and 2h+1 give lane (g, col) 8 consecutive couts of its pixel: 16-B residual loads and stores.
// ------------------------------------------------------------------------------------------------
template <int WM, int TW, int TH>
struct PipeCfg {
    static constexpr int NWAVES = 8;                          // two waves per SIMD (256-VGPR budget)
    static constexpr int RPW = TH / NWAVES;                   // tile rows per wave
    static constexpr int HWD = TW + 2, HHT = TH + 2;
    static constexpr int NQ = HWD * HHT;                      // halo pixels
    static constexpr int IN_ITEMS = (NQ + 15) / 16;           // halo pieces: 16 pixels x 64 B (4 k-groups)
    static constexpr int W_ITEMS = 9 * (WM / 16);             // weight pieces (tap, 16-cout block)
    static constexpr int ITEMS = IN_ITEMS + W_ITEMS;
    static constexpr int PER = (ITEMS + NWAVES - 1) / NWAVES; // DMA pieces per wave per stage (uniform)
    static constexpr int STAGE_U4 = ITEMS * 64;               // 16-B slots per stage buffer
    static constexpr int GPR = TW / 16;                       // 16-pixel groups per row
    static constexpr int GW = GPR * RPW;                      // pixel groups per wave
    static constexpr int NH = WM / 32;                        // 8-cout lane runs per pixel
    static constexpr int NOUT = NH * GW;                      // 16-B outputs per lane per tile
    static constexpr int BIAS_U4 = 512 / 4;                   // bias region: cout <= 512 floats
    static constexpr int LDS_U4 = 2 * STAGE_U4 + BIAS_U4;
    static_assert(TH % NWAVES == 0, "whole tile rows per wave");
    static_assert(TW % 16 == 0 && (WM == 32 || WM == 64), "tile shape");
    static_assert(LDS_U4 * 16 <= 160 * 1024, "two stage buffers + bias must fit the LDS");
};

// Pixel-major halo image: halo pixel p holds its chunk's 4 k-groups (64 B) in slots 4p..4p+3, k-group g
// at slot 4p + phys(p, g) with phys(p, g) = 2(g&1) + ((g>>1) ^ ((p>>2)&1)).  A DMA piece is then 16
// pixels x 64 B, i.e. 16 cache lines per wave-instruction instead of the 64 of a planar [k-group][pixel]
// piece, and the swizzle keeps every B-fragment ds_read_b128 conflict-free for any tap shift: within
// each of its four 16-lane groups, the 4 lanes with equal p mod 4 read 4 distinct phys values.
// Diagnostic build only (make exp EXP_FLAGS=-DDBSR_PIPE_STAMPS): per-wave s_memtime stamps around each
// stage's barrier and tap loop, read back by dbsr_diag_pipe_stamps (tools/pipe_stamps.py).  The product
// build compiles none of this.
#ifdef DBSR_PIPE_STAMPS
constexpr int STAMP_STAGES = 24, STAMP_EV = 5;
__device__ unsigned long long g_pipe_stamps[256 * 8 * (STAMP_STAGES * STAMP_EV + 2)];
#define PIPE_STAMP(slot)                                                                                        \
    do {                                                                                                       \
        const int sl_ = (slot);                                                                                \
        if (lane == 0 && blockIdx.x < 256 && sl_ < STAMP_STAGES * STAMP_EV + 2)                                 \
            g_pipe_stamps[(blockIdx.x * 8 + wave) * (STAMP_STAGES * STAMP_EV + 2) + sl_] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define PIPE_STAMP(slot) do { } while (0)
#endif

template <typename T, int WM, int TW, int TH, int EPI>
__global__ __launch_bounds__(512, 1) void conv3x3_pipe_kernel(ConvK k, int tiles_x, int tiles_y, int nct,
                                                              int ntiles) {
    using C = PipeCfg<WM, TW, TH>;
    DBSR_OWN_SIMDS();
    __shared__ __attribute__((aligned(16))) u32x4_t lds[C::LDS_U4];
    float* lbias = (float*)(lds + 2 * C::STAGE_U4);      // [nct * WM] fp32

    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // uniform: scalar DMA offsets
    const int g = lane >> 4, col = lane & 15;
    const int nchunks = k.CG / 4;
    // epilogue variants (compile-time where the forward's convs need them): 1 act(ReLU), 2 conv + residual
    // then ReLU (ResBlock conv2), 3 plain, 4 as 2 followed by a 1x1 head (<= 4 outputs) + ReLU whose fp32
    // NCHW result is the only thing stored (the decoder's last ResBlock + RGB predictor, decoders.py:59-61);
    // 0 reads act / residual / post_act at run time; 5 is 0 for the training dgrad's gate at the 32x16 tile,
    // whose gate is loaded in the epilogue itself (prefetched like the residual, as 0 does, it spills there);
    // 6 bias + LeakyReLU (PWC-Net)
    constexpr bool HEAD = EPI == 4;
    static_assert(!HEAD || WM == 32, "the head reads all 32 channels of a pixel from one cout tile");
    const bool has_res = EPI == 2 || HEAD || ((EPI == 0 || EPI == 5) && k.r != nullptr);
    auto act1 = [&](float v) {
        if constexpr (EPI == 1) return fmaxf(v, 0.f);
        else if constexpr (EPI == 0 || EPI == 5) return apply_act(v, k.act);
        else if constexpr (EPI == 6) return v > 0.f ? v : 0.1f * v;     // (apply_act's LeakyReLU)
        else return v;
    };
    auto act2 = [&](float v) {
        if constexpr (EPI == 2 || EPI == 4) return fmaxf(v, 0.f);
        else if constexpr (EPI == 0 || EPI == 5) return apply_act(v, k.post_act);
        else return v;
    };

    // bias into LDS once; ordered before its first read by the loop's first barrier
    for (int c = threadIdx.x; c < nct * WM; c += 512) lbias[c] = (k.bias && c < k.cout) ? k.bias[c] : 0.f;
    float* lhead = lbias + 256;                          // HEAD: weights [4][32] at +256, bias [4] at +384
    if constexpr (HEAD) {
        if (threadIdx.x < 128) lhead[threadIdx.x] = threadIdx.x < k.head_cout * 32 ? k.head_w[threadIdx.x] : 0.f;
        if (threadIdx.x < 4) lhead[128 + threadIdx.x] = (k.head_b && (int)threadIdx.x < k.head_cout) ? k.head_b[threadIdx.x] : 0.f;
    }

    // persistent tile walk, XCD-grouped: the blocks sharing an XCD (equal blockIdx % 8) take a
    // contiguous range of tile ids per round, so a spatial tile's cout tiles and neighbouring halos
    // meet in one L2 (grid is a multiple of 8)
    const int grid = gridDim.x, b = blockIdx.x;
    const int pb = (b & 7) * (grid >> 3) + (b >> 3);
    const int my_tiles = pb < ntiles ? (ntiles - pb + grid - 1) / grid : 0;
    if (my_tiles == 0) return;
    PIPE_STAMP(0);

    // tile descriptors hold wave-uniform values only (scalar registers); the lane's own pixel/cout offset
    // within a tile is the same for every tile
    // EPI 0 / 5: the training dgrad's ReLU-backward gate (out *= gate > 0); 0 loads it like the residual
    const bool has_gate = (EPI == 0 || EPI == 5) && k.gt != nullptr;
    struct Tile { const T* xf; long long y_off, r_off, g_off; int y0, x0, cb; };
    auto decode = [&](int i) {
        int L = i * grid + pb;
        const int ct = L % nct; L /= nct;
        const int tx = L % tiles_x; L /= tiles_x;
        const int ty = L % tiles_y;
        const int f = L / tiles_y;
        Tile t;
        t.y0 = ty * TH; t.x0 = tx * TW; t.cb = ct * WM;
        t.xf = (const T*)k.x + map_frame(k.xm, f) * k.x_is;
        const long long pix = (long long)t.y0 * k.out_w + t.x0;
        t.y_off = HEAD ? map_frame(k.ym, f) * k.y_is + pix : map_frame(k.ym, f) * k.y_is + k.y_c0 + t.cb + pix * k.y_ld;
        t.r_off = has_res ? map_frame(k.rm, f) * k.r_is + k.r_c0 + t.cb + pix * k.r_ld : 0;
        t.g_off = has_gate ? map_frame(k.gm, f) * k.g_is + k.g_c0 + t.cb + pix * k.g_ld : 0;
        return t;
    };
    const long long g_lane = has_gate ? (long long)(wave * C::RPW * k.out_w + col) * k.g_ld + g * 8 : 0;
    const long long y_lane = (long long)(wave * C::RPW * k.out_w + col) * k.y_ld + g * 8;
    const long long r_lane = has_res ? (long long)(wave * C::RPW * k.out_w + col) * k.r_ld + g * 8 : 0;
    // pixel-group jj of a wave = row jj / GPR of its RPW rows, 16-pixel column group jj % GPR
    auto grp_off = [&](int jj) { return (long long)(jj / C::GPR) * k.out_w + (jj % C::GPR) * 16; };

    // one 1-KiB DMA piece of stage (tile t, chunk c): piece `it` of this wave is item wave + 8*it of the
    // stage image (clamped: surplus slots re-issue the last piece, an identical write, so every wave
    // issues exactly PER pieces).  Halo pieces: the lane's (halo row, column, k-group) and its byte
    // offset from the halo origin are tile-invariant and precomputed; per piece only the frame bounds
    // test and one add remain (out-of-frame lanes read past the buffer resource and land zeros).
    // Weight pieces are contiguous 1 KiB: a uniform soffset on a constant lane offset.
    constexpr int HPER = (C::IN_ITEMS + C::NWAVES - 1) / C::NWAVES;   // halo pieces per wave (upper bound)
    int h_rc[HPER], h_off[HPER];
    const int pix_b = k.x_ld * (int)sizeof(T);
#pragma unroll
    for (int it = 0; it < HPER; ++it) {
        const int p = (wave + C::NWAVES * it) * 16 + (lane >> 2), ph = lane & 3;
        const int gg = 2 * ((ph & 1) ^ ((p >> 2) & 1)) + (ph >> 1);
        const int r = p / C::HWD, cc = p - r * C::HWD;
        h_rc[it] = p < C::NQ ? (r << 16) | cc : 0x7fff7fff;    // rows/cols past the halo never pass the test
        h_off[it] = (r * k.in_w + cc) * pix_b + gg * 16;
    }
    const __amdgpu_buffer_rsrc_t w_rsrc = buf_rsrc(k.w_pipe, 0xffffffffu);
    const unsigned frame_bytes = (unsigned)((long long)k.in_h * k.in_w * pix_b);
    auto dma = [&](int it, const Tile& t, int c, int buf) {
        const int item = min(wave + C::NWAVES * it, C::ITEMS - 1);
        u32x4_t* dst = lds + buf * C::STAGE_U4 + item * 64;
        if (it < HPER && item < C::IN_ITEMS) {
            const int hy = t.y0 - 1 + (h_rc[it] >> 16), hx = t.x0 - 1 + (h_rc[it] & 0xffff);
            const bool ok = (unsigned)hy < (unsigned)k.in_h && (unsigned)hx < (unsigned)k.in_w;
            const int base = ((t.y0 - 1) * k.in_w + (t.x0 - 1)) * pix_b + c * 64;
            blds16(buf_rsrc(t.xf, frame_bytes), ok ? base + h_off[it] : BUF_OOB, 0, dst);
        } else {
            // chunk-major weight copy: one contiguous 1-KiB piece per (16-cout block, chunk, tap)
            const int wi = item - C::IN_ITEMS;
            const int tap = wi / (WM / 16), blk = wi % (WM / 16);
            const int piece = (((t.cb >> 4) + blk) * nchunks + c) * 9 + tap;
            blds16(w_rsrc, lane * 16, piece * 1024, dst);
        }
    };

    f32x4_t acc[WM / 16][C::GW];
#pragma unroll
    for (int i = 0; i < WM / 16; ++i)
#pragma unroll
        for (int j = 0; j < C::GW; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    u32x4_t resv[C::NOUT];              // residual of the tile being computed (loaded in its last stage)
    u32x4_t pend[C::NOUT];              // packed outputs of the last finished tile (stored next stage)
    u32x4_t gatev[EPI == 0 ? C::NOUT : 1];   // EPI 0 gate of the tile being computed (as resv)

    // lane-dependent LDS bases within a stage buffer; tap/fragment offsets are immediates.  Halo pixel
    // P0 + imm of k-group g sits at slot 4(P0 + imm) + halo_phys(P0 + imm, g), and halo_phys depends on
    // imm only through imm & 7, so 8 per-lane bases cover every (tap, group) offset.
    const int P0 = wave * C::RPW * C::HWD + col;
    int in_base[8];
#pragma unroll
    for (int rho = 0; rho < 8; ++rho) in_base[rho] = 4 * P0 + halo_phys(P0 + rho, g);
    const int w_base = C::IN_ITEMS * 64 + g * 16 + col;

    // Epilogue of a finished tile, right after the barrier that follows its last stage (its residual,
    // loaded during that stage, has landed; no DMA is in flight yet): output piece q = (8-cout run h,
    // pixel group j) -- lane (g, col) holds couts cb + 32h + 8g .. +7 of its pixel in acc[2h][j] and
    // acc[2h+1][j] -- gets bias + act (+ residual + post-act) and is packed to bf16 for a 16-B store
    // during the next stage's taps; the accumulators restart from zero.
    auto epilogue = [&](const Tile& t) {
        u32x4_t gl[EPI == 5 ? C::NOUT : 1];             // EPI 5: this tile's gate, all pieces in flight at once
        if constexpr (EPI == 5) {
            if (has_gate) {
#pragma unroll
                for (int q = 0; q < C::NOUT; ++q) {
                    const int h = q / C::GW, j = q % C::GW;
                    gl[q] = *(const u32x4_t*)((const T*)k.gt + t.g_off + g_lane + grp_off(j) * k.g_ld +
                                              (pipe_lane_ch(t.cb, h, g, k.cout) - t.cb - 8 * g));
                }
            }
        }
#pragma unroll
        for (int q = 0; q < C::NOUT; ++q) {
            const int h = q / C::GW, j = q % C::GW;
            const float4 b0 = *(const float4*)(lbias + t.cb + 32 * h + 8 * g);
            const float4 b1 = *(const float4*)(lbias + t.cb + 32 * h + 8 * g + 4);
            const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
            float v[8];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                v[r] = act1(acc[2 * h][j][r] + bv[r]);
                v[4 + r] = act1(acc[2 * h + 1][j][r] + bv[4 + r]);
            }
            if (has_res) {
                const u32x4_t rq = resv[q];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    v[2 * e] = act2(v[2 * e] + H16<T>::lo(rq[e]));
                    v[2 * e + 1] = act2(v[2 * e + 1] + H16<T>::hi(rq[e]));
                }
            }
            if constexpr (EPI == 0 || EPI == 5) {
                if (has_gate) {
                    const u32x4_t gq = EPI == 5 ? gl[EPI == 5 ? q : 0] : gatev[EPI == 0 ? q : 0];
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        v[2 * e] = H16<T>::lo(gq[e]) > 0.f ? v[2 * e] : 0.f;
                        v[2 * e + 1] = H16<T>::hi(gq[e]) > 0.f ? v[2 * e + 1] : 0.f;
                    }
                }
            }
            u32x4_t o;
            if constexpr (HEAD) {
                // lane (g, col) holds channels 8g..8g+7 of its pixel: partial head sums, reduced over the
                // four g lanes of the column (xor 16, 32); lane g then keeps output channel g
                float hs[4];
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const float4 w0 = *(const float4*)(lhead + c * 32 + 8 * g);
                    const float4 w1 = *(const float4*)(lhead + c * 32 + 8 * g + 4);
                    float a = v[0] * w0.x;
                    a = fmaf(v[1], w0.y, a); a = fmaf(v[2], w0.z, a); a = fmaf(v[3], w0.w, a);
                    a = fmaf(v[4], w1.x, a); a = fmaf(v[5], w1.y, a); a = fmaf(v[6], w1.z, a); a = fmaf(v[7], w1.w, a);
                    a += __shfl_xor(a, 16, 64);
                    a += __shfl_xor(a, 32, 64);
                    hs[c] = a;
                }
                const float hv = g == 0 ? hs[0] : g == 1 ? hs[1] : g == 2 ? hs[2] : hs[3];
                o[0] = __float_as_uint(fmaxf(hv + lhead[128 + g], 0.f));
                o[1] = o[2] = o[3] = 0u;
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) o[e] = H16<T>::pack(v[2 * e], v[2 * e + 1]);
            }
            pend[q] = o;
            acc[2 * h][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
            acc[2 * h + 1][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        }
    };
    auto store_piece = [&](int q, const Tile& t) {   // runs of couts >= cout (partial cout tile) skipped
        const int h = q / C::GW, j = q % C::GW;
        if constexpr (HEAD) {
            // NCHW fp32: lanes of one g write 16 consecutive pixels of plane g
            if (g < k.head_cout)
                ((float*)k.y)[t.y_off + (long long)wave * C::RPW * k.out_w + col + grp_off(j) +
                              (long long)g * k.out_h * k.out_w] = __uint_as_float(pend[q][0]);
        } else if (t.cb + 32 * h + 8 * g < k.cout)
            *(u32x4_t*)((T*)k.y + t.y_off + y_lane + grp_off(j) * k.y_ld + 32 * h) = pend[q];
    };

    int s = 0;                          // global stage index (LDS buffer = s & 1)
    Tile cur = decode(0), prev = cur;
#pragma unroll
    for (int it = 0; it < C::PER; ++it) dma(it, cur, 0, 0);

    // Per stage: barrier, [epilogue of the previous tile], then the 9 taps with this stage's
    // vector-memory work spread between their MFMAs: the previous tile's output stores, this tile's
    // residual loads (last stage) and the next stage's DMA pieces (taps 0-5).
    for (int ti = 0; ti < my_tiles; ++ti) {
        for (int c = 0; c < nchunks; ++c, ++s) {
            PIPE_STAMP(2 + s * 5);
            vm_drain();                 // this wave's pieces of stage s landed ...
            PIPE_STAMP(3 + s * 5);
            __syncthreads();            // ... and everyone's (barrier); stage s-1 fully consumed
            PIPE_STAMP(4 + s * 5);
            const bool fin = c == 0 && ti > 0;
            if (fin) epilogue(prev);
            const bool last = c == nchunks - 1;
            const bool more = !(last && ti + 1 == my_tiles);
            Tile nxt = cur;
            const int nc = last ? 0 : c + 1;
            if (last && more) nxt = decode(ti + 1);
            const u32x4_t* lb_st = lds + (s & 1) * C::STAGE_U4;
            const u32x4_t* lb_w = lb_st + w_base;
            const int nbuf = (s + 1) & 1;
            auto vmem = [&](int tap) {
#pragma unroll
                for (int q = 0; q < C::NOUT; ++q) {
                    if ((q * 9) / C::NOUT != tap) continue;       // output pieces spread over the 9 taps
                    if (fin) store_piece(q, prev);
                    if (has_res && last) {
                        const int h = q / C::GW, j = q % C::GW;
                        resv[q] = *(const u32x4_t*)((const T*)k.r + cur.r_off + r_lane + grp_off(j) * k.r_ld +
                                                    (pipe_lane_ch(cur.cb, h, g, k.cout) - cur.cb - 8 * g));
                    }
                    if constexpr (EPI == 0) {
                        if (has_gate && last) {
                            const int h = q / C::GW, j = q % C::GW;
                            gatev[q] = *(const u32x4_t*)((const T*)k.gt + cur.g_off + g_lane + grp_off(j) * k.g_ld +
                                                         (pipe_lane_ch(cur.cb, h, g, k.cout) - cur.cb - 8 * g));
                        }
                    }
                }
                if (more) {
#pragma unroll
                    for (int it = 0; it < C::PER; ++it)
                        if ((it * 8) / C::PER == tap) dma(it, nxt, nc, nbuf);
                }
            };
            auto read_frags = [&](int tap, Frag<T> (&a)[WM / 16], Frag<T> (&bq)[C::GW]) {
                const int ky = tap / 3, kx = tap % 3;
#pragma unroll
                for (int i = 0; i < WM / 16; ++i) a[i].v = __builtin_bit_cast(bf16x8_t, lb_w[(tap * (WM / 16) + i) * 64]);
#pragma unroll
                for (int j = 0; j < C::GW; ++j) {
                    const int imm = (j / C::GPR + ky) * C::HWD + (j % C::GPR) * 16 + kx;
                    bq[j].v = __builtin_bit_cast(bf16x8_t, lb_st[in_base[imm & 7] + 4 * imm]);
                }
            };
            auto mfmas = [&](const Frag<T> (&a)[WM / 16], const Frag<T> (&bq)[C::GW]) {
#pragma unroll
                for (int i = 0; i < WM / 16; ++i)
#pragma unroll
                    for (int j = 0; j < C::GW; ++j) acc[i][j] = mma(a[i], bq[j], acc[i][j]);
            };
            Frag<T> a0[WM / 16], b0[C::GW], a1[WM / 16], b1[C::GW];
            read_frags(0, a0, b0);
#pragma unroll
            for (int tap = 0; tap < 9; tap += 2) {
                if (tap == 6) PIPE_STAMP(5 + s * 5);
                vmem(tap);
                if (tap + 1 < 9) read_frags(tap + 1, a1, b1);
                mfmas(a0, b0);
                if (tap + 1 < 9) {
                    vmem(tap + 1);
                    if (tap + 2 < 9) read_frags(tap + 2, a0, b0);
                    mfmas(a1, b1);
                }
            }
            PIPE_STAMP(6 + s * 5);
            if (last) {
                prev = cur;
                cur = nxt;
            }
        }
    }
    dma_barrier();                      // the last tile's residual loads landed
    epilogue(prev);
#pragma unroll
    for (int q = 0; q < C::NOUT; ++q) store_piece(q, prev);
    PIPE_STAMP(1);
}

int g_num_cus = 0;
int num_cus() {
    if (g_num_cus == 0) {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
            g_num_cus = n;
        else
            g_num_cus = 256;
    }
    return g_num_cus;
}

template <typename T, int WM, int TW, int TH>
int launch_pipe(const ConvK& k, int n_frames, hipStream_t s) {
    const int tiles_x = (k.out_w + TW - 1) / TW, tiles_y = (k.out_h + TH - 1) / TH;
    const int nct = (k.cout + WM - 1) / WM;
    const long long nt = (long long)n_frames * tiles_x * tiles_y * nct;
    if (nt >= (1LL << 31)) {
        dbsr_set_error("conv2d: grid too large");
        return DBSR_E_ARG;
    }
    const int cap = k.max_blocks > 0 ? std::min(k.max_blocks, num_cus()) : num_cus();
    int grid = (int)std::min<long long>(nt, cap);
    grid = (grid + 7) / 8 * 8;
    // compile-time epilogues for the forward's three conv flavours, run-time otherwise
    int epi = 0;                        // (a gated conv, the training dgrad, takes the run-time epilogue 0, or 5
    if (k.gt) epi = (TW == 32 && TH == 16) ? 5 : 0;   // at the 32x16 tile where 0's prefetched gate spills)
    else if (k.head_cout > 0) epi = 4;
    else if (!k.r && k.act == DBSR_ACT_RELU) epi = 1;
    else if (k.r && k.act == DBSR_ACT_NONE && k.post_act == DBSR_ACT_RELU) epi = 2;
    else if (!k.r && k.act == DBSR_ACT_NONE) epi = 3;
    // 6: bias + LeakyReLU, PWC-Net's convs: run-time epilogue 0 spilled 48 VGPRs at the 32x16 tile, 6 none
    // (pwc.refiner0 46 -> 38 us on the chip, profiles/r06e6_pipe_epi6_ab.txt)
    else if (!k.r && k.act == DBSR_ACT_LRELU) epi = 6;
#define DBSR_PIPE_LAUNCH(E)                                                                                    \
    hipLaunchKernelGGL((conv3x3_pipe_kernel<T, WM, TW, TH, E>), dim3(grid), dim3(512), 0, s, k, tiles_x, tiles_y, \
                       nct, (int)nt)
    switch (epi) {
        case 4:
            if constexpr (WM == 32) DBSR_PIPE_LAUNCH(4);
            break;
        case 1: DBSR_PIPE_LAUNCH(1); break;
        case 2: DBSR_PIPE_LAUNCH(2); break;
        case 3: DBSR_PIPE_LAUNCH(3); break;
        case 5:
            if constexpr (TW == 32 && TH == 16) DBSR_PIPE_LAUNCH(5);
            break;
        case 6: DBSR_PIPE_LAUNCH(6); break;
        default: DBSR_PIPE_LAUNCH(0); break;
    }
#undef DBSR_PIPE_LAUNCH
    DBSR_LAUNCH_CHECK();
    return 0;
}

// which pipelined tile serves `d` (0: none): bf16 3x3/s1/p1/d1 with Cin % 32 == 0 after padding, an
// aligned NHWC bf16 output (staged epilogue), and enough tiles to fill the chip
int g_pipe_enabled = 1;
int pick_pipe(const dbsr_conv_desc* d) {
    if (!g_pipe_enabled || !is16(d->x.dtype) || d->precise || d->kh != 3 || d->kw != 3 || d->stride != 1 ||
        d->pad != 1 || d->dil != 1 || d->cin <= 16 || d->out_mode != DBSR_OUT_NHWC || d->y.dtype != d->x.dtype)
        return 0;
    if (d->y.ld % 8 || d->y.c0 % 8 || d->cout % 8 || (d->res.ptr && (d->res.ld % 8 || d->res.c0 % 8))) return 0;
    if (d->gate.ptr && (d->gate.ld % 8 || d->gate.c0 % 8 || d->gate.dtype != d->y.dtype)) return 0;
    if (cin_pad(d->cin) * 2 + 64 > ZERO_PAGE_BYTES || d->cout > 512) return 0;
    if ((long long)d->in_h * d->in_w * d->x.ld * 2 >= (1LL << 31)) return 0;   // 32-bit buffer offsets per frame
    int cfg = 0, tw = 0, th = 8, wm = 0;
    if (d->cout > 32 && d->out_w % 48 == 0) { cfg = 1; tw = 48; wm = 64; }
    else if (d->cout <= 32 && d->out_w % 64 == 0) { cfg = 2; tw = 64; wm = 32; }
    // 16x16 frames (the PWC level-2 DenseNet and the refiner's first conv, pwcnet.py:123-150,188): one whole
    // frame per tile; a tile per block is enough to beat the LDS-tiled kernel on their 128 - 576 channels
    else if (d->cout > 32 && d->out_w == 16 && d->out_h == 16) { cfg = 3; tw = 16; th = 16; wm = 64; }
    // frame widths that are multiples of 32 but not 48 (the training step's 128x128 frames): 32x16 tiles
    // (gated: epilogue 5, the gate loaded in the epilogue)
    else if (d->cout > 32 && d->out_w % 32 == 0 && d->out_h % 16 == 0) { cfg = 4; tw = 32; th = 16; wm = 64; }
    if (!cfg || d->out_h % th) return 0;
    const long long nt = (long long)d->n_frames * (d->out_w / tw) * (d->out_h / th) * ((d->cout + wm - 1) / wm);
    return (nt >= (cfg == 3 ? 64 : 256) || g_pipe_enabled == 2) ? cfg : 0;
}
// a plan_h slab `g` can run pipelined tile `cfg` (chosen for the whole image)
bool pipe_fits(int cfg, const dbsr_conv_desc* g) {
    if (cfg == 3) return g->out_h == 16;
    return g->out_h % (cfg == 4 ? 16 : 8) == 0;
}

// ------------------------------------------------------------------------------------------------
// Weight-stationary 3x3 conv for Cin <= 64 (the encoder and offset-feature ResNets and enc.out at
// 48x48, the decoder's 64-channel pre-ResBlocks): a cout tile's weights for the whole K (9 taps x
// Cin) fit in the registers of the four waves that use them, so only the halo moves through the LDS.
//
// One 256-thread block per CU, one wave per SIMD (the whole register file: weights 144 VGPRs at
// Cin 64, accumulators in AGPRs), persistent over 16x16-pixel tiles of ONE 64-cout tile: wave
// (wc, wp) owns couts 32wc..32wc+31 (two 16-cout MFMA blocks whose rows the packer permuted so a
// lane ends up with 8 consecutive couts of its pixel, pipe_cout_perm) x tile rows 8wp..8wp+7.  Per
// tile the block stages the (18 x 18)-pixel halo of all Cin channels (42 KiB at Cin 64) into one of
// two LDS buffers by buffer-resource LDS-DMA (out-of-frame pixels land zeros); the next tile's halo,
// the previous tile's output stores and this tile's residual loads are spread between the MFMAs, so
// each tile costs one barrier for 288 MFMAs per wave (the pipelined kernel pays one per 108, and
// streams the weights through the LDS with every stage).  Per (chunk, tap) step a wave reads 8
// B-fragments (ds_read_b128) for 16 MFMAs: the LDS runs at half rate.
// Block -> work: blockIdx % 8 is the XCD; the PX blocks of an XCD split into the nct cout tiles x
// PX/nct spatial streams, so the cout tiles of a spatial tile (enc.out: 8) read its halo through
// one L2.
// ------------------------------------------------------------------------------------------------
template <int WM, int TW, int TH, int NCH>
struct WsCfg {
    static constexpr int NWAVES = 8;                          // two waves per SIMD
    static constexpr int WC = WM / 32;                        // waves across couts (32 couts each)
    static constexpr int WP = NWAVES / WC;                    // waves across tile rows
    static constexpr int RPW = TH / WP;                       // tile rows per wave
    static constexpr int GPR = TW / 16;                       // 16-pixel groups per row
    static constexpr int GW = RPW * GPR;                      // pixel groups per wave
    static constexpr int HWD = TW + 2, HHT = TH + 2, NQ = HWD * HHT;
    static constexpr int IN_ITEMS = (NQ + 15) / 16;           // 1-KiB halo pieces per 32-channel chunk
    static constexpr int ITEMS = NCH * IN_ITEMS;
    static constexpr int PER = (ITEMS + NWAVES - 1) / NWAVES; // pieces per wave per tile
    static constexpr int STAGE_U4 = ITEMS * 64;
    static constexpr int STEPS = NCH * 9;                     // (chunk, tap) k-steps per tile
    static constexpr int DMA_STEPS = (STEPS + 1) / 2;         // with a residual: the next halo in the first half
    static constexpr int SPP = WM / 8;                        // 16-B slots per pixel of the residual tile
    static constexpr int RES_U4 = TW * TH * SPP;              // residual tile: [pixel][WM couts], 16-B slots
    static constexpr int RES_ITEMS = RES_U4 / 64;             // its 1-KiB pieces (64 / SPP pixels each)
    static constexpr int RPER = (RES_ITEMS + NWAVES - 1) / NWAVES;
    static_assert(TH % WP == 0 && TW % 16 == 0 && (WM == 64 || WM == 32), "tile shape");
    static constexpr int W_PIECES = (WM / 16) * NCH * 9;      // the cout tile's chunk-major weights, 1-KiB pieces
    static constexpr int W_PER = (W_PIECES + NWAVES - 1) / NWAVES;
    static_assert((2 * STAGE_U4 + 2 * RES_U4 + WM / 4) * 16 <= 160 * 1024, "halo + residual stages must fit the LDS");
    static_assert((STAGE_U4 + W_PIECES * 64 + WM / 4) * 16 <= 160 * 1024, "weight staging must fit the LDS");
};

template <typename T, int WM, int TW, int TH, int NCH, int EPI>
__global__ __launch_bounds__(512, 1) void conv3x3_ws_kernel(ConvK k, int tiles_x, int tiles_y, int nct, int nsp,
                                                            int px) {
    using C = WsCfg<WM, TW, TH, NCH>;
    static_assert(EPI >= 0 && EPI <= 5 && EPI != 4, "epilogues 0-3, 5");
    DBSR_OWN_SIMDS();
    constexpr int RES_BUFS = (EPI == 0 || EPI == 2 || EPI == 5) ? 2 : 0;
    // the next tile's halo goes out over the first half of the k-steps when the residual follows in the
    // second half, else over the first two thirds (measured: enc.out 205 -> 196 us, residual convs slower)
    constexpr int DMA_STEPS = RES_BUFS > 0 ? C::DMA_STEPS : (2 * C::STEPS) / 3;
    // [halo 0][halo 1][residual 0][residual 1][bias]; at the start the block's weights are staged once at
    // [halo 1 ...) (every wave then copies its A-fragments to registers) instead of each of the 8 waves
    // fetching its fragments from L2 (4 waves share each fragment set)
    constexpr int BUF_U4 = 2 * C::STAGE_U4 + RES_BUFS * C::RES_U4;
    constexpr int STG_U4 = C::STAGE_U4 + C::W_PIECES * 64;
    __shared__ __attribute__((aligned(16))) u32x4_t lds[(BUF_U4 > STG_U4 ? BUF_U4 : STG_U4) + WM / 4];
    u32x4_t* lres = lds + 2 * C::STAGE_U4;                 // residual tiles (double-buffered)
    float* lbias = (float*)(lds + (BUF_U4 > STG_U4 ? BUF_U4 : STG_U4));   // the cout tile's bias (fp32)

    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g = lane >> 4, col = lane & 15;
    const int wc = wave % C::WC, wp = wave / C::WC;
    // EPI 5: EPI 0 plus the training dgrad's gate, out *= (gate > 0), loaded at the start of the epilogue
    const bool has_res = EPI == 2 || ((EPI == 0 || EPI == 5) && k.r != nullptr);
    const bool has_gate = EPI == 5;
    auto act1 = [&](float v) {
        if constexpr (EPI == 1) return fmaxf(v, 0.f);
        else if constexpr (EPI == 0 || EPI == 5) return apply_act(v, k.act);
        else return v;
    };
    auto act2 = [&](float v) {
        if constexpr (EPI == 2) return fmaxf(v, 0.f);
        else if constexpr (EPI == 0 || EPI == 5) return apply_act(v, k.post_act);
        else return v;
    };

    // block -> (cout tile, spatial stream); grid = 8 * px, px a multiple of nct
    const int b = blockIdx.x, slot = b >> 3, spx = px / nct;
    const int ct = slot % nct, S = 8 * spx, sid = (b & 7) * spx + slot / nct;
    const int my_tiles = sid < nsp ? (nsp - sid + S - 1) / S : 0;
    if (my_tiles == 0) return;
    PIPE_STAMP(0);

    // the cout tile's weights (chunk-major copy: contiguous 1-KiB pieces) into the staging region
    const int cb = ct * WM + wc * 32;
    {
        const __amdgpu_buffer_rsrc_t w_rsrc = buf_rsrc(k.w_pipe, 0xffffffffu);
        const int p0 = (ct * WM >> 4) * NCH * 9;
#pragma unroll
        for (int it = 0; it < C::W_PER; ++it) {
            const int piece = min(wave + C::NWAVES * it, C::W_PIECES - 1);
            blds16(w_rsrc, lane * 16, (p0 + piece) * 1024, lds + C::STAGE_U4 + piece * 64);
        }
    }
    if (threadIdx.x < WM) {             // ordered before its first read by the loop's first barrier
        const int co = ct * WM + threadIdx.x;
        lbias[threadIdx.x] = (k.bias && co < k.cout) ? k.bias[co] : 0.f;
    }
    const bool cout_ok = cb + 8 * g < k.cout;

    struct Tile { const T* xf; long long y_off, r_off, g_off; int y0, x0; };
    auto decode = [&](int i) {
        int L = sid + i * S;
        const int tx = L % tiles_x; L /= tiles_x;
        const int ty = L % tiles_y;
        const int f = L / tiles_y;
        Tile t;
        t.y0 = ty * TH; t.x0 = tx * TW;
        t.xf = (const T*)k.x + map_frame(k.xm, f) * k.x_is;
        const long long pix = (long long)t.y0 * k.out_w + t.x0;
        t.y_off = map_frame(k.ym, f) * k.y_is + k.y_c0 + cb + pix * k.y_ld;
        t.r_off = has_res ? map_frame(k.rm, f) * k.r_is : 0;   // residual frame base (buffer-resource base)
        t.g_off = has_gate ? map_frame(k.gm, f) * k.g_is + k.g_c0 + cb + pix * k.g_ld : 0;
        return t;
    };
    // pixel of group j of this lane, relative to the tile origin
    auto px_off = [&](int j) {
        return (long long)(wp * C::RPW + j / C::GPR) * k.out_w + (j % C::GPR) * 16 + col;
    };

    // halo DMA: piece `it` of this wave is item wave + 4*it (clamped: surplus slots rewrite the last
    // piece with identical bytes); lane -> (halo pixel, physical k-group slot) as in the pipelined kernel
    const int pix_b = k.x_ld * (int)sizeof(T);
    const unsigned frame_bytes = (unsigned)((long long)k.in_h * k.in_w * pix_b);
    int h_rc[C::PER], h_off[C::PER];
#pragma unroll
    for (int it = 0; it < C::PER; ++it) {
        const int item = min(wave + C::NWAVES * it, C::ITEMS - 1);
        const int cch = item / C::IN_ITEMS, ii = item - cch * C::IN_ITEMS;
        const int p = ii * 16 + (lane >> 2), ph = lane & 3;
        const int gg = 2 * ((ph & 1) ^ ((p >> 2) & 1)) + (ph >> 1);
        const int r = p / C::HWD, cc = p - r * C::HWD;
        h_rc[it] = p < C::NQ ? (r << 16) | cc : 0x7fff7fff;
        h_off[it] = (r * k.in_w + cc) * pix_b + cch * 64 + gg * 16;
    }
    auto dma = [&](int it, const Tile& t, int buf) {
        const int item = min(wave + C::NWAVES * it, C::ITEMS - 1);
        const int hy = t.y0 - 1 + (h_rc[it] >> 16), hx = t.x0 - 1 + (h_rc[it] & 0xffff);
        const bool ok = (unsigned)hy < (unsigned)k.in_h && (unsigned)hx < (unsigned)k.in_w;
        const int base = ((t.y0 - 1) * k.in_w + (t.x0 - 1)) * pix_b;
        blds16(buf_rsrc(t.xf, frame_bytes), ok ? base + h_off[it] : BUF_OOB, 0, lds + buf * C::STAGE_U4 + item * 64);
    };

    // B-fragment of group j at step (chunk c, tap): halo pixel P0 + imm, k-group g (halo_phys swizzle;
    // 8 per-lane bases cover every immediate offset)
    const int P0 = wp * C::RPW * C::HWD + col;
    int in_base[8];
#pragma unroll
    for (int rho = 0; rho < 8; ++rho) in_base[rho] = 4 * P0 + halo_phys(P0 + rho, g);
    auto read_b = [&](const u32x4_t* lb, int step, int j) {
        const int c = step / 9, tap = step % 9, ky = tap / 3, kx = tap % 3;
        const int imm = (j / C::GPR + ky) * C::HWD + (j % C::GPR) * 16 + kx;
        Frag<T> f;
        f.v = __builtin_bit_cast(bf16x8_t, lb[c * C::IN_ITEMS * 64 + in_base[imm & 7] + 4 * imm]);
        return f;
    };

    f32x4_t acc[2][C::GW];
    // residual tile via LDS-DMA: piece q = 64/SPP tile pixels x WM*2 B; lane l -> pixel (64/SPP)q + l/SPP,
    // physical slot l % SPP holding logical slot (l % SPP) ^ (pixel % SPP) -- the XOR keeps the epilogue's
    // ds_read_b128 (16 consecutive pixels x 2 slots per lane group) conflict-free.  Out-of-frame bytes
    // (a partial cout tile at the frame's last pixel) land zeros.
    // the resource spans the residual frame from its first channel, so the slots of a partial cout tile
    // past the frame's last pixel fall outside it (zeros) rather than past the allocation
    const unsigned rframe_bytes = (unsigned)((long long)k.out_h * k.out_w * k.r_ld * (int)sizeof(T));
    const int r_cb = k.r_c0 + ct * WM;
    auto res_dma = [&](int it, const Tile& t, int buf) {
        const int q = min(wave + C::NWAVES * it, C::RES_ITEMS - 1);
        const int pp = q * (64 / C::SPP) + lane / C::SPP, ls = (lane % C::SPP) ^ (pp % C::SPP);
        const int off = (((t.y0 + pp / TW) * k.out_w + t.x0 + pp % TW) * k.r_ld + r_cb + ls * 8) * (int)sizeof(T);
        blds16(buf_rsrc((const T*)k.r + t.r_off, rframe_bytes), off, 0, lres + buf * C::RES_U4 + q * 64);
    };
    u32x4_t packed[C::GW];
    // bias + act (+ residual from the LDS + post-act, + gate) of a finished tile into `packed`
    auto epilogue = [&](const Tile& t, int rbuf) {
        u32x4_t gatev[EPI == 5 ? C::GW : 1];
        if constexpr (EPI == 5) {
            // lanes of a partial cout tile past cout read the cout tile's first channel instead (never stored;
            // cb itself can be >= cout, which at the last pixel of the last frame lies past the allocation)
#pragma unroll
            for (int j = 0; j < C::GW; ++j)
                gatev[j] = *(const u32x4_t*)((const T*)k.gt + t.g_off + px_off(j) * k.g_ld +
                                             (ws_lane_ch(ct * WM, wc, g, k.cout) - cb));
        }
        const float4 b0 = *(const float4*)(lbias + wc * 32 + 8 * g);
        const float4 b1 = *(const float4*)(lbias + wc * 32 + 8 * g + 4);
        const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
        for (int j = 0; j < C::GW; ++j) {
            float v[8];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                v[r] = act1(acc[0][j][r] + bv[r]);
                v[4 + r] = act1(acc[1][j][r] + bv[4 + r]);
            }
            if (has_res) {
                const int pp = (wp * C::RPW + j / C::GPR) * TW + (j % C::GPR) * 16 + col;
                const u32x4_t rq = lres[rbuf * C::RES_U4 + pp * C::SPP + ((wc * 4 + g) ^ (pp % C::SPP))];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    v[2 * e] = act2(v[2 * e] + H16<T>::lo(rq[e]));
                    v[2 * e + 1] = act2(v[2 * e + 1] + H16<T>::hi(rq[e]));
                }
            }
            if constexpr (EPI == 5) {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    v[2 * e] = H16<T>::lo(gatev[j][e]) > 0.f ? v[2 * e] : 0.f;
                    v[2 * e + 1] = H16<T>::hi(gatev[j][e]) > 0.f ? v[2 * e + 1] : 0.f;
                }
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) packed[j][e] = H16<T>::pack(v[2 * e], v[2 * e + 1]);
        }
    };
    // the tile's packed outputs, stored right after the next barrier (issued before it, the stores would
    // hold up that barrier's vmcnt(0))
    auto store = [&](const Tile& t) {
#pragma unroll
        for (int j = 0; j < C::GW; ++j)
            if (cout_ok) *(u32x4_t*)((T*)k.y + t.y_off + px_off(j) * k.y_ld + 8 * g) = packed[j];
    };

    Tile cur = decode(0), prev = cur;
#pragma unroll
    for (int it = 0; it < C::PER; ++it) dma(it, cur, 0);
    // the wave's A-fragments of both 16-cout blocks for every (chunk, tap), from the staged weights; the
    // loop's first barrier then orders these reads before any wave's DMA into the staging region
    dma_barrier();
    Frag<T> wr[NCH][9][2];
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
        for (int tap = 0; tap < 9; ++tap)
#pragma unroll
            for (int h = 0; h < 2; ++h)
                wr[c][tap][h].v = __builtin_bit_cast(
                    bf16x8_t, lds[C::STAGE_U4 + (((wc * 2 + h) * NCH + c) * 9 + tap) * 64 + lane]);

    PIPE_STAMP(2);
    for (int ti = 0; ti < my_tiles; ++ti) {
        PIPE_STAMP(3 + ti * 5);
        vm_drain();                     // this wave's LDS-DMAs landed, then the barrier: everyone's did
        PIPE_STAMP(4 + ti * 5);
        __syncthreads();                // this tile's halo landed; the other buffer is free
        PIPE_STAMP(5 + ti * 5);
        const bool more = ti + 1 < my_tiles;
        if (ti > 0) store(prev);        // previous tile's outputs (computed before the barrier)
        PIPE_STAMP(6 + ti * 5);
        const Tile nxt = more ? decode(ti + 1) : cur;
        const u32x4_t* lb = lds + (ti & 1) * C::STAGE_U4;
        const int nbuf = (ti + 1) & 1;
        Frag<T> bq[C::GW];
#pragma unroll
        for (int j = 0; j < C::GW; ++j) bq[j] = read_b(lb, 0, j);
#pragma unroll
        for (int step = 0; step < C::STEPS; ++step) {
            // vector-memory work of this step: the next tile's halo (first half) and residual (second half;
            // its buffer was last read by the epilogue before this tile's barrier)
            if (more) {
#pragma unroll
                for (int it = 0; it < C::PER; ++it)
                    if ((it * DMA_STEPS) / C::PER == step) dma(it, nxt, nbuf);
            }
            if constexpr (RES_BUFS > 0) {
                if (has_res && ti == 0) {      // tile 0's residual (its buffer was the weight staging area)
#pragma unroll
                    for (int it = 0; it < C::RPER; ++it)
                        if (it == step) res_dma(it, cur, 0);
                }
                if (has_res && more) {
#pragma unroll
                    for (int it = 0; it < C::RPER; ++it)
                        if (DMA_STEPS + (it * (C::STEPS - 2 - DMA_STEPS)) / C::RPER == step)
                            res_dma(it, nxt, nbuf);
                }
            }
            const int c = step / 9, tap = step % 9;
#pragma unroll
            for (int j = 0; j < C::GW; ++j) {
                const f32x4_t z = {0.f, 0.f, 0.f, 0.f};
                acc[0][j] = mma(wr[c][tap][0], bq[j], step == 0 ? z : acc[0][j]);
                acc[1][j] = mma(wr[c][tap][1], bq[j], step == 0 ? z : acc[1][j]);
                if (step + 1 < C::STEPS) bq[j] = read_b(lb, step + 1, j);
            }
            // keep each B-fragment read right behind the two MFMAs that consumed its register, so it
            // has a whole step (16 MFMAs) to land: the default schedule bunched them late
#pragma unroll
            for (int j = 0; j < C::GW; ++j) {
                __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);     // 2 MFMA
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);     // 1 DS read
            }
        }
        PIPE_STAMP(7 + ti * 5);
        // this tile's epilogue before the next barrier: the waves that finish their MFMAs first fill the
        // barrier skew with it.  Its residual landed before this tile's barrier -- except tile 0's, which other
        // waves DMA'd during its k-steps (one extra barrier); buffer ti & 1 is next written by the DMA of tile
        // ti + 2's residual, issued after the next barrier
        if constexpr (RES_BUFS > 0) {
            if (has_res && ti == 0) {
                dma_barrier();
            }
        }
        epilogue(cur, ti & 1);
        prev = cur;
        cur = nxt;
    }
    store(prev);
    PIPE_STAMP(1);
}

int g_ws_enabled = 1;
// weight-stationary kernel for `d` (blocks per XCD, 0: not applicable): 16-bit 3x3/s1/p1/d1 with
// either 16 < cin <= 64, 32 < cout <= 512 on 16x16 tiles (WM 64) or 16 < cin <= 32, 16 <= cout <= 32 on 64x8
// tiles (WM 32: the decoder's 384x384 post-ResBlocks), aligned NHWC output / residual
inline bool ws_narrow(const dbsr_conv_desc* d) { return d->cout <= 32; }
// 16x8 instead of 16x16 tiles (WM 64, 32 < cin <= 64) when the 16x16 grid would cover under half the chip:
// the decoder's pre-ResBlocks (8 frames of 48x48: 72 tiles) are a block's weight staging plus one tile; and for
// every gated conv (the training step's dgrads, EPI 5): the 16x16 tile's gated epilogue spills 14 VGPRs, the 16x8
// one none (training step 55.5-55.7 against 56.0-56.4 ms on one box, profiles/r06v_ws_gate_tile_ab.txt)
inline bool ws_short(const dbsr_conv_desc* d) {
    if (d->gate.ptr && d->cout > 32 && d->cin > 32) return true;
    return !ws_narrow(d) && d->cin > 32 && d->out_w % 16 == 0 && d->out_h % 16 == 0 &&
           (long long)d->n_frames * (d->out_w / 16) * (d->out_h / 16) * ((d->cout + 63) / 64) < 128;
}
// (d: the selection view; g: the launch geometry when it differs -- a plan_h slab -- which must suit the tile
// chosen for d; the block count then follows g's own tile count)
int pick_ws(const dbsr_conv_desc* d, const dbsr_conv_desc* g = nullptr) {
    if (!g_ws_enabled || !is16(d->x.dtype) || d->precise || d->kh != 3 || d->kw != 3 || d->stride != 1 ||
        d->pad != 1 || d->dil != 1 || d->cin <= 16 || d->cin > 64 || d->out_mode != DBSR_OUT_NHWC ||
        d->y.dtype != d->x.dtype)
        return 0;
    if (d->gate.ptr && (d->gate.ld % 8 || d->gate.c0 % 8 || d->gate.dtype != d->y.dtype)) return 0;
    if (d->y.ld % 8 || d->y.c0 % 8 || d->cout % 8 || d->cout > 512 ||
        (d->res.ptr && (d->res.ld % 8 || d->res.c0 % 8)))
        return 0;
    const bool narrow = ws_narrow(d);
    const int tw = narrow ? 64 : 16, th = (narrow || ws_short(d)) ? 8 : 16, wm = narrow ? 32 : 64;
    if (narrow && (d->cout < 16 || d->cin > 32)) return 0;      // WM 32: one 32-channel chunk (LDS budget)
    if (d->out_w % tw || d->out_h % th) return 0;
    if ((long long)d->in_h * d->in_w * d->x.ld * 2 >= (1LL << 31)) return 0;   // 32-bit buffer offsets per frame
    if (d->res.ptr && (long long)d->out_h * d->out_w * d->res.ld * 2 >= (1LL << 31)) return 0;
    const int nct = (d->cout + wm - 1) / wm;
    const long long nsp = (long long)d->n_frames * (d->out_w / tw) * (d->out_h / th);
    const int cus = d->max_blocks > 0 ? std::min(d->max_blocks, num_cus()) : num_cus();
    if (cus / 8 / nct < 1 || nsp * nct < 64) return 0;
    if (!g) g = d;
    if (g->out_h % th) return -1;                                             // slab rows do not tile
    const long long nsp_g = (long long)g->n_frames * (g->out_w / tw) * (g->out_h / th);
    const long long want = (nsp_g + 7) / 8;                                   // spatial streams per XCD
    const long long spx = std::max<long long>(1, std::min<long long>(cus / 8 / nct, want));
    return (int)(spx * nct);
}

template <typename T, int WM, int TW, int TH, int NCH>
int launch_ws(const ConvK& k, const dbsr_conv_desc* d, int px, hipStream_t s) {
    const int tiles_x = k.out_w / TW, tiles_y = k.out_h / TH;
    const int nct = (k.cout + WM - 1) / WM;
    const int nsp = d->n_frames * tiles_x * tiles_y;
    int epi = 0;                        // (a gated conv, the training dgrad, takes epilogue 5)
    if (k.gt) epi = 5;
    else if (!k.r && k.act == DBSR_ACT_RELU) epi = 1;
    else if (k.r && k.act == DBSR_ACT_NONE && k.post_act == DBSR_ACT_RELU) epi = 2;
    else if (!k.r && k.act == DBSR_ACT_NONE) epi = 3;
#define DBSR_WS_LAUNCH(E)                                                                                         \
    hipLaunchKernelGGL((conv3x3_ws_kernel<T, WM, TW, TH, NCH, E>), dim3(8 * px), dim3(512), 0, s, k, tiles_x,    \
                       tiles_y, nct, nsp, px)
    switch (epi) {
        case 1: DBSR_WS_LAUNCH(1); break;
        case 2: DBSR_WS_LAUNCH(2); break;
        case 3: DBSR_WS_LAUNCH(3); break;
        case 5: DBSR_WS_LAUNCH(5); break;
        default: DBSR_WS_LAUNCH(0); break;
    }
#undef DBSR_WS_LAUNCH
    DBSR_LAUNCH_CHECK();
    return 0;
}

int g_ks128_enabled = 1;
// the K-split weight-stationary 128-channel kernel (conv128.hip) serves `d`: 16-bit 3x3/s1/p1/d1, 96 < cin <= 128,
// cout == 128, aligned NHWC output / residual / gate, frames a multiple of 16 x 8, the whole image (no plan_h slab)
// and at least 128 tiles (the weight predictor's input conv and ResBlocks, merging.py:86-90, 98-101, and their
// gated dgrads in the training step)
bool use_ks128(const dbsr_conv_desc* d) {
    if (!g_ks128_enabled || !is16(d->x.dtype) || d->precise || d->kh != 3 || d->kw != 3 || d->stride != 1 ||
        d->pad != 1 || d->dil != 1 || cin_pad(d->cin) != 128 || d->cout != 128 || d->out_mode != DBSR_OUT_NHWC ||
        d->y.dtype != d->x.dtype)
        return false;
    if (d->y.ld % 8 || d->y.c0 % 8 || (d->res.ptr && (d->res.ld % 8 || d->res.c0 % 8))) return false;
    if (d->gate.ptr && (d->gate.ld % 8 || d->gate.c0 % 8 || d->gate.dtype != d->y.dtype)) return false;
    if (d->out_w % ks128::TW || d->out_h % ks128::TH || (d->plan_h > 0 && d->plan_h != d->out_h)) return false;
    if ((long long)d->in_h * d->in_w * d->x.ld * 2 >= (1LL << 31)) return false;   // 32-bit buffer offsets per frame
    return (long long)d->n_frames * (d->out_w / ks128::TW) * (d->out_h / ks128::TH) >= 128;
}
int launch_ks128(const ConvK& k, const dbsr_conv_desc* d, hipStream_t s) {
    int epi = 0;                        // the pipelined kernel's compile-time epilogues 1-3, run-time 0 otherwise,
    if (k.gt) epi = 5;                  // 5 with the gate
    else if (!k.r && k.act == DBSR_ACT_RELU) epi = 1;
    else if (k.r && k.act == DBSR_ACT_NONE && k.post_act == DBSR_ACT_RELU) epi = 2;
    else if (!k.r && k.act == DBSR_ACT_NONE) epi = 3;
    return ks128_launch(k, d->n_frames, d->x.dtype == DBSR_F16, epi, k.max_blocks, num_cus(), s);
}

// ------------------------------------------------------------------------------------------------
// Fused 32-channel ResBlock (blocks.py:81-96: y = relu(x + conv2(relu(conv1(x)))), 3x3/s1/p1 convs with bias):
// the decoder's 384x384 post-ResBlocks (decoders.py:46-49).  The two ws32 launches it replaces move 377 MB per
// block at the bench shape (x read twice, the intermediate written and read, y written); this kernel moves
// x and y once (151 MB) -- the intermediate never leaves the LDS.
//
// Persistent blocks of 8 waves (2 per SIMD; one wave per SIMD with 4-group batches measured 87.5 against 62.7
// us); every wave keeps both convs' weights in registers (A-fragments of the chunk-major pipe copy, 2 x 72
// VGPRs) and runs 2 pixel groups per MFMA batch with its LDS reads two taps ahead.  Work unit = a 32x16 output tile.  Per tile: the input halo
// (36 x 20 pixels) arrives by LDS-DMA one tile ahead into a double buffer (the halo_phys swizzle of the
// weight-stationary kernel; out-of-frame pixels land zeros); conv1 runs on the 34 x 18 intermediate region
// (39 flattened 16-pixel MFMA groups, 1.2x the output) and writes relu(conv1 + b1), rounded to T -- or zeros
// outside the frame, conv2's padding -- into an LDS image laid out like the halo; one barrier; conv2 runs on
// the 32 flattened groups of the tile, adds b2 and the residual (the halo's centre) and stores relu(...).
// Each output is the arithmetic of conv3x3_ws_kernel's epilogues 1 and 2 (taps in order from 0, bias after,
// residual after the bias), so the result is bitwise that of the two dbsr_conv2d launches.
// Block -> tiles: the 256 tiles of a round go to the blocks so that an XCD's 32 blocks take 32 consecutive
// tiles (their halos overlap in that XCD's L2).
// ------------------------------------------------------------------------------------------------
namespace rbk {
constexpr int TW = 32, TH = 16;
constexpr int MW = TW + 2, MH = TH + 2, MPX = MW * MH;        // conv1 region 34 x 18
constexpr int IW = TW + 4, IH = TH + 4, IPX = IW * IH;        // input halo 36 x 20
constexpr int IN_PIECES = (IPX + 15) / 16;                    // 45 1-KiB pieces
constexpr int IN_U4 = IN_PIECES * 64;
constexpr int G1 = (MPX + 15) / 16;                           // 39 conv1 groups
constexpr int MID_U4 = G1 * 16 * 4;
constexpr int G2 = TW * TH / 16;                              // 32 conv2 groups
constexpr int NW = 8;                                         // two waves per SIMD
constexpr int PER = (IN_PIECES + NW - 1) / NW;                // 6 pieces per wave
constexpr int Q1 = (G1 + NW - 1) / NW;                        // conv1 groups per wave (5; wave 7: 4)
constexpr int Q2 = G2 / NW;                                   // conv2 groups per wave (4)
constexpr int NG = 2;                                         // groups per MFMA batch
constexpr int LDS_BYTES = (2 * IN_U4 + MID_U4) * 16 + 64 * 4;
static_assert(LDS_BYTES <= 160 * 1024, "resblock LDS");
}  // namespace rbk

// HEAD: the decoder's RGB predictor (decoders.py:61, 1x1 32 -> head_cout + ReLU) on the block's fp32 output, as
// the pipelined kernel's epilogue 4 computes it (same products, order and lane reduction); k2.y is then the
// head's fp32 NCHW output and the block's own output is not stored
template <typename T, bool HEAD>
__global__ __launch_bounds__(512, 1) void resblock32_kernel(ConvK k1, ConvK k2, int tiles_x, int tiles_y,
                                                            int ntiles) {
    using namespace rbk;
    DBSR_OWN_SIMDS();
    __shared__ __attribute__((aligned(16))) u32x4_t lds[2 * IN_U4 + MID_U4 + 16 + 34];
    u32x4_t* lmid = lds + 2 * IN_U4;
    float* lbias = (float*)(lds + 2 * IN_U4 + MID_U4);            // [b1 (32)][b2 (32)]
    float* lhead = lbias + 64;                                    // HEAD: weights [4][32], bias [4]
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int H = k1.in_h, W = k1.in_w;

    // both convs' A-fragments: piece (half h, tap) of the chunk-major copy is lane-major 1 KiB
    Frag<T> w1[9][2], w2[9][2];
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            w1[tap][h].load((const T*)((const char*)k1.w_pipe + (h * 9 + tap) * 1024 + lane * 16));
            w2[tap][h].load((const T*)((const char*)k2.w_pipe + (h * 9 + tap) * 1024 + lane * 16));
        }
    if (threadIdx.x < 64) {
        const ConvK& kb = threadIdx.x < 32 ? k1 : k2;
        lbias[threadIdx.x] = kb.bias ? kb.bias[threadIdx.x & 31] : 0.f;
    }
    if constexpr (HEAD) {
        if (threadIdx.x < 128) lhead[threadIdx.x] = (int)threadIdx.x < k2.head_cout * 32 ? k2.head_w[threadIdx.x] : 0.f;
        if (threadIdx.x < 4)
            lhead[128 + threadIdx.x] = (k2.head_b && (int)threadIdx.x < k2.head_cout) ? k2.head_b[threadIdx.x] : 0.f;
    }

    struct Tile { const T* xf; long long y_off; int y0, x0; };
    auto decode = [&](int i) {
        const int t = rb_tile(i, blockIdx.x, gridDim.x, ntiles);
        Tile tl;
        const int tx = t % tiles_x, r = t / tiles_x, ty = r % tiles_y, f = r / tiles_y;
        tl.y0 = ty * TH; tl.x0 = tx * TW;
        tl.xf = (const T*)k1.x + map_frame(k1.xm, f) * k1.x_is;
        tl.y_off = HEAD ? map_frame(k2.ym, f) * k2.y_is + (long long)tl.y0 * W + tl.x0
                        : map_frame(k2.ym, f) * k2.y_is + k2.y_c0 + ((long long)tl.y0 * W + tl.x0) * k2.y_ld;
        return tl;
    };
    const int my_tiles = ntiles / (int)gridDim.x + ((int)blockIdx.x < ntiles % (int)gridDim.x ? 1 : 0);
    const int pix_b = k1.x_ld * (int)sizeof(T);
    const unsigned frame_bytes = (unsigned)((long long)H * W * pix_b);
    const unsigned lds0 = (unsigned)(unsigned long long)(__attribute__((address_space(3))) u32x4_t*)lds;
    // the next tile's halo: inline-asm LDS-DMA (lds_dma16), so the compiler does not drain it before the conv1
    // epilogue's LDS writes; the drain is the vm_drain of the tile's second barrier
    auto dma = [&](const Tile& tl, int buf) {
        int ln = lane;
        asm volatile("" : "+v"(ln));
#pragma unroll
        for (int it = 0; it < PER; ++it) {
            const int piece = min(wave + NW * it, IN_PIECES - 1);
            const int p = piece * 16 + (ln >> 2), ph = ln & 3;
            const int gg = 2 * ((ph & 1) ^ ((p >> 2) & 1)) + (ph >> 1);
            const int r = p / IW, c = p - r * IW;
            const int hy = tl.y0 - 2 + r, hx = tl.x0 - 2 + c;
            const bool ok = p < IPX && (unsigned)hy < (unsigned)H && (unsigned)hx < (unsigned)W;
            lds_dma16(tl.xf, frame_bytes, ok ? (hy * W + hx) * pix_b + gg * 16 : BUF_OOB, 0,
                      lds0 + (buf * IN_U4 + piece * 64) * 16);
        }
    };

    // the 9 taps of NG 16-pixel groups (image rows iw wide, group j's tap-(0,0) pixel P0[j]): B-fragments read
    // two taps ahead (a 3-deep ring per group)
    // (NB = the batch's group count: NG, or the lone last group of conv1's odd count)
    auto taps = [&](const u32x4_t* img, int iw, int g, const auto& P0, const Frag<T> (&w)[9][2], auto& acc) {
        constexpr int NB = std::extent<std::remove_reference_t<decltype(P0)>>::value;
        int bs[NB][8];
#pragma unroll
        for (int j = 0; j < NB; ++j)
#pragma unroll
            for (int rho = 0; rho < 8; ++rho) bs[j][rho] = 4 * P0[j] + halo_phys(P0[j] + rho, g);
        Frag<T> bq[NB][3];
        auto rd = [&](int j, int tap) {
            const int imm = (tap / 3) * iw + tap % 3;
            Frag<T> b;
            b.v = __builtin_bit_cast(bf16x8_t, img[bs[j][imm & 7] + 4 * imm]);
            return b;
        };
#pragma unroll
        for (int j = 0; j < NB; ++j) {
            bq[j][0] = rd(j, 0);
            bq[j][1] = rd(j, 1);
        }
        StaticFor<0, 9>::run([&](auto t_) {
            constexpr int tap = decltype(t_)::value;
            const f32x4_t z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int j = 0; j < NB; ++j) {
                acc[j][0] = mma(w[tap][0], bq[j][tap % 3], tap == 0 ? z : acc[j][0]);
                acc[j][1] = mma(w[tap][1], bq[j][tap % 3], tap == 0 ? z : acc[j][1]);
                if constexpr (tap + 2 < 9) bq[j][(tap + 2) % 3] = rd(j, tap + 2);
            }
        });
        // the scheduler's MFMA / DS-read interleave for small GEMM loops: without it the reads sank to their uses
        // and every tap waited on its own read (measured: 69-71 us either way, two launches 75 us)
        __builtin_amdgcn_iglp_opt(0);
    };

    // a conv2 group's output: 8 channels of a pixel (16-bit NHWC), or with HEAD lane g's head channel (fp32 NCHW)
    auto store_out = [&](const Tile& tl, int i, int g, int col, const u32x4_t& o) {
        const int q = wave + NW * i;
        const long long px = (long long)(q >> 1) * W + 16 * (q & 1) + col;
        if constexpr (HEAD) {
            if (g < k2.head_cout) ((float*)k2.y)[tl.y_off + px + (long long)g * H * W] = __uint_as_float(o[0]);
        } else {
            *(u32x4_t*)((T*)k2.y + tl.y_off + px * k2.y_ld + 8 * g) = o;
        }
    };
    Tile cur = decode(0), prev = cur;
    if (my_tiles > 0) dma(cur, 0);
    u32x4_t outv[Q2];                   // the previous tile's conv2 outputs, stored after this tile's first barrier
    for (int ti = 0; ti < my_tiles; ++ti) {
        dma_barrier();                  // B0: tile ti's halo landed; the intermediate image is free
        // lane-derived values recomputed per tile from an opaque copy of the lane index (hoisted out of the loop,
        // the groups' per-lane LDS bases took registers for the whole loop)
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const int g = ln >> 4, col = ln & 15;
        if (ti > 0) {
#pragma unroll
            for (int i = 0; i < Q2; ++i) store_out(prev, i, g, col, outv[i]);
        }
        const u32x4_t* lin = lds + (ti & 1) * IN_U4;
        const bool more = ti + 1 < my_tiles;
        const Tile nxt = more ? decode(ti + 1) : cur;
        if (more) dma(nxt, (ti + 1) & 1);
        // ---- conv1 on the intermediate region: groups wave + 8 i, in batches of NG and a lone last group (the odd
        // fifth: batching it with a clamped duplicate cost a sixth of conv1's MFMAs and LDS reads) ----
        {
            const float4 b0 = *(const float4*)(lbias + 8 * g), b1 = *(const float4*)(lbias + 8 * g + 4);
            const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
            auto conv1 = [&](auto nb_, auto q0_) {
                constexpr int NB = decltype(nb_)::value, Q0 = decltype(q0_)::value;
                int pa[NB], P0[NB];
#pragma unroll
                for (int j = 0; j < NB; ++j) {
                    pa[j] = min(16 * (wave + NW * (Q0 + j)) + col, MPX - 1);
                    const int r = pa[j] / MW, c = pa[j] - r * MW;
                    P0[j] = r * IW + c;
                }
                f32x4_t acc[NB][2];
                taps(lin, IW, g, P0, w1, acc);
#pragma unroll
                for (int j = 0; j < NB; ++j) {
                    const int p = 16 * (wave + NW * (Q0 + j)) + col;
                    const int r = pa[j] / MW, c = pa[j] - r * MW;
                    const int fy = cur.y0 - 1 + r, fx = cur.x0 - 1 + c;
                    const bool inside = (unsigned)fy < (unsigned)H && (unsigned)fx < (unsigned)W;
                    u32x4_t o;
#pragma unroll
                    for (int e = 0; e < 2; ++e) {
                        o[e] = relu16x2(H16<T>::pack(acc[j][0][2 * e] + bv[2 * e], acc[j][0][2 * e + 1] + bv[2 * e + 1]));
                        o[2 + e] = relu16x2(H16<T>::pack(acc[j][1][2 * e] + bv[4 + 2 * e],
                                                         acc[j][1][2 * e + 1] + bv[4 + 2 * e + 1]));
                    }
                    if (!inside) o = u32x4_t{0u, 0u, 0u, 0u};
                    if (p < MPX) lmid[4 * p + halo_phys(p, g)] = o;
                }
            };
            StaticFor<0, Q1 / NG>::run([&](auto bt_) {
                conv1(std::integral_constant<int, NG>{}, std::integral_constant<int, NG * decltype(bt_)::value>{});
            });
            if constexpr (Q1 % NG != 0) {
                // wave-uniform: the waves whose last group lies inside the region (wave 7's fifth does not)
                if (wave + NW * (Q1 - Q1 % NG) < G1)
                    conv1(std::integral_constant<int, Q1 % NG>{}, std::integral_constant<int, Q1 - Q1 % NG>{});
            }
        }
        dma_barrier();                  // B1: the intermediate image is complete (the next halo's DMA, issued before
                                        // conv1, has landed too: no LDS-DMA crosses a barrier in flight)
        // ---- conv2 on the tile: groups wave + 4 i, in batches of NG ----
        {
            const float4 b0 = *(const float4*)(lbias + 32 + 8 * g), b1 = *(const float4*)(lbias + 32 + 8 * g + 4);
            const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
            StaticFor<0, Q2 / NG>::run([&](auto bt_) {
                constexpr int bt = decltype(bt_)::value;
                int row[NG], cc[NG], P0[NG];
#pragma unroll
                for (int j = 0; j < NG; ++j) {
                    const int q = wave + NW * (NG * bt + j);
                    row[j] = q >> 1;
                    cc[j] = 16 * (q & 1) + col;
                    P0[j] = row[j] * MW + cc[j];
                }
                f32x4_t acc[NG][2];
                taps(lmid, MW, g, P0, w2, acc);
#pragma unroll
                for (int j = 0; j < NG; ++j) {
                    const int PR = (row[j] + 2) * IW + cc[j] + 2;
                    const u32x4_t rq = lin[4 * PR + halo_phys(PR, g)];
                    float v[8];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        v[r] = acc[j][0][r] + bv[r];
                        v[4 + r] = acc[j][1][r] + bv[4 + r];
                    }
                    u32x4_t o;
                    if constexpr (HEAD) {
                        // the pipelined kernel's epilogue 4: fp32 ReLU(v + residual), partial head sums over this
                        // lane's 8 channels, reduced over the column's four g lanes; lane g keeps channel g
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            v[2 * e] = fmaxf(v[2 * e] + H16<T>::lo(rq[e]), 0.f);
                            v[2 * e + 1] = fmaxf(v[2 * e + 1] + H16<T>::hi(rq[e]), 0.f);
                        }
                        float hs[4];
#pragma unroll
                        for (int c = 0; c < 4; ++c) {
                            const float4 w0 = *(const float4*)(lhead + c * 32 + 8 * g);
                            const float4 w1 = *(const float4*)(lhead + c * 32 + 8 * g + 4);
                            float a = v[0] * w0.x;
                            a = fmaf(v[1], w0.y, a); a = fmaf(v[2], w0.z, a); a = fmaf(v[3], w0.w, a);
                            a = fmaf(v[4], w1.x, a); a = fmaf(v[5], w1.y, a); a = fmaf(v[6], w1.z, a);
                            a = fmaf(v[7], w1.w, a);
                            a += __shfl_xor(a, 16, 64);
                            a += __shfl_xor(a, 32, 64);
                            hs[c] = a;
                        }
                        const float hv = g == 0 ? hs[0] : g == 1 ? hs[1] : g == 2 ? hs[2] : hs[3];
                        o = u32x4_t{__float_as_uint(fmaxf(hv + lhead[128 + g], 0.f)), 0u, 0u, 0u};
                    } else {
#pragma unroll
                        for (int e = 0; e < 4; ++e)
                            o[e] = relu16x2(H16<T>::pack(v[2 * e] + H16<T>::lo(rq[e]), v[2 * e + 1] + H16<T>::hi(rq[e])));
                    }
                    outv[NG * bt + j] = o;
                }
            });
        }
        prev = cur;
        cur = nxt;
    }
    if (my_tiles > 0) {
#pragma unroll
        for (int i = 0; i < Q2; ++i) store_out(prev, i, lane >> 4, lane & 15, outv[i]);
    }
    vm_drain();                         // (no LDS-DMA outstanding at s_endpgm: tools/isa_audit.py)
}

// byte range [lo, hi) that `n` frames of t cover: each stored image from its first used element (c0) to the last
// pixel's last element (per_img elements past the image base: NHWC (hw - 1) * ld + c0 + ch, NCHW its plane count)
void tensor_span(const dbsr_tensor& t, int n, long long per_img, int es, unsigned long long& lo,
                 unsigned long long& hi) {
    long long mn = 0, mx = 0;
    for (int f = 0; f < n; ++f) {
        const long long img = (long long)(f / t.map.fpg) * t.map.group_stride + t.map.group_offset +
                              (long long)(f % t.map.fpg) * t.map.inner_stride;
        if (f == 0 || img < mn) mn = img;
        if (f == 0 || img > mx) mx = img;
    }
    const unsigned long long base = (unsigned long long)(uintptr_t)t.ptr;
    lo = base + (unsigned long long)((mn * t.img_stride + t.c0) * es);
    hi = base + (unsigned long long)((mx * t.img_stride + per_img) * es);
}
// the persistent ResBlock kernel reads neighbouring tiles' input halos while other blocks store finished tiles, so
// its output (c2->y, or the head's fp32 NCHW output) must not overlap its input x (an in-place call
// y == x would race; the two-call path it replaces is in-place safe)
bool resblock_out_disjoint(const dbsr_conv_desc* c1, const dbsr_conv_desc* c2, const dbsr_tensor* head_out,
                           int head_cout) {
    const long long hw = (long long)c1->in_h * c1->in_w;
    const int C = c1->cin;
    unsigned long long xl, xh, yl, yh;
    tensor_span(c1->x, c1->n_frames, (hw - 1) * c1->x.ld + c1->x.c0 + C, 2, xl, xh);
    if (head_out) tensor_span(*head_out, c1->n_frames, (long long)head_cout * hw, 4, yl, yh);
    else tensor_span(c2->y, c1->n_frames, (hw - 1) * c2->y.ld + c2->y.c0 + C, 2, yl, yh);
    return yh <= xl || xh <= yl;
}

// the fused ResBlock applies: c1 = conv1 (x -> any, ReLU), c2 = conv2 (-> y, residual x, post-ReLU), both
// 16-bit 3x3/s1/p1/d1 C -> C with chunk-major weight copies, NHWC slices aligned; returns C (32: resblock32_kernel,
// frames a multiple of 32 x 16; 64: resblock64_kernel, frames a multiple of 16 x 16) or 0
int resblock_channels(const dbsr_conv_desc* c1, const dbsr_conv_desc* c2) {
    if (!c1 || !c2) return 0;
    const int C = c1->cin;
    if (C != 32 && C != 64) return 0;
    auto conv_ok = [C](const dbsr_conv_desc* d) {
        return is16(d->x.dtype) && d->y.dtype == d->x.dtype && !d->precise && d->kh == 3 && d->kw == 3 &&
               d->stride == 1 && d->pad == 1 && d->dil == 1 && d->cin == C && d->cout == C &&
               d->out_mode == DBSR_OUT_NHWC && !d->gate.ptr && d->in_h == d->out_h && d->in_w == d->out_w;
    };
    if (!conv_ok(c1) || !conv_ok(c2)) return 0;
    if (c1->act != DBSR_ACT_RELU || c1->res.ptr || c2->act != DBSR_ACT_NONE || c2->post_act != DBSR_ACT_RELU)
        return 0;
    // the residual is conv1's input (same tensor, slice and frames)
    if (c2->res.ptr != c1->x.ptr || c2->res.c0 != c1->x.c0 || c2->res.ld != c1->x.ld ||
        c2->res.img_stride != c1->x.img_stride || c2->res.dtype != c1->x.dtype ||
        std::memcmp(&c2->res.map, &c1->x.map, sizeof(dbsr_frame_map)) != 0)
        return 0;
    if (c1->n_frames != c2->n_frames || c1->in_h != c2->in_h || c1->in_w != c2->in_w || c1->x.dtype != c2->y.dtype)
        return 0;
    if (C == 32 ? (c1->in_w % rbk::TW || c1->in_h % rbk::TH) : (c1->in_w % rb64::TW || c1->in_h % rb64::TH)) return 0;
    if (C == 64) {
        // the 64-channel kernel only where it beats the two weight-stationary launches: small grids (the decoder's
        // pre-ResBlocks, 144 tiles: 10.7 vs 12.1 us); at the encoder's 2016 tiles it measured 51 vs 49 us (uncapped)
        // and 80 vs 69 us (under the 128-CU cap) -- DESIGN.md, round 6
        const long long tiles = (long long)c1->n_frames * (c1->in_w / rb64::TW) * (c1->in_h / rb64::TH);
        const int cus = c1->max_blocks > 0 ? std::min(c1->max_blocks, num_cus()) : num_cus();
        if (tiles > 2LL * cus) return 0;
    }
    if (c1->x.ld % 8 || c1->x.c0 % 8 || c1->x.c0 + C > c1->x.ld) return 0;
    if (c2->y.ld % 8 || c2->y.c0 % 8 || c2->y.c0 + C > c2->y.ld) return 0;
    return (long long)c1->in_h * c1->in_w * c1->x.ld * 2 < (1LL << 31) ? C : 0;
}

template <typename T>
int dispatch_ws(int px, const ConvK& k, const dbsr_conv_desc* d, const dbsr_conv_desc* sel, hipStream_t s) {
    if (ws_narrow(sel)) return launch_ws<T, 32, 64, 8, 1>(k, d, px, s);
    if (ws_short(sel)) return launch_ws<T, 64, 16, 8, 2>(k, d, px, s);
    if (k.CG / 4 == 1) return launch_ws<T, 64, 16, 16, 1>(k, d, px, s);
    return launch_ws<T, 64, 16, 16, 2>(k, d, px, s);
}

template <typename T>
int dispatch_pipe(int cfg, const ConvK& k, const dbsr_conv_desc* d, hipStream_t s) {
    if (cfg == 1) return launch_pipe<T, 64, 48, 8>(k, d->n_frames, s);
    if (cfg == 3) return launch_pipe<T, 64, 16, 16>(k, d->n_frames, s);
    if (cfg == 4) return launch_pipe<T, 64, 32, 16>(k, d->n_frames, s);
    return launch_pipe<T, 32, 64, 8>(k, d->n_frames, s);
}

template <typename T, int MT, int NT, typename XT = T>
int launch_conv(const ConvK& k0, hipStream_t s) {
    ConvK k = k0;
    k.stage_epi = MT * NT >= 2 && sizeof(T) == 2 && sizeof(XT) == 2 && k.ksplit == 1 &&
                  k.out_mode == DBSR_OUT_NHWC && !k.y_f32 && !k.r && !k.gt && k.cout % 8 == 0 && k.y_ld % 8 == 0 &&
                  k.y_c0 % 8 == 0 && k.head_cout == 0;
    dim3 grid((k.npix + 4 * NT * 16 - 1) / (4 * NT * 16), (k.cout + MT * 16 - 1) / (MT * 16), k.ksplit);
    hipLaunchKernelGGL((conv2d_kernel<T, MT, NT, XT>), grid, dim3(256), 0, s, k);
    DBSR_LAUNCH_CHECK();
    if (k.ksplit > 1) {
        const long long n = (long long)k.npix * (k.cw / 4);
        hipLaunchKernelGGL((conv_splitk_finalize<T>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, k);
        DBSR_LAUNCH_CHECK();
    }
    return 0;
}

// Split-K for the generic kernel when the grid cannot fill the chip (PWC coarse levels, 2-channel
// flow heads): K slices of >= 8 k-steps until there are ~512 blocks.
int choose_ksplit(const ConvK& k, int mt, int nt) {
    const long long blocks = (long long)((k.npix + 64 * nt - 1) / (64 * nt)) * ((k.cout + 16 * mt - 1) / (16 * mt));
    const int nks = k.KGp >> 2;
    // long-K convs (the 2-channel flow heads: K = 9 x 565) also split while the grid is < 4 blocks/CU
    const long long target = nks >= 64 ? 1024 : 512;
    if (blocks >= target / 2 || nks < 16) return 1;
    int sp = (int)((target + blocks - 1) / blocks);
    sp = std::min(sp, nks / 8);
    sp = std::min(sp, 32);
    return std::max(sp, 1);
}
size_t splitk_bytes(const ConvK& k, int sp) {
    return sp > 1 ? (size_t)sp * k.npix * k.cw * sizeof(float) : 0;
}
// generic kernel: the largest tile that still gives >= 2 blocks per CU (512 blocks); tiny PWC levels
// (a few hundred pixels) fall through to 16 x 64-pixel tiles (and split-K) for parallelism
void pick_generic_tile(const ConvK& k, int& best_m, int& best_n) {
    const int mts[3] = {4, 2, 1}, nts[3] = {4, 2, 1};
    const long long minb = 512;   // 1024 / 2048 / 4096 measured: enc.init 21.4 / 25.7 / 29.3 us vs 23.1
    best_m = 1;
    best_n = 1;
    for (int a = 0; a < 3; ++a) {
        if (mts[a] > 1 && k.cout <= (mts[a] / 2) * 16) continue;          // do not pad cout beyond need
        for (int b = 0; b < 3; ++b) {
            const long long blocks = (long long)((k.npix + 64 * nts[b] - 1) / (64 * nts[b])) *
                                     ((k.cout + 16 * mts[a] - 1) / (16 * mts[a]));
            if (blocks >= minb) {
                best_m = mts[a];
                best_n = nts[b];
                return;
            }
        }
    }
}

// ------------------------------------------------------------------------------------------------
// 3x3 conv of an 8-channel (padded) 16-bit input: the frame encoder's first conv (encoders.py:36, 4 raw channels ->
// 64) and the offset-feature extractor's (merging.py:85, the 2 offset channels -> 64).  K = 9 taps x 8 channels = 72,
// packed as 3 MFMA k-steps of 4 taps (the packer's rows: k = tap * 8 + channel, taps 9-11 zero).  Each wave keeps
// the 64 x 96 weights as A-fragments in registers (48 VGPRs) and walks 16-pixel groups: per group lane (g, col)
// loads tap 4s + g of pixel col (16 B, one input pixel's 8 channels; out-of-frame taps zero) for k-step s, then
// 12 MFMAs (4 16-cout blocks x 3 k-steps) and bias + act, 8-B stores of 4 couts.  The generic kernel ran these
// as general implicit GEMMs at 22-25 us each on the whole chip (r06f) for ~31 MB of output.
// ------------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void conv3x3_small_kernel(ConvK k, int groups_x, long long ngroups) {
    const int lane = threadIdx.x & 63, g = lane >> 4, col = lane & 15;
    const int nco = k.cout / 16;                       // 16-cout blocks (cout % 16 == 0, <= 64)
    Frag<T> a[4][3];
    f32x4_t bias[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        bias[b] = load_bias4(k, min(b, nco - 1) * 16 + g * 4);
#pragma unroll
        for (int st = 0; st < 3; ++st)
            a[b][st].load((const T*)k.w + (long long)(min(b, nco - 1) * 16 + col) * k.Kp + 32 * st + 8 * g);
    }
    const long long wave0 = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const long long nwaves = ((long long)gridDim.x * blockDim.x) >> 6;
    for (long long gi = wave0; gi < ngroups; gi += nwaves) {
        const int gx = (int)(gi % groups_x);
        const long long r = gi / groups_x;
        const int y = (int)(r % k.out_h), f = (int)(r / k.out_h);
        const int x = gx * 16 + col;
        const T* xf = (const T*)k.x + map_frame(k.xm, f) * k.x_is;
        Frag<T> bq[3];
#pragma unroll
        for (int st = 0; st < 3; ++st) {
            const int tap = 4 * st + g, ky = tap / 3, kx = tap - 3 * (tap / 3);
            const int iy = y + ky - 1, ix = x + kx - 1;
            if (tap < 9 && (unsigned)iy < (unsigned)k.in_h && (unsigned)ix < (unsigned)k.in_w)
                bq[st].load(xf + ((long long)iy * k.in_w + ix) * k.x_ld);
            else
                bq[st].zero();
        }
        f32x4_t acc[4];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            acc[b] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int st = 0; st < 3; ++st) acc[b] = mma(a[b][st], bq[st], acc[b]);
        }
        if (x < k.out_w) {
            T* yp = (T*)k.y + map_frame(k.ym, f) * k.y_is + k.y_c0 + ((long long)y * k.out_w + x) * k.y_ld + 4 * g;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                if (b >= nco) break;
                uint2 o;
                o.x = H16<T>::pack(apply_act(acc[b][0] + bias[b][0], k.act), apply_act(acc[b][1] + bias[b][1], k.act));
                o.y = H16<T>::pack(apply_act(acc[b][2] + bias[b][2], k.act), apply_act(acc[b][3] + bias[b][3], k.act));
                *(uint2*)(yp + 16 * b) = o;
            }
        }
    }
}

int g_small_enabled = 1;
// conv3x3_small_kernel serves `d`: 16-bit 3x3/s1/p1/d1, cin <= 8, cout a multiple of 16 up to 64, NHWC output of the
// input dtype (y.ld, y.c0 multiples of 4), no residual or gate
bool use_small(const dbsr_conv_desc* d) {
    return g_small_enabled && is16(d->x.dtype) && !d->precise && d->kh == 3 && d->kw == 3 && d->stride == 1 &&
           d->pad == 1 && d->dil == 1 && d->cin <= 8 && d->cout % 16 == 0 && d->cout <= 64 &&
           d->out_mode == DBSR_OUT_NHWC && d->y.dtype == d->x.dtype && d->y.ld % 4 == 0 && d->y.c0 % 4 == 0 &&
           !d->res.ptr && !d->gate.ptr;
}
template <typename T>
int launch_small(const ConvK& k, const dbsr_conv_desc* d, hipStream_t s) {
    const int gx = (d->out_w + 15) / 16;
    const long long ng = (long long)d->n_frames * d->out_h * gx;
    const long long want = (ng + 15) / 16;             // ~4 groups per wave
    const unsigned grid = (unsigned)std::max<long long>(1, std::min<long long>(want, 4096));
    hipLaunchKernelGGL((conv3x3_small_kernel<T>), dim3(grid), dim3(256), 0, s, k, gx, ng);
    DBSR_LAUNCH_CHECK();
    return 0;
}

// narrow-output 3x3 convs over a long K (conv3x3_narrow_kernel): 16-bit 3x3/s1/p1/d1, cout <= 4, cin >= 256,
// NHWC output without gate
int g_narrow_enabled = 1;
bool use_narrow(const dbsr_conv_desc* d) {
    return g_narrow_enabled && is16(d->x.dtype) && !d->precise && d->kh == 3 && d->kw == 3 && d->stride == 1 &&
           d->pad == 1 && d->dil == 1 && d->cout <= 4 && d->cin >= 256 && d->out_mode == DBSR_OUT_NHWC &&
           !d->gate.ptr;
}
template <typename T>
int launch_narrow(const ConvK& k, const dbsr_conv_desc* d, hipStream_t s) {
    const int tiles_x = (d->out_w + 15) / 16, tiles_y = (d->out_h + 3) / 4;
    const long long blocks = (long long)d->n_frames * tiles_x * tiles_y;
    DBSR_CHECK_ARG(blocks < (1LL << 31), "conv2d: too many narrow tiles");
    hipLaunchKernelGGL((conv3x3_narrow_kernel<T>), dim3((unsigned)blocks), dim3(256), 0, s, k, tiles_x, tiles_y);
    DBSR_LAUNCH_CHECK();
    return 0;
}

// 3x3 'same' convolutions (pad == dilation) with dilation 1/2/4/8 (the PWC refiner's context
// network, pwcnet.py:227-241, has 2/4/8; fp32 tiles with dilation 8 exceed the LDS)
bool use_tiled(const dbsr_conv_desc* d) {
    const bool bf = is16(d->x.dtype);
    const bool dil_ok = (d->dil == 1 || d->dil == 2 || d->dil == 4 || (d->dil == 8 && bf)) && d->pad == d->dil;
    return !d->precise && cin_pad(d->cin) * (bf ? 2 : 4) + 64 <= ZERO_PAGE_BYTES && d->kh == 3 && d->kw == 3 &&
           d->stride == 1 && dil_ok && d->cin > 16 && d->out_h >= 8 && d->out_w >= 8 &&
           d->out_mode == DBSR_OUT_NHWC && g_tiled_enabled;
}

// Tile shape: 64 couts x 16x16 pixels by default; 32 couts for narrow convs (and 32x16 pixels on
// large images); when the grid would leave CUs idle (< 2 blocks per CU: PWC coarse levels, the
// 8-frame decoder convs) first 32 couts, then 16x4-pixel tiles.
int tiled_blocks(const dbsr_conv_desc* d, int wm, int wn) {
    const int th = 4 * wn / 16;
    return d->n_frames * ((d->out_w + 15) / 16) * ((d->out_h + th - 1) / th) * ((d->cout + wm - 1) / wm);
}
#ifndef DBSR_TILE_WM32_MAX_COUT
#define DBSR_TILE_WM32_MAX_COUT 64      // wider convs keep 64-cout tiles (halving re-reads the halo twice)
#endif
void pick_tiled_tile(const dbsr_conv_desc* d, int& wm, int& wn) {     // (d: the selection view)
    wm = d->cout <= 32 ? 32 : 64;
    wn = (wm == 32 && d->out_h >= 32) ? 128 : 64;
    if (tiled_blocks(d, wm, wn) >= 512) return;
    if (wm == 64) {
        if (d->cout > DBSR_TILE_WM32_MAX_COUT && d->out_w > 8) return;   // 8x8 PWC level 3: parallelism wins
        wm = 32;
        if (tiled_blocks(d, wm, wn) >= 512) return;
    }
    wn = 64;
    if (tiled_blocks(d, wm, wn) >= 512) return;
    wn = 16;
}

// Split-K for the LDS-tiled kernel (16-bit, dilation 1): a long-K conv (>= 8 chunks of 32 channels) whose natural
// tile (64 couts x 16x16 pixels) gives under 256 blocks keeps that tile and splits its chunks into K slices of >= 2
// chunks until there are ~512 blocks -- the decoder's first conv (decoders.py:37, 512 -> 64 on
// 8 frames of 48x48: 72 tiles x 8 slices: 55.6 -> 47.5 us in the step, r06q); the slices' fp32 partials go to the
// workspace and conv_splitk_finalize adds them in slice order.  Only for cout >= 64: PWC-Net's last level-2
// DenseNet conv (533 -> 32 on 104 16x16 frames) measured 36.0 -> 41.2 us split against the 16x4-pixel tiles.
// Returns the split (1: none) and sets the tile.
int g_tiled_split_enabled = 1;
int tiled_ksplit(const dbsr_conv_desc* d, int& wm, int& wn) {
    if (!g_tiled_split_enabled || !is16(d->x.dtype) || d->dil != 1 || d->cout < 64) return 1;
    const int nch = cin_pad(d->cin) / 32;
    const int wm0 = 64;
    const int nb = tiled_blocks(d, wm0, 64);
    if (nb >= 256 || nch < 8) return 1;
    const int sp = std::min(nch / 2, (512 + nb - 1) / nb);
    if (sp < 2) return 1;
    wm = wm0;
    wn = 64;
    return sp;
}

template <typename T, int D>
int dispatch_tiled_d(const ConvK& k0, const dbsr_conv_desc* d, const dbsr_conv_desc* sel, hipStream_t s) {
    int wm, wn;
    pick_tiled_tile(sel, wm, wn);
    ConvK k = k0;
    k.ksplit = tiled_ksplit(sel, wm, wn);
    if (k.ksplit > 1 && splitk_bytes(k, k.ksplit) > d->workspace_bytes) {
        k.ksplit = 1;
        pick_tiled_tile(sel, wm, wn);
    }
    if (wm == 64) return launch_tiled<T, 64, 64, D>(k, d->n_frames, s);
    if (wn == 128) return launch_tiled<T, 32, 128, D>(k, d->n_frames, s);
    if (wn == 64) return launch_tiled<T, 32, 64, D>(k, d->n_frames, s);
    return launch_tiled<T, 32, 16, D>(k, d->n_frames, s);
}

ConvK make_convk(const dbsr_conv_desc* d);

int slab_misfit(const dbsr_conv_desc* d, const dbsr_conv_desc* sel) {
    dbsr_set_error("conv2d: a %d-row slab cannot take the tile chosen for plan_h = %d rows (use a multiple of 16)",
                   d->out_h, sel->out_h);
    return DBSR_E_ARG;
}

// d: the launch geometry; sel: the selection view (sel_view)
template <typename T>
int dispatch_conv(const ConvK& k, const dbsr_conv_desc* d, const dbsr_conv_desc* sel, hipStream_t s) {
    if constexpr (sizeof(T) == 2) {
        const int px = pick_ws(sel, d);
        if (px < 0) return slab_misfit(d, sel);
        if (px) return dispatch_ws<T>(px, k, d, sel, s);
        if (use_ks128(sel)) return launch_ks128(k, d, s);
        const int cfg = pick_pipe(sel);
        if (cfg && !pipe_fits(cfg, d)) return slab_misfit(d, sel);
        if (cfg) return dispatch_pipe<T>(cfg, k, d, s);
        if (use_narrow(sel)) return launch_narrow<T>(k, d, s);
        if (use_small(sel)) return launch_small<T>(k, d, s);
    }
    if (use_tiled(sel)) {
        switch (d->dil) {
            case 1: return dispatch_tiled_d<T, 1>(k, d, sel, s);
            case 2: return dispatch_tiled_d<T, 2>(k, d, sel, s);
            case 4: return dispatch_tiled_d<T, 4>(k, d, sel, s);
            default:
                if constexpr (sizeof(T) == 2) return dispatch_tiled_d<T, 8>(k, d, sel, s);
                dbsr_set_error("conv2d: no fp32 tile for dilation %d", d->dil);
                return DBSR_E_ARG;
        }
    }
    int best_m, best_n;
    const ConvK ksel = sel == d ? k : make_convk(sel);
    pick_generic_tile(ksel, best_m, best_n);
    ConvK kk = k;
    kk.ksplit = choose_ksplit(ksel, best_m, best_n);
    if (kk.ksplit > 1 && splitk_bytes(k, kk.ksplit) > d->workspace_bytes) kk.ksplit = 1;
#define DBSR_CONV_CASE(M, N) if (best_m == M && best_n == N) return launch_conv<T, M, N>(kk, s);
    DBSR_CONV_CASE(4, 4) DBSR_CONV_CASE(4, 2) DBSR_CONV_CASE(4, 1)
    DBSR_CONV_CASE(2, 4) DBSR_CONV_CASE(2, 2) DBSR_CONV_CASE(2, 1)
    DBSR_CONV_CASE(1, 4) DBSR_CONV_CASE(1, 2) DBSR_CONV_CASE(1, 1)
#undef DBSR_CONV_CASE
    return launch_conv<T, 1, 1>(kk, s);
}

// ------------------------------------------------------------------------------------------------
// PixelShuffle upsampler (upsampling.py:51-66; decoders.py:43): 1x1 conv Cin -> s*s*32 (+ bias, act),
// written as PixelShuffle(s) of the result.  bf16, Cin padded to a multiple of 32 (<= 128), 32 output
// channels per sub-pixel, s*s % 8 == 0.
// Block = 8 waves over PG*16 consecutive low-res pixels; wave w owns sub-pixels w, w+8, ... (for s = 8
// the column sx = w of every sub-pixel row).  The pixels' K values are loaded once (PG*KS B-fragments);
// per sub-pixel the wave runs 2 x PG x KS MFMAs against that sub-pixel's 32 weight rows (prefetched
// one sub-pixel ahead), read in the order c = 8(m>>2) + 4h + (m&3) for MFMA row m of half h, so lane
// (g, col) ends up with channels 8g..8g+7 of its pixel: one 16-B store per lane, 64 contiguous bytes
// (the whole 32-channel output pixel) per 4 lanes.
// ------------------------------------------------------------------------------------------------
template <typename T, int PG, int KS>
__global__ __launch_bounds__(512) void upsample_shuffle_kernel(ConvK k) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane >> 4, col = lane & 15;
    const int s = k.shuffle, s2 = s * s;
    const int hw = k.out_h * k.out_w;
    Frag<T> b[PG][KS];
    int pf[PG], py[PG], px[PG];
#pragma unroll
    for (int j = 0; j < PG; ++j) {
        const int p = blockIdx.x * (PG * 16) + j * 16 + col;
        const bool ok = p < k.npix;
        const int f = ok ? p / hw : 0, rr = ok ? p - f * hw : 0;
        pf[j] = ok ? f : -1;
        py[j] = rr / k.out_w;
        px[j] = rr - py[j] * k.out_w;
        const T* xp = (const T*)k.x + map_frame(k.xm, f) * k.x_is + (long long)rr * k.x_ld + g * 8;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            if (ok) b[j][ks].load(xp + ks * 32);
            else b[j][ks].zero();
        }
    }
    const int m_row = 8 * (col >> 2) + (col & 3);           // + 4h: packed row within the sub-pixel's 32
    auto load_a = [&](int sub, Frag<T> (&a)[2][KS]) {
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int ks = 0; ks < KS; ++ks)
                a[h][ks].load((const T*)k.w + (long long)(sub * 32 + m_row + 4 * h) * k.Kp + ks * 32 + g * 8);
    };
    Frag<T> a_cur[2][KS], a_nxt[2][KS];
    int sub = wave;
    if (sub < s2) load_a(sub, a_cur);
    for (; sub < s2; sub += 8) {
        if (sub + 8 < s2) load_a(sub + 8, a_nxt);
        // the bias is the accumulators' initial value (bias + sum_k, the order upsample_blur_kernel sums in)
        f32x4_t bq[2] = {f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f}};
        if (k.bias) {
            bq[0] = *(const f32x4_t*)(k.bias + sub * 32 + 8 * g);
            bq[1] = *(const f32x4_t*)(k.bias + sub * 32 + 8 * g + 4);
        }
        f32x4_t acc[2][PG];
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int j = 0; j < PG; ++j) {
                acc[h][j] = bq[h];
#pragma unroll
                for (int ks = 0; ks < KS; ++ks) acc[h][j] = mma(a_cur[h][ks], b[j][ks], acc[h][j]);
            }
        const int sy = sub / s, sx = sub - sy * s;
#pragma unroll
        for (int j = 0; j < PG; ++j) {
            if (pf[j] < 0) continue;
            u32x4_t o;
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                o[e] = H16<T>::pack(apply_act(acc[0][j][2 * e], k.act), apply_act(acc[0][j][2 * e + 1], k.act));
                o[2 + e] = H16<T>::pack(apply_act(acc[1][j][2 * e], k.act), apply_act(acc[1][j][2 * e + 1], k.act));
            }
            const long long Y = (long long)py[j] * s + sy, X = (long long)px[j] * s + sx;
            *(u32x4_t*)((T*)k.y + map_frame(k.ym, pf[j]) * k.y_is + (Y * (k.out_w * s) + X) * k.y_ld + k.y_c0 +
                        8 * g) = o;
        }
        if (sub + 8 < s2) {
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int ks = 0; ks < KS; ++ks) a_cur[h][ks] = a_nxt[h][ks];
        }
    }
}

bool use_upsample(const dbsr_conv_desc* d, const ConvK& k) {
    return is16(d->x.dtype) && d->y.dtype == d->x.dtype && !d->precise && d->out_mode == DBSR_OUT_SHUFFLE && !d->gate.ptr &&
           d->kh == 1 && d->kw == 1 && d->stride == 1 && d->pad == 0 && k.cps == 32 &&
           (d->shuffle * d->shuffle) % 8 == 0 && k.Kp % 32 == 0 && k.Kp <= 128 && d->y.ld % 8 == 0 &&
           d->y.c0 % 8 == 0 && g_tiled_enabled;
}

template <typename T>
int launch_upsample(const ConvK& k, hipStream_t s) {
    // 2 pixel groups below 512 waves of work (the decoder's 18k LR pixels: pg 4 measured 46.6 vs 38.0 us;
    // PMC WRITE_SIZE equals the 75.5 MB written, so the kernel is latency-, not write-bound)
    const int pg = (k.npix + 63) / 64 >= 512 ? 4 : 2;
    const unsigned grid = (unsigned)((k.npix + pg * 16 - 1) / (pg * 16));
    const int ks = k.Kp / 32;
#define DBSR_UP(PG, KS) \
    if (pg == PG && ks == KS) hipLaunchKernelGGL((upsample_shuffle_kernel<T, PG, KS>), dim3(grid), dim3(512), 0, s, k)
    DBSR_UP(2, 1); DBSR_UP(2, 2); DBSR_UP(2, 3); DBSR_UP(2, 4);
    DBSR_UP(4, 1); DBSR_UP(4, 2); DBSR_UP(4, 3); DBSR_UP(4, 4);
#undef DBSR_UP
    DBSR_LAUNCH_CHECK();
    return 0;
}

// ------------------------------------------------------------------------------------------------
// PixelShuffle upsampler + Gaussian blur in one pass (upsampling.py:51-66, decoders.py:43): the
// decoder's 1x1 conv Cin -> 64 x 32 (+ bias, act), PixelShuffle(8) and the 3x3 depthwise blur with zero
// padding, without the pre-blur tensor's HBM round trip (75.5 MB written and read back at the bench shape).
//
// Persistent blocks of 8 waves (2 per SIMD).  Wave w keeps in registers the packed weight rows of output
// channels 4w..4w+3 for all 64 sub-pixels: 16 row blocks x KS k-steps (128 VGPRs at Cin 64).  Work unit =
// a 4x4 low-res tile = 32x32 output pixels.  Conv phase: the tile's 16 pixels and its ring of 20 (three
// 16-pixel MFMA column groups) run through the row blocks; lane (g, col) of row block rb gets channels
// 4w..4w+3 of sub-pixel (rb / 2, 4(rb & 1) + g) of pixel col, which -- + bias, act, rounded to T exactly as
// upsample_shuffle_kernel stores it -- goes to an LDS image of the tile's 32x32 output pixels plus a 1-pixel
// halo (of a ring pixel only the sub-pixels inside that halo are computed and kept; pixels outside the frame
// are zeros, the blur's padding).  Blur phase: thread (strip, column, 8-channel group) slides a 3-row window
// of horizontal sums down 8 output rows (the separable Gaussian: blur_row / blur_col, as blur3_h16_kernel
// sums), so the output is bitwise that of dbsr_conv2d followed by dbsr_gauss_blur3.  The image is double-buffered: one barrier per tile.
// Image pixel (Ys, Xs) = 64 B = 8 positions of 4 channels; channel quad q sits at position q ^ key, key =
// (Lx & 3) | (Ly & 1) << 2 of the pixel's low-res coordinates in the ringed tile, (Ly, Lx) = ((Ys + 7) / 8,
// (Xs + 7) / 8): the 16 lanes of a conv-phase ds_write_b64 (one sub-pixel of 16 low-res pixels, which
// without the key share one address mod 128 B) then hit 8 distinct positions (2-way, the minimum).
// ------------------------------------------------------------------------------------------------
#ifndef DBSR_UB_ABL
#define DBSR_UB_ABL 0        // timing-only ablations: 1 no conv phase, 2 no blur phase, 4 no blur stores
#endif
namespace ub {
constexpr int LT = 4, S = 8, HS = LT * S + 2, NPX = HS * HS;      // image: HS x HS pixels
constexpr int IMG_U2 = NPX * 8;                                   // ... in 8-B units
constexpr int ROWS = 2048;                                        // conv rows: 64 sub-pixels x 32 channels
__host__ __device__ constexpr int key(int Ly, int Lx) { return (Lx & 3) | ((Ly & 1) << 2); }
// ringed-tile coordinates (Ly, Lx) in [0, 6)^2 of column c of group G (0: the 16 interior pixels, 1 and 2:
// the 20 ring pixels: top row, bottom row, left column, right column); false past the ring
__device__ __forceinline__ bool ring_px(int G, int c, int& Ly, int& Lx) {
    if (G == 0) { Ly = 1 + (c >> 2); Lx = 1 + (c & 3); return true; }
    const int r = (G - 1) * 16 + c;
    if (r < 6) { Ly = 0; Lx = r; }
    else if (r < 12) { Ly = 5; Lx = r - 6; }
    else if (r < 16) { Ly = r - 11; Lx = 0; }
    else if (r < 20) { Ly = r - 15; Lx = 5; }
    else { Ly = 0; Lx = 0; return false; }
    return true;
}
// row blocks whose sub-pixels reach the halo of group G's pixels: group 1 (top: sub-row 7 = rb 14, 15;
// bottom: sub-row 0 = rb 0, 1; left: sub-column 7 = odd rb) and group 2 (right: sub-column 0 = even rb)
constexpr bool rb_used(int G, int rb) {
    return G == 0 || (G == 1 && (rb >= 14 || rb <= 1 || (rb & 1))) || (G == 2 && !(rb & 1));
}
}  // namespace ub

template <typename T, int KS, int ACT>
__global__ __launch_bounds__(512, 1) void upsample_blur_kernel(ConvK k, Blur3 kb, int tiles_x, int tiles_y,
                                                               int ntiles) {
    using namespace ub;
    auto act = [](float v) { return apply_act(v, ACT); };        // (compile-time: a runtime act branched per value)
    constexpr int UB_BATCH = KS == 2 ? 2 : 4;                     // row blocks per MFMA batch (registers at KS 2)
    __shared__ __attribute__((aligned(16))) u32x2_t img[2 * IMG_U2 + 64];   // + the conv phase's dummy slots
    __shared__ __attribute__((aligned(16))) float lbias[ROWS];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane >> 4, col = lane & 15;

    // the wave's weight rows: row m of row block rb = sub-pixel 4 rb + m / 4, channel 4 wave + m % 4, packed as
    // row sub * 32 + channel (dbsr_conv_pack_weights with shuffle)
    Frag<T> wr[16][KS];
#pragma unroll
    for (int rb = 0; rb < 16; ++rb)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
            wr[rb][ks].load((const T*)k.w + (long long)((4 * rb + (col >> 2)) * 32 + 4 * wave + (col & 3)) * k.Kp +
                            ks * 32 + g * 8);
    for (int i = threadIdx.x; i < ROWS; i += 512) lbias[i] = k.bias ? k.bias[i] : 0.f;

    const int Wh = k.in_w * S;                                    // output row length
    auto decode = [&](int t, int& f, int& ty, int& tx) {
        tx = t % tiles_x; t /= tiles_x;
        ty = t % tiles_y; f = t / tiles_y;
    };
    // B-fragments of the three column groups of tile t (zeros outside the frame / past the ring)
    auto load_b = [&](int t, Frag<T> (&b)[3][KS]) {
        int f, ty, tx;
        decode(t, f, ty, tx);
        const T* xf = (const T*)k.x + map_frame(k.xm, f) * k.x_is;
#pragma unroll
        for (int G = 0; G < 3; ++G) {
            int Ly, Lx;
            const bool in_ring = ring_px(G, col, Ly, Lx);
            const int ly = ty * LT + Ly - 1, lx = tx * LT + Lx - 1;
            const bool ok = in_ring && (unsigned)ly < (unsigned)k.in_h && (unsigned)lx < (unsigned)k.in_w;
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                if (ok) b[G][ks].load(xf + (long long)(ly * k.in_w + lx) * k.x_ld + ks * 32 + g * 8);
                else b[G][ks].zero();
            }
        }
    };

    Frag<T> bcur[3][KS];
    int t = blockIdx.x;
    if (t < ntiles) load_b(t, bcur);
    PIPE_STAMP(0);
    __syncthreads();                                              // lbias
    PIPE_STAMP(1);
    for (int it = 0; t < ntiles; ++it, t += gridDim.x) {
        int f, ty, tx;
        decode(t, f, ty, tx);
        u32x2_t* im = img + (it & 1) * IMG_U2;
        // lane-derived values recomputed per tile from an opaque copy of the thread index: hoisted out of the loop,
        // the conv phase's per-row-block LDS addresses and masks took ~40 registers and spilled
        int tid = threadIdx.x;
        asm volatile("" : "+v"(tid));
        const int lane = tid & 63, g = lane >> 4, col = lane & 15;
        PIPE_STAMP(2 + 4 * it);
        // ---- conv phase ----
        // branch-free: a lane whose sub-pixel falls outside the image writes its own dummy slot, pixels outside
        // the frame write zeros; row blocks in batches (MFMAs of a batch, then its epilogue) so the
        // compiler overlaps one batch's epilogue with the next batch's MFMAs
        StaticFor<0, (DBSR_UB_ABL & 1) ? 0 : 3>::run([&](auto G_) {
            constexpr int G = decltype(G_)::value;
            int Ly, Lx;
            const bool in_ring = ring_px(G, col, Ly, Lx);
            const int ly = ty * LT + Ly - 1, lx = tx * LT + Lx - 1;
            const bool inside = G == 0 || (in_ring && (unsigned)ly < (unsigned)k.in_h && (unsigned)lx < (unsigned)k.in_w);
            const int pos = wave ^ key(Ly, Lx);                 // channel quad `wave`'s position
            // byte address of this lane's quad in the image for row block 0 (row block rb adds a constant)
            const int lb = (((8 * Ly - 7) * HS + 8 * Lx - 7 + g) * 8 + pos) * 8;
            char* ib = (char*)(img + (it & 1) * IMG_U2) + lb;
            StaticFor<0, 16 / UB_BATCH>::run([&](auto bt_) {
                constexpr int bt = decltype(bt_)::value;
                f32x4_t acc[UB_BATCH];
                StaticFor<0, UB_BATCH>::run([&](auto j_) {
                    constexpr int j = decltype(j_)::value, rb = UB_BATCH * bt + j;
                    if constexpr (rb_used(G, rb)) {
                        // the bias is the accumulator's initial value (as upsample_shuffle_kernel sums)
                        acc[j] = *(const f32x4_t*)(lbias + (4 * rb + g) * 32 + 4 * wave);
#pragma unroll
                        for (int ks = 0; ks < KS; ++ks) acc[j] = mma(wr[rb][ks], bcur[G][ks], acc[j]);
                    }
                });
                StaticFor<0, UB_BATCH>::run([&](auto j_) {
                    constexpr int j = decltype(j_)::value, rb = UB_BATCH * bt + j;
                    if constexpr (!rb_used(G, rb)) return;
                    constexpr int sy = rb >> 1, sx0 = 4 * (rb & 1);
                    constexpr int off = (sy * HS + sx0) * 64;        // bytes past ib
                    u32x2_t o;
                    if constexpr (ACT == DBSR_ACT_RELU) {
                        // ReLU on the rounded values' sign bits (v_pk_max_i16 with 0): bitwise the rounding of the
                        // fp32 ReLU, -0 included
                        o[0] = relu16x2(H16<T>::pack(acc[j][0], acc[j][1]));
                        o[1] = relu16x2(H16<T>::pack(acc[j][2], acc[j][3]));
                    } else {
                        o[0] = H16<T>::pack(act(acc[j][0]), act(acc[j][1]));
                        o[1] = H16<T>::pack(act(acc[j][2]), act(acc[j][3]));
                    }
                    if constexpr (G == 0) {
                        *(u32x2_t*)(ib + off) = o;
                    } else {
                        const int Ys = 8 * Ly + sy - 7, Xs = 8 * Lx + sx0 + g - 7;
                        const bool keep = in_ring && (unsigned)Ys < (unsigned)HS && (unsigned)Xs < (unsigned)HS;
                        if (!inside) o = u32x2_t{0u, 0u};
                        *(u32x2_t*)(keep ? ib + off : (char*)(img + 2 * IMG_U2 + lane)) = o;
                    }
                });
            });
        });
        PIPE_STAMP(3 + 4 * it);
        // the next tile's input pixels, in flight over the blur phase (issued before its stores)
        if (t + (int)gridDim.x < ntiles) load_b(t + gridDim.x, bcur);
        __syncthreads();
        PIPE_STAMP(4 + 4 * it);
        // ---- blur phase: thread = (strip of 8 output rows, output column, 8-channel group) ----
        if constexpr ((DBSR_UB_ABL & 2) != 0) continue;
        const int cg = tid & 3, ox = (tid >> 2) & 31, st = tid >> 7;
        // raw 16-B read of the thread's 8 channels of image pixel (Ys, Xs) and its key's half swap (applied when the
        // row enters the window, an iteration after its reads were issued)
        auto raw = [&](int Ys, int Xs) {
            const int ky = key((Ys + 7) >> 3, (Xs + 7) >> 3);
            return *(const u32x4_t*)(im + (Ys * HS + Xs) * 8 + 2 * (cg ^ (ky >> 1)));
        };
        auto fix = [&](int Ys, int Xs, const u32x4_t& v) {
            return (key((Ys + 7) >> 3, (Xs + 7) >> 3) & 1) ? u32x4_t{v[2], v[3], v[0], v[1]} : v;
        };
        T* yb = (T*)k.y + map_frame(k.ym, f) * k.y_is + k.y_c0 + 8 * cg +
                ((long long)(ty * LT * S + 8 * st) * Wh + tx * LT * S + ox) * k.y_ld;
        // horizontal sums of window rows r, r + 1, r + 2 in h0, h1, h2 (blur_row / blur_col: the separable Gaussian in
        // blur3_h16_kernel's order); row r + 3's reads (wn) are issued an iteration ahead.  Unrolled with a scheduling
        // fence per row (without it the compiler hoisted every LDS read and spilled)
        const int y0 = 8 * st;
        float h0[8], h1[8], h2[8];
        {
            u32x4_t a[3], b[3], c[3];
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                a[j] = raw(y0, ox + j);
                b[j] = raw(y0 + 1, ox + j);
                c[j] = raw(y0 + 2, ox + j);
            }
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                a[j] = fix(y0, ox + j, a[j]);
                b[j] = fix(y0 + 1, ox + j, b[j]);
                c[j] = fix(y0 + 2, ox + j, c[j]);
            }
            blur_row<T>(kb, a[0], a[1], a[2], h0);
            blur_row<T>(kb, b[0], b[1], b[2], h1);
            blur_row<T>(kb, c[0], c[1], c[2], h2);
        }
        u32x4_t wn[3];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            __builtin_amdgcn_sched_barrier(0);              // (keeps each row's LDS reads in its own iteration)
            const int yn = min(y0 + r + 3, HS - 1);       // (the last iteration's read is unused)
#pragma unroll
            for (int j = 0; j < 3; ++j) wn[j] = raw(yn, ox + j);
            float acc[8];
            blur_col(kb, h0, h1, h2, acc);
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                h0[q] = h1[q];
                h1[q] = h2[q];
            }
#pragma unroll
            for (int j = 0; j < 3; ++j) wn[j] = fix(yn, ox + j, wn[j]);
            blur_row<T>(kb, wn[0], wn[1], wn[2], h2);
            if constexpr ((DBSR_UB_ABL & 4) != 0) {
                if (acc[0] == 123.f && acc[7] == 7.f) store8(yb, acc);
            } else {
                store8(yb + (long long)r * Wh * k.y_ld, acc);
            }
        }
        PIPE_STAMP(5 + 4 * it);
    }
}

// the fused upsampler + blur applies: 16-bit 1x1 conv Cin (<= 64, padded to 32 or 64) -> 64 sub-pixels x 32
// channels, PixelShuffle(8), low-res frame a multiple of 4 x 4, aligned NHWC output
bool use_upsample_blur(const dbsr_conv_desc* d) {
    if (!d || !is16(d->x.dtype) || d->y.dtype != d->x.dtype || d->precise || d->out_mode != DBSR_OUT_SHUFFLE) return false;
    if (d->shuffle != 8 || d->cout != 2048 || d->kh != 1 || d->kw != 1 || d->stride != 1 || d->pad != 0 ||
        d->dil != 1 || d->res.ptr || d->gate.ptr)
        return false;
    const int cp = cin_pad(d->cin);
    if (cp != 32 && cp != 64) return false;
    if (d->in_h % ub::LT || d->in_w % ub::LT || d->in_h != d->out_h || d->in_w != d->out_w) return false;
    if (d->x.ld % 8 || d->x.c0 % 8 || d->x.c0 + cp > d->x.ld) return false;
    if (d->y.ld % 8 || d->y.c0 % 8 || d->y.c0 + 32 > d->y.ld) return false;
    return (long long)d->n_frames * d->in_h * d->in_w * 64 < (1LL << 31);
}

// ------------------------------------------------------------------------------------------------
// Pointwise (1x1) projection: the merge's feat_project_layer (merging.py:34, 75: 1x1 conv 512 -> 64
// + ReLU over every frame's embedding).  HBM-bound (1 KB read per pixel, 128 B written): the kernel
// reads each pixel once with 16-B loads and never touches the weights in HBM after the prologue.
// Block = 8 waves.  The whole weight matrix (cout x Kp, <= 64 KB) is copied once per block into the
// LDS, 16-B chunk (row c, chunk q) at row c, position q ^ key(c) (key(c) = the MFMA row lane col that
// reads row c, so the 16 rows of one A fragment hit 16 distinct bank groups).  Each wave then takes
// groups of PG*16 pixels independently (no barriers): loads all PG x KS B-fragments of its pixels
// (16 KB in flight per wave at PG 1, Kp 512), runs CT x 2 x PG x KS MFMAs against A fragments read
// from the LDS, and stores 8 contiguous channels per lane (rows ordered c = 8(m>>2) + 4h + (m&3) as
// in upsample_shuffle_kernel).  16-bit, cin % 32 == 0, cout % 32 == 0, cout * cin <= 32768.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ int pw_key(int c) { return (c & 3) | ((c >> 1) & 12); }

template <typename T, int CT, int KS, int PG, int NW, int RES>
__global__ __launch_bounds__(NW * 64, CT > 2 ? 1 : (PG == 1 ? 4 : 2)) void conv1x1_kernel(ConvK k, int ngroups) {
    constexpr int KQ = KS * 4;                            // 16-B chunks per weight row
    __shared__ __attribute__((aligned(16))) u32x4_t pw_lds[CT * 32 * KQ];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane >> 4, col = lane & 15;
    for (int i = threadIdx.x; i < CT * 32 * KQ; i += NW * 64) {
        const int c = i / KQ, q = i - c * KQ;
        pw_lds[c * KQ + (q ^ pw_key(c))] = *((const u32x4_t*)k.w + (long long)c * (k.Kp / 8) + q);
    }
    __syncthreads();
    const int hw = k.out_h * k.out_w;
    constexpr bool HOIST = CT <= 2;                       // bias in registers across pixel groups (projections)
    f32x4_t bias[HOIST ? CT : 1][2];
    if constexpr (HOIST) {
#pragma unroll
        for (int ct = 0; ct < CT; ++ct)
#pragma unroll
            for (int h = 0; h < 2; ++h) bias[ct][h] = load_bias4(k, ct * 32 + 8 * g + 4 * h);
    }
    for (int grp = blockIdx.x * NW + wave; grp < ngroups; grp += gridDim.x * NW) {
        Frag<T> b[PG][KS];
        int pf[PG], prr[PG];
#pragma unroll
        for (int j = 0; j < PG; ++j) {
            const int p = grp * (PG * 16) + j * 16 + col;
            const bool ok = p < k.npix;
            const int f = ok ? p / hw : 0, rr = ok ? p - f * hw : 0;
            pf[j] = ok ? f : -1;
            prr[j] = rr;
            const T* xp = (const T*)k.x + map_frame(k.xm, f) * k.x_is + (long long)rr * k.x_ld + g * 8;
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                if (ok) b[j][ks].load(xp + ks * 32);
                else b[j][ks].zero();
            }
        }
        // the wide-cout dgrad (64 -> 512 + residual): the residual quads of RPD cout tiles issued together (RPD x 4
        // VGPRs), instead of one per cout tile (each tile's epilogue waited a full memory latency for its own).
        // bwd.proj.oth at configs[3]: one per tile 1006 us, RPD 16 889 (the 16-tile unroll spills 104 VGPRs), 8 831,
        // 4 805 (79 VGPRs; profiles/r06p_pw_prefetch_ab.txt)
#ifndef DBSR_PW_RPD
#define DBSR_PW_RPD 4
#endif
        constexpr bool RPRE = RES && CT > 2;
        constexpr int RPD = RPRE ? (DBSR_PW_RPD < CT ? DBSR_PW_RPD : CT) : 1;
        auto tile = [&](int ct, auto&& resq) {
            f32x4_t acc[2][PG];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                int c = ct * 32 + 8 * (col >> 2) + 4 * h + (col & 3);
                asm volatile("" : "+v"(c));            // keep the A reads in the loop (hoisted: 4 VGPRs per read)
                const u32x4_t* arow = pw_lds + c * KQ;
                const int key = pw_key(c);
#pragma unroll
                for (int j = 0; j < PG; ++j) acc[h][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int ks = 0; ks < KS; ++ks) {
                    Frag<T> a;
                    a.v = __builtin_bit_cast(bf16x8_t, arow[(ks * 4 + g) ^ key]);
#pragma unroll
                    for (int j = 0; j < PG; ++j) acc[h][j] = mma(a, b[j][ks], acc[h][j]);
                }
            }
            f32x4_t bv[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) bv[h] = HOIST ? bias[HOIST ? ct : 0][h] : load_bias4(k, ct * 32 + 8 * g + 4 * h);
#pragma unroll
            for (int j = 0; j < PG; ++j) {
                if (pf[j] < 0) continue;
                float v[8];
#pragma unroll
                for (int h = 0; h < 2; ++h)
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[4 * h + e] = apply_act(acc[h][j][e] + bv[h][e], k.act);
                if constexpr (RES) {                      // (training dgrad of the projection: + residual, post-act)
                    const u32x4_t rq = resq(j);
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        v[2 * e] = apply_act(v[2 * e] + H16<T>::lo(rq[e]), k.post_act);
                        v[2 * e + 1] = apply_act(v[2 * e + 1] + H16<T>::hi(rq[e]), k.post_act);
                    }
                }
                u32x4_t o;
#pragma unroll
                for (int e = 0; e < 4; ++e) o[e] = H16<T>::pack(v[2 * e], v[2 * e + 1]);
                *(u32x4_t*)((T*)k.y + map_frame(k.ym, pf[j]) * k.y_is + (long long)prr[j] * k.y_ld + k.y_c0 + ct * 32 +
                            8 * g) = o;
            }
        };
        if constexpr (RPRE) {
#pragma unroll 1
            for (int c0 = 0; c0 < CT; c0 += RPD) {
                u32x4_t rqc[RPD][PG];
#pragma unroll
                for (int j = 0; j < PG; ++j) {
                    const T* rb = (const T*)k.r + map_frame(k.rm, pf[j] < 0 ? 0 : pf[j]) * k.r_is +
                                  (long long)prr[j] * k.r_ld + k.r_c0 + 8 * g;
#pragma unroll
                    for (int i = 0; i < RPD; ++i)
                        rqc[i][j] = pf[j] >= 0 ? *(const u32x4_t*)(rb + (c0 + i) * 32) : u32x4_t{0u, 0u, 0u, 0u};
                }
#pragma unroll
                for (int i = 0; i < RPD; ++i) tile(c0 + i, [&](int j) { return rqc[i][j]; });
            }
        } else {
            constexpr int CTU = CT <= 2 ? CT : 1;        // (wide couts: one 32-cout tile at a time)
#pragma unroll CTU
            for (int ct = 0; ct < CT; ++ct)
                tile(ct, [&](int j) {
                    return *(const u32x4_t*)((const T*)k.r + map_frame(k.rm, pf[j]) * k.r_is + (long long)prr[j] * k.r_ld +
                                             k.r_c0 + ct * 32 + 8 * g);
                });
        }
    }
}

bool use_pointwise(const dbsr_conv_desc* d) {
    const int ct = d->cout / 32;
    return is16(d->x.dtype) && d->y.dtype == d->x.dtype && !d->precise && d->out_mode == DBSR_OUT_NHWC &&
           (!d->res.ptr || (d->res.dtype == d->y.dtype && d->res.ld % 8 == 0 && d->res.c0 % 8 == 0)) &&
           !d->gate.ptr && d->kh == 1 && d->kw == 1 && d->stride == 1 && d->pad == 0 &&
           d->cin % 32 == 0 && d->cin <= 512 && ((d->cin / 32) & (d->cin / 32 - 1)) == 0 && d->cout % 32 == 0 &&
           ct >= 1 && ct <= 16 && (ct & (ct - 1)) == 0 && d->cout * d->cin <= 32768 &&
           d->y.ld % 8 == 0 && d->y.c0 % 8 == 0 && g_tiled_enabled &&
           (long long)d->n_frames * d->out_h * d->out_w >= 4096;
}

template <typename T, int CT, int PG, int NW>
int launch_pointwise_cfg(const ConvK& k, hipStream_t s) {
    const int ngroups = (k.npix + PG * 16 - 1) / (PG * 16);
    const int ks = k.Kp / 32;
    const int lds = CT * 32 * k.Kp * 2;                 // bytes of the block's weight copy
    const unsigned grid = (unsigned)std::min((ngroups + NW - 1) / NW, 256 * (lds <= 40960 ? 3 : 2));
    // (weight copies up to 64 KiB: CT * KS <= 32; use_pointwise admits only those)
#define DBSR_PW(KS) \
    if constexpr (CT * KS <= 32) { \
        if (ks == KS) { \
            if (k.r) hipLaunchKernelGGL((conv1x1_kernel<T, CT, KS, PG, NW, 1>), dim3(grid), dim3(NW * 64), 0, s, k, ngroups); \
            else hipLaunchKernelGGL((conv1x1_kernel<T, CT, KS, PG, NW, 0>), dim3(grid), dim3(NW * 64), 0, s, k, ngroups); } }
    DBSR_PW(1) DBSR_PW(2) DBSR_PW(4) DBSR_PW(8) DBSR_PW(16)
#undef DBSR_PW
    DBSR_CHECK_ARG((ks == 1 || ks == 2 || ks == 4 || ks == 8 || ks == 16) && CT * ks <= 32,
                   "conv1x1: cin %d x cout %d not served", k.Kp, CT * 32);
    DBSR_LAUNCH_CHECK();
    return 0;
}

template <typename T, int CT>
int launch_pointwise_ct(const ConvK& k, hipStream_t s) {
    // 16-pixel groups, 8 waves, 4 waves per SIMD: proj_oth 55 us (32-pixel groups at 2 waves per SIMD,
    // 4 or 8 waves per block: 57-59 us)
    return launch_pointwise_cfg<T, CT, 1, 8>(k, s);
}

template <typename T>
int launch_pointwise(const ConvK& k, hipStream_t s) {
    switch (k.cout / 32) {
        case 16: return launch_pointwise_ct<T, 16>(k, s);   // (training: dgrad of the 512 -> 64 projection)
        case 8: return launch_pointwise_ct<T, 8>(k, s);
        case 4: return launch_pointwise_ct<T, 4>(k, s);
        case 2: return launch_pointwise_ct<T, 2>(k, s);
        default: return launch_pointwise_ct<T, 1>(k, s);
    }
}

ConvK make_convk(const dbsr_conv_desc* d) {
    ConvK k;
    k.x = d->x.ptr; k.x_is = d->x.img_stride; k.x_ld = d->x.ld; k.xm = d->x.map; k.in_h = d->in_h; k.in_w = d->in_w;
    // the channel offset is folded into the base pointer (x.c0 is a multiple of 8)
    const int esz = esize(d->x.dtype);
    k.x = (const char*)d->x.ptr + (long long)d->x.c0 * esz;
    const int CG = cin_pad(d->cin) / 8;
    k.CG = CG; k.KG = d->kh * d->kw * CG; k.KGp = round_up(k.KG, 4); k.Kp = k.KGp * 8;
    k.w = d->w; k.bias = d->bias; k.kw = d->kw; k.stride = d->stride; k.pad = d->pad; k.dil = d->dil; k.cout = d->cout;
    k.y = d->y.ptr; k.y_f32 = d->y.dtype == DBSR_F32; k.y_is = d->y.img_stride; k.y_ld = d->y.ld; k.y_c0 = d->y.c0;
    k.ym = d->y.map; k.out_h = d->out_h; k.out_w = d->out_w; k.act = d->act;
    k.r = d->res.ptr; k.r_is = d->res.img_stride; k.r_ld = d->res.ld; k.r_c0 = d->res.c0; k.rm = d->res.map;
    if (!k.r) k.rm = d->y.map;
    k.gt = d->gate.ptr; k.g_is = d->gate.img_stride; k.g_ld = d->gate.ld; k.g_c0 = d->gate.c0; k.gm = d->gate.map;
    if (!k.gt) k.gm = d->y.map;
    k.post_act = d->post_act; k.out_mode = d->out_mode; k.shuffle = d->shuffle;
    k.cps = d->out_mode == DBSR_OUT_SHUFFLE ? d->cout / (d->shuffle * d->shuffle) : 0;
    k.npix = (int)((long long)d->n_frames * d->out_h * d->out_w);
    k.vec_store = (d->out_mode != DBSR_OUT_NCHW_F32) && (d->y.ld % 4 == 0) && (d->y.c0 % 4 == 0);
    k.ksplit = 1;
    k.ws = (float*)d->workspace;
    k.cw = round_up(d->cout, 4);
    k.w_pipe = (const char*)d->w + (size_t)round_up(d->cout, 64) * k.Kp * esz;
    k.max_blocks = d->max_blocks;
    k.head_w = nullptr; k.head_b = nullptr; k.head_cout = 0;
    k.stage_epi = 0;
    return k;
}

}  // namespace

#ifdef DBSR_PIPE_STAMPS
extern "C" int dbsr_diag_pipe_stamps(unsigned long long* host, long long n) {
    const long long cap = (long long)sizeof(g_pipe_stamps) / 8;
    if (n > cap) n = cap;
    if (!host) {
        static unsigned long long zeros[sizeof(g_pipe_stamps) / 8];
        return hipMemcpyToSymbol(HIP_SYMBOL(g_pipe_stamps), zeros, sizeof(zeros)) == hipSuccess ? 0 : -1;
    }
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_pipe_stamps), n * 8) == hipSuccess ? (int)n : -1;
}
#endif

// the order dbsr_conv2d tries the kernels in, on the selection view (16-bit kernels first)
int kernel_for(const dbsr_conv_desc* d) {
    dbsr_conv_desc v;
    const dbsr_conv_desc* sel = sel_view(d, v);
    if (d->precise) return 0;
    if (use_upsample(sel, make_convk(sel))) return 3;
    if (use_pointwise(sel)) return 5;
    if (is16(d->x.dtype)) {
        if (pick_ws(sel)) return 4;
        if (use_ks128(sel)) return 7;
        if (pick_pipe(sel)) return 2;
        if (use_narrow(sel)) return 6;
        if (use_small(sel)) return 8;
    }
    return use_tiled(sel) ? 1 : 0;
}

// Host model of the highest channel of a pixel (c0 included) that any lane of the kernel dbsr_conv2d launches
// for `d` touches in y (which 0), the residual (1) or the gate (2); -1 when that tensor is unused (or y is not
// NHWC).  The pipelined and weight-stationary kernels address a partial cout tile's lanes through
// pipe_lane_ch / ws_lane_ch, enumerated here over the last cout tile; the other kernels bound every element by
// cout (epilogue_px's nvalid) and store only runs below cout; the weight-stationary residual arrives through a
// buffer resource that spans its frame's ld-wide pixels, so a run past the last pixel lands zeros.
int conv_lane_reach(const dbsr_conv_desc* d, int which) {
    const dbsr_tensor& t = which == 0 ? d->y : which == 1 ? d->res : d->gate;
    if (!t.ptr || d->out_mode != DBSR_OUT_NHWC) return -1;
    dbsr_conv_desc v;
    const dbsr_conv_desc* sel = sel_view(d, v);
    const int kf = kernel_for(d);
    int hi = d->cout - 1;
    if (kf == 2 && which > 0) {
        const int wm = pick_pipe(sel) == 2 ? 32 : 64;
        const int cb = (d->cout - 1) / wm * wm;                 // the last, possibly partial, cout tile
        for (int h = 0; h < wm / 32; ++h)
            for (int g = 0; g < 4; ++g) hi = std::max(hi, pipe_lane_ch(cb, h, g, d->cout) + 7);
    } else if (kf == 4 && which == 2) {
        const int wm = ws_narrow(sel) ? 32 : 64;
        const int ctb = (d->cout - 1) / wm * wm;
        for (int wc = 0; wc < wm / 32; ++wc)
            for (int g = 0; g < 4; ++g) hi = std::max(hi, ws_lane_ch(ctb, wc, g, d->cout) + 7);
    } else if (kf == 4 && which == 1) {
        return std::min(t.c0 + ((d->cout - 1) / 64 + 1) * 64 - 1, t.ld - 1);   // clamped by the frame's resource
    }
    return t.c0 + hi;
}

extern "C" int dbsr_conv_lane_reach(const dbsr_conv_desc* d, int which) {
    return (d && which >= 0 && which <= 2) ? conv_lane_reach(d, which) : -2;
}

extern "C" int dbsr_conv_kernel_for(const dbsr_conv_desc* d) {
    return d ? kernel_for(d) : -1;
}

extern "C" int dbsr_conv_dispatch_variant(const dbsr_conv_desc* d) {
    if (!d) return -1;
    dbsr_conv_desc v;
    const dbsr_conv_desc* sel = sel_view(d, v);
    const int kf = kernel_for(d);
    int var = 0;
    if (d->precise) {
        const long long np = (long long)sel->n_frames * sel->out_h * sel->out_w;
        var = np >= 512 * 256 ? 4 : np >= 512 * 128 ? 2 : 1;
    } else if (kf == 4) {
        var = ws_narrow(sel) ? 6408 : ws_short(sel) ? 1608 : 1616;
    } else if (kf == 7) {
        var = ks128::TW * 100 + ks128::TH;
    } else if (kf == 2) {
        var = pick_pipe(sel);
    } else if (kf == 1) {
        int wm, wn;
        pick_tiled_tile(sel, wm, wn);
        const int sp = tiled_ksplit(sel, wm, wn);
        var = (sp > 1 ? sp * 100000 : 0) + wm * 1000 + wn;
    } else if (kf == 0) {
        const ConvK k = make_convk(sel);
        int m, n;
        pick_generic_tile(k, m, n);
        var = m * 10000 + n * 1000 + choose_ksplit(k, m, n);
    }
    return kf * 1000000 + var;
}

extern "C" int dbsr_conv_head_ok(const dbsr_conv_desc* d) {
    if (!d) return 0;
    dbsr_conv_desc v;
    const dbsr_conv_desc* sel = sel_view(d, v);
    return pick_pipe(sel) == 2 && pipe_fits(2, d) && d->cout == 32 && d->res.ptr &&
           d->act == DBSR_ACT_NONE && d->post_act == DBSR_ACT_RELU;
}

extern "C" size_t dbsr_conv_workspace_bytes(const dbsr_conv_desc* d) {
    if (!d || d->precise) return 0;
    const int kf = kernel_for(d);
    dbsr_conv_desc v;
    const dbsr_conv_desc* sel = sel_view(d, v);
    if (kf == 1) {
        int wm, wn;
        pick_tiled_tile(sel, wm, wn);
        return splitk_bytes(make_convk(d), tiled_ksplit(sel, wm, wn));
    }
    if (kf != 0) return 0;
    const ConvK ksel = make_convk(sel);
    int m, n;
    pick_generic_tile(ksel, m, n);
    return splitk_bytes(make_convk(d), choose_ksplit(ksel, m, n));
}

extern "C" int dbsr_set_conv_algo(int algo) {
    DBSR_CHECK_ARG(algo >= 0 && algo <= 5, "set_conv_algo: 0 generic, 1 two-barrier tiled, 2 weight-stationary + "
                   "K-split 128-channel + pipelined + tiled (default), 3 pipelined wherever the shape allows, 4 as 2 "
                   "without the weight-stationary kernels, 5 as 2 without the K-split 128-channel kernel");
    g_tiled_enabled = algo >= 1;
    g_pipe_enabled = algo == 3 ? 2 : algo >= 2 ? 1 : 0;
    g_ws_enabled = algo == 2 || algo == 5;
    g_ks128_enabled = algo == 2;
    g_narrow_enabled = algo >= 2;
    g_small_enabled = algo >= 2;
    return 0;
}

// packed weights carry the chunk-major copy for the pipelined kernel when it can apply
inline bool has_pipe_copy(int cin, int kh, int kw) { return kh == 3 && kw == 3 && cin > 16; }

extern "C" size_t dbsr_conv_packed_elems(int cout, int cin, int kh, int kw) {
    const int KGp = round_up(kh * kw * (cin_pad(cin) / 8), 4);
    const size_t rows = (size_t)round_up(cout, 64) * KGp * 8;
    return has_pipe_copy(cin, kh, kw) ? 2 * rows : rows;
}

extern "C" int dbsr_conv_pack_weights(const float* w_f32, const float* bias_f32, int cout, int cin, int kh, int kw,
                                      int dtype, int shuffle, void* w_packed, float* bias_out, void* stream) {
    DBSR_CHECK_ARG(w_f32 && w_packed, "pack_weights: null pointer");
    DBSR_CHECK_ARG(cout > 0 && cin > 0 && kh > 0 && kw > 0, "pack_weights: bad shape");
    DBSR_CHECK_ARG(dtype == DBSR_F32 || is16(dtype), "pack_weights: bad dtype");
    if (shuffle > 1)
        DBSR_CHECK_ARG(cout % (shuffle * shuffle) == 0 && (cout / (shuffle * shuffle)) % 4 == 0,
                       "pack_weights: cout %d not divisible for shuffle %d", cout, shuffle);
    const int CG = cin_pad(cin) / 8, KG = kh * kw * CG, KGp = round_up(KG, 4), Kp = KGp * 8;
    const int cout_pad = round_up(cout, 64);
    const long long total = (long long)cout_pad * Kp;
    hipLaunchKernelGGL(pack_weights_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       w_f32, bias_f32, cout, cin, kh, kw, CG, KG, Kp, cout_pad, shuffle, dtype,
                       w_packed, bias_out);
    DBSR_LAUNCH_CHECK();
    if (has_pipe_copy(cin, kh, kw) && is16(dtype)) {
        hipLaunchKernelGGL(pack_weights_pipe_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                           (hipStream_t)stream, (const bf16_t*)w_packed, CG, Kp, cout <= 32 ? 32 : 64, total,
                           (bf16_t*)w_packed + total);
        DBSR_LAUNCH_CHECK();
    }
    return 0;
}

extern "C" long long dbsr_pack_batch_prepare(dbsr_pack_job* jobs, int n) {
    if (!jobs || n <= 0) { dbsr_set_error("pack_batch_prepare: no jobs"); return -1; }
    long long blk = 0;
    for (int i = 0; i < n; ++i) {
        dbsr_pack_job& j = jobs[i];
        if (!j.w || !j.w_packed || j.cout <= 0 || j.cin <= 0 || j.kh <= 0 || j.kw <= 0 ||
            !(j.dtype == DBSR_F32 || is16(j.dtype)) || j.shuffle < 1) {
            dbsr_set_error("pack_batch_prepare: bad job %d", i);
            return -1;
        }
        if (j.shuffle > 1 && (j.transposed || j.cout % (j.shuffle * j.shuffle) || (j.cout / (j.shuffle * j.shuffle)) % 4)) {
            dbsr_set_error("pack_batch_prepare: job %d: cout %d not divisible for shuffle %d", i, j.cout, j.shuffle);
            return -1;
        }
        if (j.transposed && (j.lo < 0 || j.src_cin < j.lo + j.cout)) {
            dbsr_set_error("pack_batch_prepare: job %d: rows [%d, %d) past the source's %d input channels", i, j.lo,
                      j.lo + j.cout, j.src_cin);
            return -1;
        }
        const PackGeom g = pack_geom(j);
        j.blk0 = blk;
        blk += ((g.pipe ? 2 : 1) * g.rows + 255) / 256;
    }
    if (blk >= (1LL << 31)) { dbsr_set_error("pack_batch_prepare: too many elements"); return -1; }
    return blk;
}

extern "C" int dbsr_conv_pack_weights_batch(const dbsr_pack_job* jobs_dev, int n, long long n_blocks, void* stream) {
    DBSR_CHECK_ARG(jobs_dev && n > 0 && n_blocks > 0 && n_blocks < (1LL << 31), "pack_weights_batch: bad arguments");
    hipLaunchKernelGGL(pack_weights_batch_kernel, dim3((unsigned)n_blocks), dim3(256), 0, (hipStream_t)stream,
                       jobs_dev, n);
    DBSR_LAUNCH_CHECK();
    return 0;
}

extern "C" int dbsr_conv2d(const dbsr_conv_desc* d, void* stream) {
    DBSR_CHECK_ARG(d, "conv2d: null desc");
    DBSR_CHECK_ARG(d->x.ptr && d->w && d->y.ptr, "conv2d: null pointer");
    DBSR_CHECK_ARG(d->x.dtype == DBSR_F32 || is16(d->x.dtype), "conv2d: bad input dtype");
    DBSR_CHECK_ARG(d->y.dtype == DBSR_F32 || d->y.dtype == d->x.dtype, "conv2d: output dtype must be f32 or input dtype");
    DBSR_CHECK_ARG(d->n_frames > 0 && d->in_h > 0 && d->in_w > 0 && d->out_h > 0 && d->out_w > 0, "conv2d: bad sizes");
    DBSR_CHECK_ARG(d->cin > 0 && d->cout > 0 && d->kh > 0 && d->kw > 0 && d->stride > 0 && d->dil > 0, "conv2d: bad shape");
    DBSR_CHECK_ARG(d->x.ld % 8 == 0 && d->x.c0 % 8 == 0, "conv2d: input ld/c0 must be multiples of 8 (got %d/%d)",
                   d->x.ld, d->x.c0);
    DBSR_CHECK_ARG(d->x.c0 + cin_pad(d->cin) <= d->x.ld, "conv2d: input slice [c0, c0+cin_pad) exceeds ld");
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
    if (d->gate.ptr)
        DBSR_CHECK_ARG(d->gate.dtype == d->y.dtype && d->gate.map.fpg > 0 && d->out_mode == DBSR_OUT_NHWC && !d->precise,
                       "conv2d: gate must be an NHWC tensor of the output dtype (NHWC output)");
    // every lane's reads of the residual / gate and its stores stay inside the pixel's [c0, ld) slice, also for
    // a partial cout tile at the last pixel of the last frame (where a run past ld would leave the allocation)
    if (d->res.ptr) DBSR_CHECK_ARG(d->res.c0 + d->cout <= d->res.ld, "conv2d: residual slice exceeds ld");
    if (d->gate.ptr) DBSR_CHECK_ARG(d->gate.c0 + d->cout <= d->gate.ld, "conv2d: gate slice exceeds ld");
    for (int w = 0; w < 3; ++w) {
        const dbsr_tensor& t = w == 0 ? d->y : w == 1 ? d->res : d->gate;
        const int reach = conv_lane_reach(d, w);
        DBSR_CHECK_ARG(reach < t.ld, "conv2d: a lane of the %s would address channel %d of a %d-channel pixel",
                       w == 0 ? "output" : w == 1 ? "residual" : "gate", reach, t.ld);
    }
    const long long npix = (long long)d->n_frames * d->out_h * d->out_w;
    DBSR_CHECK_ARG(npix < (1LL << 31), "conv2d: too many pixels");

    DBSR_CHECK_ARG(d->plan_h >= 0, "conv2d: plan_h must be >= 0");
    ConvK k = make_convk(d);
    hipStream_t s = (hipStream_t)stream;
    dbsr_conv_desc v;
    const dbsr_conv_desc* sel = sel_view(d, v);
    const long long npix_sel = (long long)sel->n_frames * sel->out_h * sel->out_w;
    if (d->precise && d->x.dtype == DBSR_F16) {
        DBSR_CHECK_ARG(d->y.dtype == DBSR_F32 && d->cout <= 16, "conv2d: precise mode needs fp32 output, cout <= 16");
        k.ksplit = 1;
        if (npix_sel >= 512 * 256) return launch_conv<float, 1, 4, f16_t>(k, s);
        if (npix_sel >= 512 * 128) return launch_conv<float, 1, 2, f16_t>(k, s);
        return launch_conv<float, 1, 1, f16_t>(k, s);
    }
    if (d->precise && d->x.dtype == DBSR_BF16) {
        // bf16 activations, fp32-packed weights, fp32 MFMA: small fp32-output heads (the RGB predictor)
        DBSR_CHECK_ARG(d->y.dtype == DBSR_F32 && d->cout <= 16, "conv2d: precise mode needs fp32 output, cout <= 16");
        k.ksplit = 1;
        if (npix_sel >= 512 * 256) return launch_conv<float, 1, 4, bf16_t>(k, s);
        if (npix_sel >= 512 * 128) return launch_conv<float, 1, 2, bf16_t>(k, s);
        return launch_conv<float, 1, 1, bf16_t>(k, s);
    }
    if (use_upsample(sel, k)) return d->x.dtype == DBSR_F16 ? launch_upsample<f16_t>(k, s) : launch_upsample<bf16_t>(k, s);
    if (use_pointwise(sel)) return d->x.dtype == DBSR_F16 ? launch_pointwise<f16_t>(k, s) : launch_pointwise<bf16_t>(k, s);
    if (d->x.dtype == DBSR_F16) return dispatch_conv<f16_t>(k, d, sel, s);
    return d->x.dtype == DBSR_BF16 ? dispatch_conv<bf16_t>(k, d, sel, s) : dispatch_conv<float>(k, d, sel, s);
}

extern "C" int dbsr_resblock_ok(const dbsr_conv_desc* c1, const dbsr_conv_desc* c2) {
    return resblock_channels(c1, c2) && c2->y.ptr && resblock_out_disjoint(c1, c2, nullptr, 0) ? 1 : 0;
}

int resblock_launch(const dbsr_conv_desc* c1, const dbsr_conv_desc* c2, const float* head_w, const float* head_b,
                    int head_cout, const dbsr_tensor* head_out, void* stream) {
    DBSR_CHECK_ARG(c1 && c2 && c1->x.ptr && c1->w && c2->w, "resblock: null pointer");
    DBSR_CHECK_ARG(head_out || c2->y.ptr, "resblock: null output");
    DBSR_CHECK_ARG(c1->x.map.fpg > 0 && c2->y.map.fpg > 0 && c1->n_frames > 0, "resblock: bad frame map / sizes");
    const int C = resblock_channels(c1, c2);
    DBSR_CHECK_ARG(C, "resblock: needs two 16-bit 3x3/s1/p1 C -> C convs, C = 32 or 64 (conv1 ReLU; conv2 residual = "
                   "conv1's input, post-ReLU), frames a multiple of 32 x 16 (C 32) / 16 x 16 (C 64), NHWC slices "
                   "aligned to 8");
    DBSR_CHECK_ARG(!head_out || C == 32, "resblock_head: 32-channel ResBlocks only");
    const ConvK k1 = make_convk(c1);
    ConvK k2 = make_convk(c2);
    if (C == 64) {
        DBSR_CHECK_ARG(resblock_out_disjoint(c1, c2, nullptr, 0),
                       "resblock: the output must not overlap the input x (other blocks still read x's halos)");
        return resblock64_launch(k1, k2, c1->n_frames, c1->x.dtype == DBSR_F16, c1->max_blocks, num_cus(),
                                 (hipStream_t)stream);
    }
    if (head_out) {
        DBSR_CHECK_ARG(head_w && head_out->ptr, "resblock_head: null pointer");
        DBSR_CHECK_ARG(head_cout >= 1 && head_cout <= 4, "resblock_head: head_cout must be 1..4");
        DBSR_CHECK_ARG(head_out->dtype == DBSR_F32 && head_out->map.fpg > 0, "resblock_head: fp32 NCHW output");
        k2.head_w = head_w; k2.head_b = head_b; k2.head_cout = head_cout;
        k2.y = head_out->ptr; k2.y_f32 = 1; k2.y_is = head_out->img_stride; k2.y_ld = 1; k2.y_c0 = 0;
        k2.ym = head_out->map;
    }
    DBSR_CHECK_ARG(resblock_out_disjoint(c1, c2, head_out, head_cout),
                   "resblock: the output must not overlap the input x (other blocks still read x's halos)");
    const int tiles_x = c1->in_w / rbk::TW, tiles_y = c1->in_h / rbk::TH;
    const int ntiles = c1->n_frames * tiles_x * tiles_y;
    int grid = c1->max_blocks > 0 ? std::min(c1->max_blocks, num_cus()) : num_cus();
    grid = std::min(grid, ntiles);
    DBSR_CHECK_ARG(rb_mapping_ok(grid, ntiles), "resblock: tile mapping out of range (grid %d, %d tiles)", grid, ntiles);
    hipStream_t s = (hipStream_t)stream;
    if (k2.head_w) {
        if (c1->x.dtype == DBSR_F16)
            hipLaunchKernelGGL((resblock32_kernel<f16_t, true>), dim3(grid), dim3(512), 0, s, k1, k2, tiles_x, tiles_y, ntiles);
        else
            hipLaunchKernelGGL((resblock32_kernel<bf16_t, true>), dim3(grid), dim3(512), 0, s, k1, k2, tiles_x, tiles_y, ntiles);
    } else {
        if (c1->x.dtype == DBSR_F16)
            hipLaunchKernelGGL((resblock32_kernel<f16_t, false>), dim3(grid), dim3(512), 0, s, k1, k2, tiles_x, tiles_y, ntiles);
        else
            hipLaunchKernelGGL((resblock32_kernel<bf16_t, false>), dim3(grid), dim3(512), 0, s, k1, k2, tiles_x, tiles_y, ntiles);
    }
    DBSR_LAUNCH_CHECK();
    return 0;
}

extern "C" int dbsr_resblock(const dbsr_conv_desc* c1, const dbsr_conv_desc* c2, void* stream) {
    return resblock_launch(c1, c2, nullptr, nullptr, 0, nullptr, stream);
}

extern "C" int dbsr_resblock_head(const dbsr_conv_desc* c1, const dbsr_conv_desc* c2, const float* head_w,
                                  const float* head_b, int head_cout, dbsr_tensor head_out, void* stream) {
    return resblock_launch(c1, c2, head_w, head_b, head_cout, &head_out, stream);
}

extern "C" int dbsr_conv_shuffle_blur_ok(const dbsr_conv_desc* d) { return use_upsample_blur(d) ? 1 : 0; }

extern "C" int dbsr_conv_shuffle_blur(const dbsr_conv_desc* d, const float* k9, void* stream) {
    DBSR_CHECK_ARG(d && k9 && d->x.ptr && d->w && d->y.ptr, "conv_shuffle_blur: null pointer");
    DBSR_CHECK_ARG(d->x.map.fpg > 0 && d->y.map.fpg > 0, "conv_shuffle_blur: frame map fpg must be > 0");
    DBSR_CHECK_ARG(d->n_frames > 0, "conv_shuffle_blur: bad sizes");
    DBSR_CHECK_ARG(use_upsample_blur(d), "conv_shuffle_blur: needs a 16-bit 1x1 conv cin <= 64 -> 2048 with "
                   "PixelShuffle(8) output (32 channels), a low-res frame of multiples of 4, aligned NHWC slices");
    const ConvK k = make_convk(d);
    Blur3 kk;
    DBSR_CHECK_ARG(blur_separable(k9, kk), "conv_shuffle_blur: the blur kernel must be separable (a Gaussian)");
    const int tiles_x = d->in_w / ub::LT, tiles_y = d->in_h / ub::LT;
    const int ntiles = d->n_frames * tiles_x * tiles_y;
    int grid = d->max_blocks > 0 ? std::min(d->max_blocks, num_cus()) : num_cus();
    grid = std::min(grid, ntiles);
    hipStream_t s = (hipStream_t)stream;
#define DBSR_UB(TT, KS, ACT) \
    hipLaunchKernelGGL((upsample_blur_kernel<TT, KS, ACT>), dim3(grid), dim3(512), 0, s, k, kk, tiles_x, tiles_y, ntiles)
#define DBSR_UB_ACT(TT, KS)                                   \
    switch (d->act) {                                         \
        case DBSR_ACT_RELU: DBSR_UB(TT, KS, DBSR_ACT_RELU); break;   \
        case DBSR_ACT_LRELU: DBSR_UB(TT, KS, DBSR_ACT_LRELU); break; \
        default: DBSR_UB(TT, KS, DBSR_ACT_NONE); break;             \
    }
    if (k.Kp == 64) {
        if (d->x.dtype == DBSR_F16) { DBSR_UB_ACT(f16_t, 2) } else { DBSR_UB_ACT(bf16_t, 2) }
    } else {
        if (d->x.dtype == DBSR_F16) { DBSR_UB_ACT(f16_t, 1) } else { DBSR_UB_ACT(bf16_t, 1) }
    }
#undef DBSR_UB_ACT
#undef DBSR_UB
    DBSR_LAUNCH_CHECK();
    return 0;
}

extern "C" int dbsr_conv2d_head(const dbsr_conv_desc* d, const float* head_w, const float* head_b, int head_cout,
                                dbsr_tensor head_out, void* stream) {
    DBSR_CHECK_ARG(d && head_w && head_out.ptr, "conv2d_head: null pointer");
    DBSR_CHECK_ARG(dbsr_conv_head_ok(d), "conv2d_head: the conv must be a pipelined 32-channel ResBlock conv2 "
                   "(bf16 3x3/s1/p1, residual, act none, post-act ReLU, width %% 64 == 0, height %% 8 == 0)");
    DBSR_CHECK_ARG(head_cout >= 1 && head_cout <= 4, "conv2d_head: head_cout must be 1..4");
    DBSR_CHECK_ARG(head_out.dtype == DBSR_F32 && head_out.map.fpg > 0, "conv2d_head: fp32 NCHW output");
    DBSR_CHECK_ARG(d->x.ld % 8 == 0 && d->x.c0 % 8 == 0 && d->x.c0 + cin_pad(d->cin) <= d->x.ld,
                   "conv2d_head: bad input slice");
    DBSR_CHECK_ARG(d->res.dtype == d->x.dtype && d->res.map.fpg > 0, "conv2d_head: residual dtype must equal input dtype");
    ConvK k = make_convk(d);
    k.head_w = head_w; k.head_b = head_b; k.head_cout = head_cout;
    k.y = head_out.ptr; k.y_f32 = 1; k.y_is = head_out.img_stride; k.y_ld = 1; k.y_c0 = 0; k.ym = head_out.map;
    if (d->x.dtype == DBSR_F16) return launch_pipe<f16_t, 32, 64, 8>(k, d->n_frames, (hipStream_t)stream);
    return launch_pipe<bf16_t, 32, 64, 8>(k, d->n_frames, (hipStream_t)stream);
}
