// Fused PWC-Net decoder DenseNet for the coarse pyramid levels (pwcnet.py:115-184, Decoder.forward
// :153-184): the five 3x3 convs of a level (each LeakyReLU(0.1), its output concatenated in front of its
// input: cat([conv(x), x], 1)) and the 2-channel flow conv, in one launch.
//
// At levels 6..3 a pair's feature map is 1x1 .. 8x8 pixels, so the per-conv launches of the generic
// kernel (plus their split-K finalize launches) were latency-bound: ~100-150 us per level for a few
// hundred MFLOP.  Here one block (8 waves; waves split each conv's 16-cout blocks) owns `ppb` whole pairs
// (one 16-slot MFMA column tile of pairs, or one pair of up to 64 pixels = NT tiles) and keeps their dense buffer D (all ld channels, the same NHWC channel layout the engine uses:
// [dense4 | dense3 | dense2 | dense1 | dense0 | corr, first, upflow, upfeat]) in LDS for the whole
// level; each conv reads its input slice from LDS, streams its packed weights (the generic kernel's
// [cout][tap][channel] layout) from L2 as MFMA A-fragments, and writes LeakyReLU(conv + bias) back
// into LDS for the next conv.  The dense channels go back to global D at the end (the next level's
// upfeat ConvT reads all of D); the flow conv writes fp32 flow.  The base channels (correlation, first
// features, upflow, upfeat) are produced by the level's prologue kernels as before.
#include "common.hpp"

#include <algorithm>
#include <type_traits>

using namespace dbsr;

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bfv8_t;
typedef __attribute__((ext_vector_type(8))) _Float16 hv8_t;

template <typename T>
__device__ __forceinline__ f32x4_t mma16x16x32(bf16x8_t a, bf16x8_t b, f32x4_t c) {
    if constexpr (std::is_same<T, bf16_t>::value)
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bfv8_t, a), __builtin_bit_cast(bfv8_t, b), c,
                                                       0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(hv8_t, a), __builtin_bit_cast(hv8_t, b), c,
                                                      0, 0, 0);
}

struct DenseConv {
    const void* w_pipe;     // chunk-major copy of the packed weights (after the [cout_pad][Kp] rows)
    const float* bias;
    int Kp, cg;             // packed K, 8-channel input groups per tap
    int start;              // first input channel in D
    int cout, out_off;      // output channels and their offset in D (conv 5: the flow, fp32 to `flow`)
};

struct DenseArgs {
    int P, h, w, ld, ppb, dense_ch;      // pairs, level size, D channels, pairs per block, [0, dense_ch) written
    dbsr_tensor D;                        // [P][h][w][ld]
    dbsr_tensor flow;                     // fp32 [P][h][w][>= 2]
    DenseConv cv[6];
};

#ifdef DBSR_PIPE_STAMPS
__device__ unsigned long long g_dense_stamps[128 * 8 * 16];
#define DSTAMP(slot) do { if ((threadIdx.x & 63) == 0 && blockIdx.x < 128) g_dense_stamps[(blockIdx.x * 8 + (threadIdx.x >> 6)) * 16 + (slot)] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define DSTAMP(slot) do { } while (0)
#endif
constexpr int KCH = 16;                  // k-steps of A-fragments per load chunk (two chunks in flight per wave)

// LDS tile capacity (elements) per instantiation: NT = 1 serves levels 6..4 (<= 16 pixel slots), NT = 4
// level 3 (one 8x8 pair); the tile holds each pair with a one-pixel zero border
template <int NT> struct DenseTile { static constexpr int ELEMS = NT == 1 ? 72 * 616 : 100 * 648; };

template <typename T, int NT>
__global__ __launch_bounds__(512) void pwc_dense_kernel(DenseArgs a) {
    // D of the block's pairs with a zero border ((h+2) x (w+2) rows of ld channels, +8 channels of row
    // padding so the 16 rows of a B-fragment read spread over the banks): a 3x3 tap is then one uniform
    // row offset and the B gathers need no bounds tests
    __shared__ __attribute__((aligned(16))) u32x4_t smem[DenseTile<NT>::ELEMS / 8];
    __shared__ f32x4_t red[7 * NT * 64];  // K-split partial sums: (kid - 1) * mb + m0, tile, lane
    T* tile = (T*)smem;
    const int lds_ld = a.ld + 8;
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g = lane >> 4, col = lane & 15;
    const int hw = a.h * a.w, bw = a.w + 2, bhw = (a.h + 2) * bw;
    const int pair0 = blockIdx.x * a.ppb;
    const int npairs = min(a.ppb, a.P - pair0);
    const int np = npairs * hw;                           // valid pixel slots of this block
    const int c8 = a.ld / 8;
    DSTAMP(0);

    for (int i = threadIdx.x; i < npairs * bhw * (lds_ld / 8); i += 512)
        *(u32x4_t*)(tile + i * 8) = u32x4_t{0u, 0u, 0u, 0u};
    __syncthreads();
    for (int i = threadIdx.x; i < np * c8; i += 512) {
        const int slot = i / c8, c = i - slot * c8;
        const int pl = slot / hw, px = slot - pl * hw, y = px / a.w, x = px - y * a.w;
        *(u32x4_t*)(tile + (pl * bhw + (y + 1) * bw + x + 1) * lds_ld + c * 8) =
            *(const u32x4_t*)(img_ptr<T>(a.D, pair0 + pl) + (long long)px * a.D.ld + c * 8);
    }
    // this lane's 3x3 window origin (bordered coordinates) per column tile; pad slots read pair 0's rows
    // (finite values; their MFMA columns are discarded)
    int base[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const int slot = t * 16 + col;
        const int pl = slot / hw, px = slot - pl * hw, y = px / a.w, x = px - y * a.w;
        base[t] = (slot < np ? (pl * bhw + y * bw + x) * lds_ld : 0) + g * 8;
    }
    const bool single = a.h == 1 && a.w == 1;             // 1x1 level: only the centre tap sees data
    __syncthreads();

    for (int ci = 0; ci < 6; ++ci) {
        DSTAMP(1 + ci * 2);
        const DenseConv cv = a.cv[ci];
        const int mb = (cv.cout + 15) / 16;
        const int gpt = cv.cg / 4;                        // k-steps per tap
        const int ksteps = single ? gpt : 9 * gpt;
        const int kfirst = single ? 4 * gpt : 0;          // packed k-step of the first live step
        // waves = (cout block m0, K slice kid): convs with few cout blocks split K over more waves, so no
        // wave runs a long serial chain of weight-chunk loads
        const int ksplit = mb >= 5 ? 1 : mb >= 3 ? 2 : mb == 2 ? 4 : 8;
        const int m0 = wave / ksplit, kid = wave - m0 * ksplit;
        const int nch = (ksteps + KCH - 1) / KCH;
        f32x4_t acc[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        if (m0 < mb) {
            // A-fragments from the chunk-major copy of the packed weights (dbsr_conv_pack_weights' pipe copy,
            // [cout / 16][channel quad c][tap][4 k-groups][16 rows][8]): one contiguous KiB per k-step.  (Row-
            // major rows 2-6 KiB apart put each wave load on 16 pages; the TLB, not the MFMAs, set the time.)
            // k-step ks = c * 9 + tap (single: ks = c, tap 4)
            const T* wblk = (const T*)cv.w_pipe + (long long)m0 * gpt * 9 * 512 + lane * 8;
            auto load_a = [&](int ch, u32x4_t (&dst)[KCH]) {
                const int ks0 = min(ch, nch - 1) * KCH;
#pragma unroll
                for (int j = 0; j < KCH; ++j) {
                    const int ks = min(ks0 + j, ksteps - 1);
                    const int piece = single ? ks * 9 + 4 : ks;
                    dst[j] = *(const u32x4_t*)(wblk + piece * 512);
                }
            };
            auto tap_row = [&](int tap) { return ((tap / 3) * bw + tap % 3) * lds_ld + cv.start; };
            auto compute = [&](int ch, const u32x4_t (&ab)[KCH]) {
                constexpr int PD = NT == 1 ? 8 : 2;       // B-fragment reads in flight ahead of the MFMAs
                const int ks0 = ch * KCH;
                int c = single ? ks0 : ks0 / 9;           // read pointer: the next step to fetch
                int tap = single ? 4 : ks0 - c * 9;
                bf16x8_t Bq[PD][NT];
                auto fetch = [&](bf16x8_t (&dst)[NT]) {
                    const int off = tap_row(tap) + c * 32;
#pragma unroll
                    for (int t = 0; t < NT; ++t) dst[t] = *(const bf16x8_t*)(tile + base[t] + off);
                    if (single) {
                        ++c;
                    } else if (++tap == 9) {
                        tap = 0;
                        ++c;
                    }
                };
#pragma unroll
                for (int d = 0; d < PD; ++d)
                    if (ks0 + d < ksteps) fetch(Bq[d]);
#pragma unroll
                for (int j = 0; j < KCH; ++j) {
                    if (ks0 + j >= ksteps) break;
                    bf16x8_t B[NT];
#pragma unroll
                    for (int t = 0; t < NT; ++t) B[t] = Bq[j % PD][t];
                    if (j + PD < KCH && ks0 + j + PD < ksteps) fetch(Bq[j % PD]);
                    const bf16x8_t A = __builtin_bit_cast(bf16x8_t, ab[j]);
#pragma unroll
                    for (int t = 0; t < NT; ++t) acc[t] = mma16x16x32<T>(A, B[t], acc[t]);
                }
            };
            // this wave's chunks kid, kid + ksplit, ...: the next one streams from L2 during the MFMAs
            u32x4_t a0[KCH], a1[KCH];
            load_a(kid, a0);
            for (int c = kid; c < nch; c += 2 * ksplit) {
                load_a(c + ksplit, a1);
                compute(c, a0);
                load_a(c + 2 * ksplit, a0);
                if (c + ksplit < nch) compute(c + ksplit, a1);
            }
            DSTAMP(2 + ci * 2);
            if (kid > 0) {
#pragma unroll
                for (int t = 0; t < NT; ++t) red[(((kid - 1) * mb + m0) * NT + t) * 64 + lane] = acc[t];
            }
        }
        if (ksplit > 1) __syncthreads();
        if (m0 < mb && kid == 0) {
            for (int k2 = 1; k2 < ksplit; ++k2) {
#pragma unroll
                for (int t = 0; t < NT; ++t) acc[t] += red[(((k2 - 1) * mb + m0) * NT + t) * 64 + lane];
            }
            // epilogue: MFMA row 4g + r of block m0 is cout 32(m0 >> 1) + 8g + 4(m0 & 1) + r (the copy's row
            // permutation, pipe_cout_perm)
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const int slot = t * 16 + col;
                if (slot >= np) continue;
                const int pl = slot / hw, px = slot - pl * hw, y = px / a.w, x = px - y * a.w;
                const int row = pl * bhw + (y + 1) * bw + x + 1;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int co = 32 * (m0 >> 1) + 8 * g + 4 * (m0 & 1) + r;
                    if (co >= cv.cout) continue;
                    const float v = acc[t][r] + (cv.bias ? cv.bias[co] : 0.f);
                    if (ci < 5) {
                        elem<T>::st(tile + row * lds_ld + cv.out_off + co, v > 0.f ? v : 0.1f * v);
                    } else {
                        float* fo = (float*)a.flow.ptr + map_frame(a.flow.map, pair0 + pl) * a.flow.img_stride +
                                    (long long)px * a.flow.ld + a.flow.c0 + co;
                        *fo = v;
                    }
                }
            }
        }
        __syncthreads();                // this conv's outputs are the next conv's input
    }
    DSTAMP(13);
    // dense channels back to global D (read by the next level's upfeat ConvT)
    const int d8 = a.dense_ch / 8;
    for (int i = threadIdx.x; i < np * d8; i += 512) {
        const int slot = i / d8, c = i - slot * d8;
        const int pl = slot / hw, px = slot - pl * hw, y = px / a.w, x = px - y * a.w;
        *(u32x4_t*)(img_ptr<T>(a.D, pair0 + pl) + (long long)px * a.D.ld + c * 8) =
            *(const u32x4_t*)(tile + (pl * bhw + (y + 1) * bw + x + 1) * lds_ld + c * 8);
    }
}


// ------------------------------------------------------------------------------------------------
// The same DenseNet specialised per coarse level of the 64x64 pyramid (levels 6..3: 1x1 .. 8x8 pixels per
// pair): every conv's geometry is a compile-time constant, so the k-loops unroll and the index math folds
// (the run-time kernel above spends most of its time in loop and address overhead), and each wave loads the
// first 16 A-fragments of its next conv right after the current conv's barrier so they arrive while it runs.
// ------------------------------------------------------------------------------------------------
__host__ __device__ constexpr int dcpad(int c) { return (c + 31) / 32 * 32; }
__host__ __device__ constexpr int dense_out(int i) { return i == 0 ? 128 : i == 1 ? 128 : i == 2 ? 96 : i == 3 ? 64 : 32; }
__host__ __device__ constexpr int dense_off(int i) { return i == 0 ? 320 : i == 1 ? 192 : i == 2 ? 96 : i == 3 ? 32 : 0; }

template <int LEVEL> struct DenseLevel {
    static constexpr int H = LEVEL == 6 ? 1 : LEVEL == 5 ? 2 : LEVEL == 4 ? 4 : 8;
    static constexpr int C = LEVEL == 6 ? 196 : LEVEL == 5 ? 128 : LEVEL == 4 ? 96 : 64;
    static constexpr int BASE = LEVEL == 6 ? 81 : 81 + C + 4;
    static constexpr int LD = 448 + dcpad(BASE), LDS_LD = LD + 8;
    static constexpr int HW = H * H, BW = H + 2, BHW = BW * BW;
    static constexpr int PPB = HW == 1 ? 8 : (16 / HW > 1 ? 16 / HW : 1);
    static constexpr int NT = (PPB * HW + 15) / 16;
    static constexpr bool SINGLE = HW == 1;
    static_assert(NT == 1 || NT == 4, "tile");
    static_assert(PPB * BHW * LDS_LD <= DenseTile<NT>::ELEMS, "LDS tile");
};
template <int LEVEL, int I> struct DenseConvSpec {
    using Lv = DenseLevel<LEVEL>;
    static constexpr int CIN = I == 5 ? Lv::BASE + 448 : Lv::BASE + (I > 0 ? 128 : 0) + (I > 1 ? 128 : 0) +
                                                           (I > 2 ? 96 : 0) + (I > 3 ? 64 : 0);
    static constexpr int START = I == 5 ? 0 : I == 0 ? 448 : dense_off(I - 1);
    static constexpr int COUT = I == 5 ? 2 : dense_out(I), OUT_OFF = I == 5 ? 0 : dense_off(I);
    static constexpr int GPT = dcpad(CIN) / 32;                 // k-steps (32-channel chunks) per tap
    static constexpr int NKS = Lv::SINGLE ? GPT : 9 * GPT;
    static constexpr int MB = (COUT + 15) / 16;
    static constexpr int KSPLIT = MB >= 5 ? 1 : MB >= 3 ? 2 : MB == 2 ? 4 : 8;
    static constexpr int KPW = (NKS + KSPLIT - 1) / KSPLIT;     // k-steps per wave (upper bound)
};

template <typename T, int NT> struct DenseCtx {
    T* tile;
    const DenseArgs* a;
    int lane, wave, g, col, np, pair0;
    int base[NT];
    bf16x8_t pa[2][16];
};

template <int LEVEL, int I, typename T, int NT>
__device__ __forceinline__ const T* dense_wrow(const DenseCtx<T, NT>& c) {
    using S = DenseConvSpec<LEVEL, I>;
    const int m0 = c.wave / S::KSPLIT;
    return (const T*)c.a->cv[I].w_pipe + (long long)(m0 < S::MB ? m0 : 0) * S::GPT * 9 * 512 + c.lane * 8;
}
// packed piece of this wave's k-step j (relative to its K slice) of conv I
template <int LEVEL, int I>
__device__ __forceinline__ int dense_piece(int kid, int j) {
    using S = DenseConvSpec<LEVEL, I>;
    int ks = kid * S::KPW + j;
    ks = ks < S::NKS ? ks : S::NKS - 1;
    return DenseLevel<LEVEL>::SINGLE ? ks * 9 + 4 : ks;
}
template <int LEVEL, int I, typename T, int NT>
__device__ __forceinline__ void dense_prefetch(DenseCtx<T, NT>& c) {
    if constexpr (I < 6) {
        using S = DenseConvSpec<LEVEL, I>;
        const T* w = dense_wrow<LEVEL, I>(c);
        const int kid = c.wave % S::KSPLIT;
#pragma unroll
        for (int j = 0; j < 16; ++j)
            c.pa[I % 2][j] = j < S::KPW ? *(const bf16x8_t*)(w + dense_piece<LEVEL, I>(kid, j) * 512)
                                       : bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
    }
}

template <int LEVEL, int I, typename T, int NT>
__device__ __forceinline__ void dense_conv(DenseCtx<T, NT>& c, f32x4_t* red) {
    using S = DenseConvSpec<LEVEL, I>;
    using Lv = DenseLevel<LEVEL>;
    __syncthreads();                                   // the previous conv's outputs are in the tile
    dense_prefetch<LEVEL, I + 1>(c);
    const int m0 = c.wave / S::KSPLIT, kid = c.wave % S::KSPLIT;
    const bool active = m0 < S::MB;
    f32x4_t acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    if (active) {
        const T* w = dense_wrow<LEVEL, I>(c);
        const int k_lo = kid * S::KPW;
        auto b_at = [&](int j, int t) {                // B-fragment of the wave's k-step j, column tile t
            int ks = k_lo + j;
            ks = ks < S::NKS ? ks : S::NKS - 1;
            const int ch = Lv::SINGLE ? ks : ks / 9, tap = Lv::SINGLE ? 4 : ks % 9;
            const int off = ((tap / 3) * Lv::BW + tap % 3) * Lv::LDS_LD + S::START + ch * 32;
            return *(const bf16x8_t*)(c.tile + c.base[t] + off);
        };
        const int nj = k_lo + S::KPW <= S::NKS ? S::KPW : S::NKS - k_lo;   // this wave's k-steps (wave-uniform)
        constexpr int KH = S::KPW < 16 ? S::KPW : 16;
#pragma unroll
        for (int j0 = 0; j0 < KH; j0 += 4) {
            bf16x8_t B[4][NT];
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int t = 0; t < NT; ++t) B[j][t] = b_at(j0 + j, t);
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (j0 + j < KH && j0 + j < nj) {
#pragma unroll
                    for (int t = 0; t < NT; ++t) acc[t] = mma16x16x32<T>(c.pa[I % 2][j0 + j], B[j][t], acc[t]);
                }
            __builtin_amdgcn_sched_barrier(0);
        }
        // the rest streams from global memory one batch of 4 ahead of its MFMAs
        if constexpr (S::KPW > 16) {
            bf16x8_t An[4];
#pragma unroll
            for (int j = 0; j < 4; ++j)
                An[j] = *(const bf16x8_t*)(w + dense_piece<LEVEL, I>(kid, 16 + j < S::KPW ? 16 + j : 16) * 512);
#pragma unroll
            for (int j0 = 16; j0 < S::KPW; j0 += 4) {
                bf16x8_t A[4], B[4][NT];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    A[j] = An[j];
                    const int jn = j0 + 4 + j < S::KPW ? j0 + 4 + j : j0;
                    if (j0 + 4 < S::KPW) An[j] = *(const bf16x8_t*)(w + dense_piece<LEVEL, I>(kid, jn) * 512);
#pragma unroll
                    for (int t = 0; t < NT; ++t) B[j][t] = b_at(j0 + j, t);
                }
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (j0 + j < S::KPW && j0 + j < nj) {
#pragma unroll
                        for (int t = 0; t < NT; ++t) acc[t] = mma16x16x32<T>(A[j], B[j][t], acc[t]);
                    }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        if constexpr (S::KSPLIT > 1) {
            if (kid > 0) {
#pragma unroll
                for (int t = 0; t < NT; ++t) red[(((kid - 1) * S::MB + m0) * NT + t) * 64 + c.lane] = acc[t];
            }
        }
    }
    if constexpr (S::KSPLIT > 1) __syncthreads();
    if (active && kid == 0) {
        if constexpr (S::KSPLIT > 1) {
#pragma unroll
            for (int k2 = 1; k2 < S::KSPLIT; ++k2)
#pragma unroll
                for (int t = 0; t < NT; ++t) acc[t] += red[(((k2 - 1) * S::MB + m0) * NT + t) * 64 + c.lane];
        }
        const DenseConv& cv = c.a->cv[I];
        // MFMA row 4g + r of block m0 is cout 32(m0 >> 1) + 8g + 4(m0 & 1) + r (pipe_cout_perm)
        const int co0 = 32 * (m0 >> 1) + 8 * c.g + 4 * (m0 & 1);
        float bias[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) bias[r] = (cv.bias && co0 + r < S::COUT) ? cv.bias[co0 + r] : 0.f;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const int slot = t * 16 + c.col;
            if (slot >= c.np) continue;
            const int pl = slot / Lv::HW, px = slot % Lv::HW, y = px / Lv::H, x = px % Lv::H;
            const int row = pl * Lv::BHW + (y + 1) * Lv::BW + x + 1;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                if (co0 + r >= S::COUT) continue;
                const float v = acc[t][r] + bias[r];
                if constexpr (I < 5) {
                    elem<T>::st(c.tile + row * Lv::LDS_LD + S::OUT_OFF + co0 + r, v > 0.f ? v : 0.1f * v);
                } else {
                    const DenseArgs& a = *c.a;
                    float* fo = (float*)a.flow.ptr + map_frame(a.flow.map, c.pair0 + pl) * a.flow.img_stride +
                                (long long)px * a.flow.ld + a.flow.c0 + co0 + r;
                    *fo = v;
                }
            }
        }
    }
}

template <typename T, int LEVEL>
__global__ __launch_bounds__(512) void pwc_dense_level_kernel(DenseArgs a) {
    using Lv = DenseLevel<LEVEL>;
    constexpr int NT = Lv::NT;
    __shared__ __attribute__((aligned(16))) u32x4_t smem[DenseTile<NT>::ELEMS / 8];
    __shared__ f32x4_t red[7 * NT * 64];
    DenseCtx<T, NT> c;
    c.tile = (T*)smem;
    c.a = &a;
    c.lane = threadIdx.x & 63;
    c.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    c.g = c.lane >> 4;
    c.col = c.lane & 15;
    c.pair0 = blockIdx.x * Lv::PPB;
    const int npairs = min(Lv::PPB, a.P - c.pair0);
    c.np = npairs * Lv::HW;
    constexpr int C8 = Lv::LD / 8, L8 = Lv::LDS_LD / 8;
    dense_prefetch<LEVEL, 0>(c);
    for (int i = threadIdx.x; i < npairs * Lv::BHW * L8; i += 512)
        *(u32x4_t*)(c.tile + i * 8) = u32x4_t{0u, 0u, 0u, 0u};
    __syncthreads();
    for (int i = threadIdx.x; i < c.np * C8; i += 512) {
        const int slot = i / C8, ch = i % C8;
        const int pl = slot / Lv::HW, px = slot % Lv::HW, y = px / Lv::H, x = px % Lv::H;
        *(u32x4_t*)(c.tile + (pl * Lv::BHW + (y + 1) * Lv::BW + x + 1) * Lv::LDS_LD + ch * 8) =
            *(const u32x4_t*)(img_ptr<T>(a.D, c.pair0 + pl) + (long long)px * a.D.ld + ch * 8);
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const int slot = t * 16 + c.col;
        const int pl = slot / Lv::HW, px = slot % Lv::HW, y = px / Lv::H, x = px % Lv::H;
        c.base[t] = (slot < c.np ? (pl * Lv::BHW + y * Lv::BW + x) * Lv::LDS_LD : 0) + c.g * 8;
    }
    dense_conv<LEVEL, 0>(c, red);
    dense_conv<LEVEL, 1>(c, red);
    dense_conv<LEVEL, 2>(c, red);
    dense_conv<LEVEL, 3>(c, red);
    dense_conv<LEVEL, 4>(c, red);
    dense_conv<LEVEL, 5>(c, red);
    __syncthreads();
    // dense channels back to global D (read by the next level's upfeat ConvT)
    const int d8 = a.dense_ch / 8;
    for (int i = threadIdx.x; i < c.np * d8; i += 512) {
        const int slot = i / d8, ch = i % d8;
        const int pl = slot / Lv::HW, px = slot % Lv::HW, y = px / Lv::H, x = px % Lv::H;
        *(u32x4_t*)(img_ptr<T>(a.D, c.pair0 + pl) + (long long)px * a.D.ld + ch * 8) =
            *(const u32x4_t*)(c.tile + (pl * Lv::BHW + (y + 1) * Lv::BW + x + 1) * Lv::LDS_LD + ch * 8);
    }
}

// the specialised level (6..3) for an h x h level with ld channels in D, 0 if none
int dense_level_of(int h, int w, int ld) {
    if (h != w) return 0;
    if (h == DenseLevel<6>::H && ld == DenseLevel<6>::LD) return 6;
    if (h == DenseLevel<5>::H && ld == DenseLevel<5>::LD) return 5;
    if (h == DenseLevel<4>::H && ld == DenseLevel<4>::LD) return 4;
    if (h == DenseLevel<3>::H && ld == DenseLevel<3>::LD) return 3;
    return 0;
}
}  // namespace

#ifdef DBSR_PIPE_STAMPS
extern "C" int dbsr_diag_dense_stamps(unsigned long long* host, long long n) {
    if (!host) {
        static unsigned long long z[128 * 8 * 16];
        return hipMemcpyToSymbol(HIP_SYMBOL(g_dense_stamps), z, sizeof(z)) == hipSuccess ? 0 : -1;
    }
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_dense_stamps), n * 8) == hipSuccess ? 0 : -1;
}
#endif

namespace {
int dense_ppb(int h, int w) { return h * w == 1 ? 8 : std::max(1, 16 / (h * w)); }
bool dense_fits(int h, int w, int ld) {
    if (h <= 0 || w <= 0 || h * w > 64) return false;
    const int ppb = dense_ppb(h, w), nt = (ppb * h * w + 15) / 16;
    if (nt != 1 && nt != 4) return false;
    return (long long)ppb * (h + 2) * (w + 2) * (ld + 8) <= (nt == 1 ? DenseTile<1>::ELEMS : DenseTile<4>::ELEMS);
}
}  // namespace

extern "C" int dbsr_pwc_dense_supported(int h, int w, int ld) { return dense_fits(h, w, ld) ? 1 : 0; }

extern "C" int dbsr_pwc_dense(int P, int h, int w, dbsr_tensor D, int dense_ch, const dbsr_pwc_dense_conv* convs,
                              dbsr_tensor flow, void* stream) {
    DBSR_CHECK_ARG(D.ptr && D.map.fpg > 0 && flow.ptr && flow.map.fpg > 0 && convs, "pwc_dense: null tensor");
    DBSR_CHECK_ARG(D.dtype == DBSR_BF16 || D.dtype == DBSR_F16, "pwc_dense: D must be bf16 or fp16");
    DBSR_CHECK_ARG(flow.dtype == DBSR_F32 && flow.c0 + 2 <= flow.ld, "pwc_dense: flow must be fp32 with >= 2 channels");
    DBSR_CHECK_ARG(P > 0 && h > 0 && w > 0 && h * w <= 64, "pwc_dense: needs 1..64 pixels per pair (got %dx%d)", h, w);
    DBSR_CHECK_ARG(D.ld % 8 == 0 && D.c0 == 0 && dense_ch % 8 == 0 && dense_ch <= D.ld, "pwc_dense: D layout");
    DenseArgs a;
    a.P = P; a.h = h; a.w = w; a.ld = D.ld; a.D = D; a.flow = flow; a.dense_ch = dense_ch;
    for (int i = 0; i < 6; ++i) {
        const dbsr_pwc_dense_conv& c = convs[i];
        DBSR_CHECK_ARG(c.w && c.cg > 0 && c.cg % 4 == 0 && c.kp == 9 * c.cg * 8 && c.cout > 0,
                       "pwc_dense: conv %d: packed weights must be 3x3 with cin padded to 32", i);
        DBSR_CHECK_ARG(c.start % 8 == 0 && c.start + c.cg * 8 <= D.ld, "pwc_dense: conv %d input slice exceeds ld", i);
        DBSR_CHECK_ARG(i == 5 ? c.cout <= 2 : (c.out_off % 8 == 0 && c.out_off + c.cout <= c.start),
                       "pwc_dense: conv %d output must lie below its input slice", i);
        // the chunk-major copy follows the round_up(cout, 64) x kp row-major weights (dbsr_conv_packed_elems)
        const void* wp = (const char*)c.w + (size_t)((c.cout + 63) / 64 * 64) * c.kp * 2;
        a.cv[i] = DenseConv{wp, c.bias, c.kp, c.cg, c.start, c.cout, c.out_off};
    }
    const int hw = h * w;
    hipStream_t s = (hipStream_t)stream;
    if (const int lvl = dense_level_of(h, w, D.ld)) {
        // the conv list must be the level's DenseNet (pwcnet.py:123-150) for the specialised kernel
        bool std_convs = true;
        const int base = lvl == 6 ? 81 : 81 + (lvl == 5 ? 128 : lvl == 4 ? 96 : 64) + 4;
        int cin = base;
        for (int i = 0; i < 6; ++i) {
            const int start = i == 5 ? 0 : i == 0 ? 448 : dense_off(i - 1);
            const int cout = i == 5 ? 2 : dense_out(i);
            std_convs = std_convs && convs[i].cg * 8 == dcpad(i == 5 ? base + 448 : cin) && convs[i].start == start &&
                        convs[i].cout == cout && (i == 5 || convs[i].out_off == dense_off(i));
            if (i < 5) cin += cout;
        }
        if (std_convs && dense_ch == 448) {
            const int ppb = lvl == 6 ? 8 : lvl == 5 ? 4 : 1;
            a.ppb = ppb;
            const unsigned grid = (unsigned)((P + ppb - 1) / ppb);
#define DBSR_DENSE_LVL(L)                                                                                 \
    if (lvl == L) {                                                                                      \
        if (D.dtype == DBSR_BF16)                                                                        \
            hipLaunchKernelGGL((pwc_dense_level_kernel<bf16_t, L>), dim3(grid), dim3(512), 0, s, a);     \
        else                                                                                             \
            hipLaunchKernelGGL((pwc_dense_level_kernel<f16_t, L>), dim3(grid), dim3(512), 0, s, a);      \
    }
            DBSR_DENSE_LVL(6) DBSR_DENSE_LVL(5) DBSR_DENSE_LVL(4) DBSR_DENSE_LVL(3)
#undef DBSR_DENSE_LVL
            DBSR_LAUNCH_CHECK();
            return 0;
        }
    }
    DBSR_CHECK_ARG(dense_fits(h, w, D.ld), "pwc_dense: no LDS tile for %dx%d pixels x %d channels "
                   "(dbsr_pwc_dense_supported)", h, w, D.ld);
    a.ppb = dense_ppb(h, w);             // one 16-slot column tile of pairs, or one pair of 64 pixels
    const int nt = (a.ppb * hw + 15) / 16;
    const unsigned grid = (unsigned)((P + a.ppb - 1) / a.ppb);
#define DBSR_DENSE(T, NT) \
    hipLaunchKernelGGL((pwc_dense_kernel<T, NT>), dim3(grid), dim3(512), 0, s, a)
    if (D.dtype == DBSR_BF16) {
        if (nt == 1) DBSR_DENSE(bf16_t, 1); else DBSR_DENSE(bf16_t, 4);
    } else {
        if (nt == 1) DBSR_DENSE(f16_t, 1); else DBSR_DENSE(f16_t, 4);
    }
#undef DBSR_DENSE
    DBSR_LAUNCH_CHECK();
    return 0;
}
