// PWC-Net feature pyramid in one launch (models/alignment/pwcnet.py:45-111, Extractor.forward :103-111):
// six levels of (3x3 stride-2 conv, 3x3 conv, 3x3 conv), each followed by LeakyReLU(0.1), on a 64x64 frame
// (the 48x48 bench bursts resized to a multiple of 64, pwcnet.py:262-271).
//
// Layer by layer this was 18 launches (+ 9 split-K finalizes), ~150 us of event time and ~300 us of the
// side lane's timeline for ~5 GFLOP: every level after the first is a few hundred pixels per frame.  Here
// one 8-wave block owns one frame for the whole pyramid.  Activations never leave the LDS except the six
// level outputs (read by the decoders): the input frame sits in a 66x66 zero-bordered image, each conv's
// output goes to one of two ping-pong images with a one-pixel zero border, so a 3x3 tap of any output
// pixel -- stride 1 or 2 -- is one unconditional LDS read.  Per conv the work is (16-cout M tile, 16-pixel
// N tile) items over the 8 waves; A-fragments (the generic kernel's packed weight rows, read by every block
// and so L2-resident) come from global memory, B-fragments from the LDS image, and each item's k-steps run
// in batches of 8 (all loads first, then the MFMA chain).  Taps that never see an in-frame pixel (the 1x1
// and 2x2 coarse levels) are skipped.  The epilogue (bias, LeakyReLU) writes the pixel's 4 channels to the
// next LDS image -- couts are computed up to the padded width, so the pad channels the next conv reads are
// exact zeros -- and, for a level's last conv, to the level output in global memory.
#include "common.hpp"

#include <algorithm>
#include <type_traits>
#include <utility>

using namespace dbsr;

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bfv8_t;
typedef __attribute__((ext_vector_type(8))) _Float16 hv8_t;

template <typename T>
__device__ __forceinline__ f32x4_t mfma16(bf16x8_t a, bf16x8_t b, f32x4_t c) {
    if constexpr (std::is_same<T, bf16_t>::value)
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bfv8_t, a), __builtin_bit_cast(bfv8_t, b), c,
                                                       0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(hv8_t, a), __builtin_bit_cast(hv8_t, b), c,
                                                      0, 0, 0);
}

inline int cpad_i(int c) { return c <= 16 ? (c + 7) / 8 * 8 : (c + 31) / 32 * 32; }

constexpr int EXT_CONVS = 18;
constexpr int EXT_R0 = 66 * 66 * 8;                 // input frame, bordered, 8 channels
constexpr int EXT_R1 = 34 * 34 * 16;                // level-1 images, bordered, 16 channels
constexpr int EXT_ELEMS = EXT_R0 + 2 * EXT_R1;      // 143.7 KiB of 16-bit elements

__host__ __device__ constexpr int ext_ch(int l) {   // channels of pyramid level l (0 = the RGB input), pwcnet.py:49-100
    return l == 0 ? 3 : l == 1 ? 16 : l == 2 ? 32 : l == 3 ? 64 : l == 4 ? 96 : l == 5 ? 128 : 196;
}
__host__ __device__ constexpr int cpad_c(int c) { return c <= 16 ? (c + 7) / 8 * 8 : (c + 31) / 32 * 32; }
__host__ __device__ constexpr int ldsld_c(int c) { return cpad_c(c) <= 16 ? cpad_c(c) : cpad_c(c) + 8; }
// does tap offset k (0..2) of a stride-s, pad-1 conv see an in-frame input pixel for some output pixel?
__host__ __device__ constexpr bool tap_live(int k, int s, int ih, int oh) {
    bool ok = false;
    for (int o = 0; o < oh; ++o) ok = ok || (o * s - 1 + k >= 0 && o * s - 1 + k < ih);
    return ok;
}
__host__ __device__ constexpr int tap_lo(int s, int ih, int oh) {
    int lo = 9;
    for (int t = 8; t >= 0; --t)
        if (tap_live(t / 3, s, ih, oh) && tap_live(t % 3, s, ih, oh)) lo = t;
    return lo;
}
__host__ __device__ constexpr int tap_hi(int s, int ih, int oh) {
    int hi = -1;
    for (int t = 0; t < 9; ++t)
        if (tap_live(t / 3, s, ih, oh) && tap_live(t % 3, s, ih, oh)) hi = t;
    return hi;
}

// Compile-time geometry of conv I of the pyramid (level I / 3, conv I % 3)
template <int I> struct ExtSpec {
    static constexpr int L = I / 3, J = I % 3;
    static constexpr int CIN = J == 0 ? ext_ch(L) : ext_ch(L + 1), COUT = ext_ch(L + 1), S = J == 0 ? 2 : 1;
    static constexpr int IH = J == 0 ? (64 >> L) : (64 >> (L + 1)), OH = 64 >> (L + 1);
    static constexpr int IBW = IH + 2, OBW = OH + 2;
    static constexpr int ILD = I == 0 ? 8 : ldsld_c(CIN), OLD = ldsld_c(COUT);
    static constexpr int IN_BUF = I == 0 ? 0 : ((I - 1) % 2 == 0 ? 1 : 2), OUT_BUF = I % 2 == 0 ? 1 : 2;
    static constexpr int CG = cpad_c(CIN) / 8;
    static constexpr int KP = (9 * CG + 3) / 4 * 4 * 8;                  // packed row length
    static constexpr bool PIPE = CIN > 16;                                // chunk-major copy (1-KiB pieces)
    static constexpr int NCH = cpad_c(CIN) / 32;
    static constexpr int TLO = tap_lo(S, IH, OH), THI = tap_hi(S, IH, OH), NTAP = THI - TLO + 1;
    static constexpr int KS_LO = PIPE ? 0 : (TLO * CG) / 4;
    static constexpr int NKS = PIPE ? NCH * NTAP : ((THI + 1) * CG + 3) / 4 - KS_LO;
    static constexpr int MT = cpad_c(COUT) / 16, NPIX = OH * OH, NT = (NPIX + 15) / 16;
    static constexpr int P = COUT <= 32 ? 32 : 64;                        // pipe_cout_perm tile
    static constexpr bool FIXED_M = 8 % MT == 0;
    static constexpr int WPIPE = (COUT + 63) / 64 * 64 * KP;              // offset of the chunk-major copy
    static_assert(NTAP >= 1 && NKS >= 1, "no live tap");
    static_assert((OH + 2) * (OH + 2) * OLD <= EXT_R1, "output image exceeds its LDS buffer");
};

struct ExtArgs {
    int F;
    dbsr_tensor rgb;                   // [F][64][64][8]
    dbsr_tensor lv[6];                 // level outputs [F][64 >> (l+1)]^2 [cpad(C_l)]
    const void* w[EXT_CONVS];          // packed weights (row layout, then the chunk-major copy for cin > 16)
    const float* bias[EXT_CONVS];
};

// Diagnostic build only (make exp EXP_FLAGS=-DDBSR_EXT_STAMPS): s_memtime per wave after every conv's barrier
// and after its compute, read back by dbsr_diag_ext_stamps (tools/ext_stamps.py).
#ifdef DBSR_EXT_STAMPS
__device__ unsigned long long g_ext_stamps[128 * 8 * 40];
#define EXT_STAMP(slot) do { if (c.lane == 0 && blockIdx.x < 128) g_ext_stamps[(blockIdx.x * 8 + c.wave) * 40 + (slot)] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define EXT_STAMP(slot) do { } while (0)
#endif

template <typename T> struct ExtCtx {
    const ExtArgs* a;
    T* base;
    int f, lane, wave, kgl, col;
    bf16x8_t pa[2][16];                // A-fragment sets: conv I computes from set I % 2, prefetches set (I+1) % 2
    float pb[2][4];
    __device__ T* img(int b) const { return base + (b == 0 ? 0 : b == 1 ? EXT_R0 : EXT_R0 + EXT_R1); }
};

// A-fragment of k-step ks of M tile m (lane layout of mfma 16x16x32: row col, k-group kgl)
template <int I, typename T>
__device__ __forceinline__ bf16x8_t ext_a(const ExtCtx<T>& c, int m, int ks) {
    using S = ExtSpec<I>;
    const T* w = (const T*)c.a->w[I];
    if constexpr (S::PIPE) {
        const int ch = ks / S::NTAP, tap = S::TLO + ks % S::NTAP;
        return *(const bf16x8_t*)(w + S::WPIPE + ((m * S::NCH + ch) * 9 + tap) * 512 + c.lane * 8);
    } else {
        return *(const bf16x8_t*)(w + (m * 16 + c.col) * S::KP + (S::KS_LO + ks) * 32 + c.kgl * 8);
    }
}
// physical cout of accumulator row 4*kgl + r of M tile m
template <int I, typename T>
__device__ __forceinline__ int ext_co(const ExtCtx<T>& c, int m) {
    using S = ExtSpec<I>;
    if constexpr (S::PIPE) {
        constexpr int BPT = S::P / 16;
        const int i = m % BPT;
        return (m / BPT) * S::P + 32 * (i >> 1) + 8 * c.kgl + 4 * (i & 1);
    } else {
        return m * 16 + 4 * c.kgl;
    }
}
template <int I, typename T>
__device__ __forceinline__ void ext_bias(const ExtCtx<T>& c, int m, float (&b)[4]) {
    using S = ExtSpec<I>;
    const int co = ext_co<I>(c, m);
    const float* bias = c.a->bias[I];
#pragma unroll
    for (int r = 0; r < 4; ++r) b[r] = co + r < S::COUT ? bias[co + r] : 0.f;
}
// LDS offset of k-step ks's B-fragment from a pixel's window origin; live = the k-group is a real one
template <int I, typename T>
__device__ __forceinline__ int ext_boff(const ExtCtx<T>& c, int ks, bool& live) {
    using S = ExtSpec<I>;
    if constexpr (S::PIPE) {
        const int ch = ks / S::NTAP, tap = S::TLO + ks % S::NTAP;
        live = true;
        return ((tap / 3) * S::IBW + tap % 3) * S::ILD + ch * 32 + c.kgl * 8;
    } else {
        const int kg = (S::KS_LO + ks) * 4 + c.kgl;
        const int tap = kg / S::CG, cg = kg - tap * S::CG;
        live = kg < 9 * S::CG;
        return ((tap / 3) * S::IBW + tap % 3) * S::ILD + cg * 8;
    }
}

template <int I, typename T>
__device__ __forceinline__ void ext_prefetch(ExtCtx<T>& c) {
    if constexpr (I < EXT_CONVS) {
        using S = ExtSpec<I>;
        const int m = c.wave % S::MT;
#pragma unroll
        for (int j = 0; j < 16; ++j)
            c.pa[I % 2][j] = j < S::NKS ? ext_a<I>(c, m, j) : bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
        ext_bias<I>(c, m, c.pb[I % 2]);
    }
}

// One conv: barrier, prefetch of the next conv's fragments, border zeroing, the wave's items, epilogues.
template <int I, typename T>
__device__ __forceinline__ void ext_conv(ExtCtx<T>& c) {
    using S = ExtSpec<I>;
    const bf16x8_t zero8 = bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
    __syncthreads();                      // the previous conv's output is complete; its input is consumed
    EXT_STAMP(1 + 2 * I);
    ext_prefetch<I + 1>(c);
    const T* in = c.img(S::IN_BUF);
    T* out = c.img(S::OUT_BUF);
    {   // the output image's border, all channel slots: the buffer held another geometry before
        constexpr int S8 = S::OLD / 8, NB = 2 * S::OBW + 2 * S::OH;
        for (int i = threadIdx.x; i < NB * S8; i += 512) {
            const int bp = i / S8, ch = i - bp * S8;
            int y, x;
            if (bp < S::OBW) { y = 0; x = bp; }
            else if (bp < 2 * S::OBW) { y = S::OBW - 1; x = bp - S::OBW; }
            else { const int r = bp - 2 * S::OBW; y = 1 + (r >> 1); x = (r & 1) ? S::OBW - 1 : 0; }
            *(u32x4_t*)(out + (y * S::OBW + x) * S::OLD + ch * 8) = u32x4_t{0u, 0u, 0u, 0u};
        }
    }
    auto origin = [&](int n) {            // window origin of this lane's pixel in N tile n (pad slots: pixel 0)
        const int p = n * 16 + c.col;
        const int oy = p < S::NPIX ? p / S::OH : 0, ox = p < S::NPIX ? p % S::OH : 0;
        return in + ((oy * S::S) * S::IBW + ox * S::S) * S::ILD;
    };
    auto store = [&](const f32x4_t& acc, const float (&bias)[4], int m, int n) {
        const int p = n * 16 + c.col;
        if (p >= S::NPIX) return;
        const int oy = p / S::OH, ox = p % S::OH;
        const int co = ext_co<I>(c, m);
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float t = acc[r] + bias[r];
            v[r] = t > 0.f ? t : 0.1f * t;
        }
        uint2 q;
        q.x = H16<T>::pack(v[0], v[1]);
        q.y = H16<T>::pack(v[2], v[3]);
        *(uint2*)(out + ((oy + 1) * S::OBW + ox + 1) * S::OLD + co) = q;
        if constexpr (S::J == 2) {
            const dbsr_tensor& L = c.a->lv[S::L];
            *(uint2*)(img_ptr<T>(L, c.f) + (long long)p * L.ld + co) = q;
        }
    };
    // k-steps [k0, k1) with fragments from registers (A) or streamed from global memory (A == nullptr):
    // batches of 4 (B reads, then MFMAs), one or two pixel tiles
    auto mma = [&](const bf16x8_t* A, int m, int k0, int k1, const T* b1, const T* b2, f32x4_t& acc1,
                   f32x4_t& acc2, bool two) {
#pragma unroll
        for (int j0 = k0; j0 < k1; j0 += 4) {
            bf16x8_t Aq[4], B1[4], B2[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int ks = j0 + j < k1 ? j0 + j : k0;
                Aq[j] = A ? A[ks] : ext_a<I>(c, m, ks);
                bool live;
                const int off = ext_boff<I>(c, ks, live);
                B1[j] = live ? *(const bf16x8_t*)(b1 + off) : zero8;
                B2[j] = (live && two) ? *(const bf16x8_t*)(b2 + off) : zero8;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (j0 + j < k1) {
                    acc1 = mfma16<T>(Aq[j], B1[j], acc1);
                    if (two) acc2 = mfma16<T>(Aq[j], B2[j], acc2);
                }
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    constexpr int KH = S::NKS < 16 ? S::NKS : 16;        // k-steps held in the prefetched set
    const bf16x8_t* A0 = c.pa[I % 2];
    if constexpr (S::FIXED_M) {
        // every item of this wave has M tile wave % MT; it walks its N tiles two at a time
        constexpr int NSTEP = 8 / S::MT;
        const int m = c.wave % S::MT;
        for (int n = c.wave / S::MT; n < S::NT; n += 2 * NSTEP) {
            const int n2 = n + NSTEP;
            const bool two = n2 < S::NT;
            const T* b1 = origin(n);
            const T* b2 = origin(two ? n2 : n);
            f32x4_t acc1 = f32x4_t{0.f, 0.f, 0.f, 0.f}, acc2 = acc1;
            mma(A0, m, 0, KH, b1, b2, acc1, acc2, two);
            if constexpr (S::NKS > 16) mma(nullptr, m, 16, S::NKS, b1, b2, acc1, acc2, two);
            store(acc1, c.pb[I % 2], m, n);
            if (two) store(acc2, c.pb[I % 2], m, n2);
        }
    } else {
        // one N tile (the 4x4 and 1x1 levels): M tiles wave and wave + 8
        static_assert(S::NT == 1 && S::MT <= 16, "general path: one pixel tile, <= 16 M tiles");
        const T* b1 = origin(0);
        if (c.wave < S::MT) {
            f32x4_t acc1 = f32x4_t{0.f, 0.f, 0.f, 0.f}, acc2 = acc1;
            mma(A0, c.wave, 0, KH, b1, b1, acc1, acc2, false);
            if constexpr (S::NKS > 16) mma(nullptr, c.wave, 16, S::NKS, b1, b1, acc1, acc2, false);
            store(acc1, c.pb[I % 2], c.wave, 0);
        }
        if (c.wave + 8 < S::MT) {
            float bb[4];
            ext_bias<I>(c, c.wave + 8, bb);
            f32x4_t acc1 = f32x4_t{0.f, 0.f, 0.f, 0.f}, acc2 = acc1;
            mma(nullptr, c.wave + 8, 0, S::NKS, b1, b1, acc1, acc2, false);
            store(acc1, bb, c.wave + 8, 0);
        }
    }
    EXT_STAMP(2 + 2 * I);
}

template <typename T, int... Is>
__device__ __forceinline__ void ext_all(ExtCtx<T>& c, std::integer_sequence<int, Is...>) {
    (ext_conv<Is>(c), ...);
}

template <typename T>
__global__ __launch_bounds__(512) void pwc_extract_kernel(ExtArgs a) {
    __shared__ __attribute__((aligned(16))) u32x4_t smem[EXT_ELEMS / 8];
    ExtCtx<T> c;
    c.a = &a;
    c.base = (T*)smem;
    c.f = blockIdx.x;
    c.lane = threadIdx.x & 63;
    c.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    c.kgl = c.lane >> 4;
    c.col = c.lane & 15;
    EXT_STAMP(0);
    ext_prefetch<0>(c);
    {   // the frame into image 0 (66x66, zero border)
        const T* src = img_ptr<T>(a.rgb, c.f);
        for (int i = threadIdx.x; i < 66 * 66; i += 512) {
            const int y = i / 66 - 1, x = i - (i / 66) * 66 - 1;
            u32x4_t v = u32x4_t{0u, 0u, 0u, 0u};
            if ((unsigned)y < 64u && (unsigned)x < 64u) v = *(const u32x4_t*)(src + (y * 64 + x) * a.rgb.ld);
            *(u32x4_t*)(c.base + i * 8) = v;
        }
    }
    ext_all<T>(c, std::make_integer_sequence<int, EXT_CONVS>{});
    EXT_STAMP(39);
}

}  // namespace

#ifdef DBSR_EXT_STAMPS
extern "C" int dbsr_diag_ext_stamps(unsigned long long* host, long long n) {
    if (!host) {
        static unsigned long long z[128 * 8 * 40];
        return hipMemcpyToSymbol(HIP_SYMBOL(g_ext_stamps), z, sizeof(z)) == hipSuccess ? 0 : -1;
    }
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ext_stamps), n * 8) == hipSuccess ? 0 : -1;
}
#endif

extern "C" int dbsr_pwc_extract_supported(int Hp, int Wp) { return Hp == 64 && Wp == 64 ? 1 : 0; }

extern "C" int dbsr_pwc_extract(int F, int Hp, int Wp, dbsr_tensor rgb, const dbsr_pwc_ext_conv* convs,
                                const dbsr_tensor* levels, void* stream) {
    DBSR_CHECK_ARG(convs && levels && rgb.ptr && rgb.map.fpg > 0, "pwc_extract: null argument");
    DBSR_CHECK_ARG(dbsr_pwc_extract_supported(Hp, Wp), "pwc_extract: needs a 64x64 frame (got %dx%d)", Hp, Wp);
    DBSR_CHECK_ARG(rgb.dtype == DBSR_BF16 || rgb.dtype == DBSR_F16, "pwc_extract: 16-bit activations only");
    DBSR_CHECK_ARG(rgb.ld == 8 && rgb.c0 == 0, "pwc_extract: rgb must be the 8-channel packed frame");
    DBSR_CHECK_ARG(F > 0, "pwc_extract: no frames");
    ExtArgs a;
    a.F = F;
    a.rgb = rgb;
    for (int l = 0; l < 6; ++l) {
        const dbsr_tensor& L = levels[l];
        const int C = ext_ch(l + 1);
        DBSR_CHECK_ARG(L.ptr && L.dtype == rgb.dtype && L.map.fpg > 0 && L.c0 == 0 && L.ld == cpad_c(C),
                       "pwc_extract: level %d output must be a %d-channel slice of ld %d", l + 1, C, cpad_c(C));
        a.lv[l] = L;
        for (int j = 0; j < 3; ++j) {
            const int i = 3 * l + j;
            const dbsr_pwc_ext_conv& cv = convs[i];
            const int cin = j == 0 ? ext_ch(l) : C, s = j == 0 ? 2 : 1;
            DBSR_CHECK_ARG(cv.w && cv.bias && cv.cin == cin && cv.cout == C && cv.stride == s,
                           "pwc_extract: conv %d must be %d -> %d, stride %d, with a bias", i, cin, C, s);
            a.w[i] = cv.w;
            a.bias[i] = cv.bias;
        }
    }
    hipStream_t s = (hipStream_t)stream;
    if (rgb.dtype == DBSR_BF16)
        hipLaunchKernelGGL(pwc_extract_kernel<bf16_t>, dim3(F), dim3(512), 0, s, a);
    else
        hipLaunchKernelGGL(pwc_extract_kernel<f16_t>, dim3(F), dim3(512), 0, s, a);
    DBSR_LAUNCH_CHECK();
    return 0;
}

// ------------------------------------------------------------------------------------------------
// PWC-Net decoder level input in one launch (Decoder.forward, pwcnet.py:153-171): for each pair
//   upflow = ConvT(prev flow), upfeat = ConvT(prev dense features)            (:162-167, k4 s2 p1)
//   warped = backwarp(second, upflow * fltBackwarp)                           (:169, pwcnet.py:16-38)
//   D[:, c0 + 0..80] = LeakyReLU(correlation(first, warped))                  (:161,169, K2)
//   D[:, c0 + 81..]  = [first | upflow | upfeat]                              (:171)
// (the coarsest level: no previous level, the correlation of the unwarped features only).  These were five
// launches per level (ConvT x2, backwarp, assembly, correlation: 20-70 us per level, mostly launch gaps);
// here one block per pair keeps the level's upsampled flow, its first features and its warped second
// features (with the correlation's 4-pixel zero border) in the LDS.  The arithmetic of each step is the
// stand-alone kernel's (same formulas and channel order; the ConvT sums its input channels in lane slices
// reduced by shuffles, like convt_k4s2_kernel).
// ------------------------------------------------------------------------------------------------
namespace {

constexpr int PREP_LDS_BYTES = 64 * 1024;

struct PrepArgs {
    int P, h, w, C, Cp;           // pairs, level size, channels and their padded stride (feature tensors)
    float scale;                  // fltBackwarp of this level
    dbsr_tensor first, second;    // level features, pair -> frame maps
    dbsr_tensor D;                // decoder buffer; c0 = the base channels (BASE_OFF)
    int has_prev, pcin32;         // previous level present; its dense-buffer channels read (multiple of 32)
    dbsr_tensor pD, pflow;        // previous level's D [P][h/2][w/2] and flow (fp32, 2 of >= 8 channels)
    const float* wflow; const float* bflow;   // upflow ConvT: fp32 [4][4][2][8], bias [2]
    const void* wfeat; const float* bfeat;    // upfeat ConvT: 16-bit rows [(ky*4+kx)*2 + co][pcin32], bias [2]
};

template <typename T>
__device__ __forceinline__ void convt_px(const PrepArgs& a, const dbsr_tensor& in, int pair, int cin8,
                                         const float* __restrict__ wgt, int oy, int ox, int sl, int SG, float (&acc)[2]) {
    const int h = a.h / 2, w = a.w / 2;
    acc[0] = acc[1] = 0.f;
    const T* base = img_ptr<T>(in, pair);
    const int ky0 = (oy + 1) & 1, kx0 = (ox + 1) & 1;
    const int ngroups = cin8 / 8;
    for (int aa = 0; aa < 2; ++aa) {
        const int ky = ky0 + 2 * aa, iy = (oy + 1 - ky) >> 1;
        if (iy < 0 || iy >= h) continue;
        for (int bq = 0; bq < 2; ++bq) {
            const int kx = kx0 + 2 * bq, ix = (ox + 1 - kx) >> 1;
            if (ix < 0 || ix >= w) continue;
            const T* src = base + ((long long)iy * w + ix) * in.ld;
            const float* wt = wgt + (long long)((ky * 4 + kx) * 2) * cin8;
            for (int cgi = sl; cgi < ngroups; cgi += SG) {
                float v[8], w0[8], w1[8];
                load8(src + cgi * 8, v);
                load8(wt + cgi * 8, w0);
                load8(wt + cin8 + cgi * 8, w1);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    acc[0] = fmaf(v[j], w0[j], acc[0]);
                    acc[1] = fmaf(v[j], w1[j], acc[1]);
                }
            }
        }
    }
}

// Specialised per level (H x H pixels, C channels; PREV: a previous level exists) so every loop bound and
// index is a compile-time constant.
template <typename T, int H, int C, bool PREV, int NT>
__global__ __launch_bounds__(NT) void pwc_level_prep_kernel(PrepArgs a) {
    constexpr int NWV = NT / 64;                       // waves per block
    constexpr int W = H, NPIX = H * W, CP = cpad_c(C), C8 = CP / 8, BW = W + 8, BH = H + 8;
    __shared__ __attribute__((aligned(16))) unsigned char smem[PREP_LDS_BYTES];
    static_assert(NPIX * 16 + NPIX * CP * 2 + BH * BW * CP * 2 <= PREP_LDS_BYTES, "level tile exceeds the LDS");
    const int pair = blockIdx.x;
    float* up = (float*)smem;                          // [NPIX][4]: upflow x, y, upfeat 0, 1
    T* fst = (T*)(smem + NPIX * 16);                   // [NPIX][CP]
    T* wrp = fst + NPIX * CP;                          // [(H+8) x (W+8)][CP], 4-pixel zero border
    const int t = threadIdx.x;
    const int lane = t & 63, wave = t >> 6, kgl = lane >> 4, col = lane & 15;

    // ---- upflow / upfeat (ConvTranspose2d k4 s2 p1) of the previous level ----
    // upfeat: every (tap, cout) contribution of every previous-level pixel as one small GEMM on MFMA,
    // part[in_px][(ky*4+kx)*2+co] = sum_ci D_prev[in_px][ci] * w[ky][kx][co][ci] (M = 32 rows, N = the previous
    // level's pixels, K = its channels), then each output pixel sums its <= 4 (input pixel, tap) terms.  The
    // 2-channel upflow keeps the scalar form (convt_k4s2_kernel's arithmetic).
    if constexpr (PREV) {
        constexpr int PW = W / 2, PNP = NPIX / 4, NTN = (PNP + 15) / 16;
        float* part = (float*)(smem + NPIX * 16);     // [PNP][32] (before the first-feature image exists)
        const int nks = a.pcin32 / 32;
        const T* pd = img_ptr<T>(a.pD, pair);
        for (int item = wave; item < 2 * NTN; item += NWV) {
            const int mt = item & 1, nt = item >> 1;
            const int q = nt * 16 + col;
            const T* brow = pd + (long long)(q < PNP ? q : 0) * a.pD.ld + kgl * 8;
            const T* arow = (const T*)a.wfeat + (long long)(mt * 16 + col) * a.pcin32 + kgl * 8;
            f32x4_t acc = f32x4_t{0.f, 0.f, 0.f, 0.f};
            for (int k0 = 0; k0 < nks; k0 += 8) {
                bf16x8_t A[8], B[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int ks = k0 + j < nks ? k0 + j : nks - 1;
                    A[j] = *(const bf16x8_t*)(arow + ks * 32);
                    B[j] = *(const bf16x8_t*)(brow + ks * 32);
                }
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    if (k0 + j < nks) acc = mfma16<T>(A[j], B[j], acc);
            }
            if (q < PNP) {
#pragma unroll
                for (int r = 0; r < 4; ++r) part[q * 32 + mt * 16 + 4 * kgl + r] = acc[r];
            }
        }
        __syncthreads();
        for (int q = t; q < NPIX; q += NT) {
            const int oy = q / W, ox = q % W;
            float af[2];
            convt_px<float>(a, a.pflow, pair, 8, a.wflow, oy, ox, 0, 1, af);
            float ad0 = 0.f, ad1 = 0.f;
            const int ky0 = (oy + 1) & 1, kx0 = (ox + 1) & 1;
#pragma unroll
            for (int aa = 0; aa < 2; ++aa) {
                const int ky = ky0 + 2 * aa, iy = (oy + 1 - ky) >> 1;
                if (iy < 0 || iy >= H / 2) continue;
#pragma unroll
                for (int bq = 0; bq < 2; ++bq) {
                    const int kx = kx0 + 2 * bq, ix = (ox + 1 - kx) >> 1;
                    if (ix < 0 || ix >= PW) continue;
                    const float* pp = part + (iy * PW + ix) * 32 + (ky * 4 + kx) * 2;
                    ad0 += pp[0];
                    ad1 += pp[1];
                }
            }
            up[q * 4 + 0] = af[0] + a.bflow[0];
            up[q * 4 + 1] = af[1] + a.bflow[1];
            up[q * 4 + 2] = ad0 + a.bfeat[0];
            up[q * 4 + 3] = ad1 + a.bfeat[1];
        }
        __syncthreads();                               // part[] is overwritten by the first-feature image
    }
    // ---- first features into the LDS; the warped image's border to zero ----
    {
        const T* f1 = img_ptr<T>(a.first, pair);
        for (int i = t; i < NPIX * C8; i += NT) {
            const int q = i / C8, c = i % C8;
            *(u32x4_t*)(fst + q * CP + c * 8) = *(const u32x4_t*)(f1 + (long long)q * a.first.ld + c * 8);
        }
        for (int i = t; i < BH * BW * C8; i += NT) {
            const int q = i / C8, c = i % C8;
            const int y = q / BW - 4, x = q % BW - 4;
            if ((unsigned)y >= (unsigned)H || (unsigned)x >= (unsigned)W)
                *(u32x4_t*)(wrp + q * CP + c * 8) = u32x4_t{0u, 0u, 0u, 0u};
        }
    }
    __syncthreads();                                   // upflow ready
    // ---- backwarp of the second features (backwarp_kernel's arithmetic) into the bordered image ----
    {
        const T* sb = img_ptr<T>(a.second, pair);
        for (int i = t; i < NPIX * C8; i += NT) {
            const int q = i / C8, g = i % C8;
            const int y = q / W, x = q % W;
            float v[8];
            if constexpr (!PREV) {
                load8(sb + (long long)q * a.second.ld + g * 8, v);
            } else {
                const float fx = up[q * 4 + 0] * a.scale, fy = up[q * 4 + 1] * a.scale;
                const float gxn = (-1.0f + (2.0f * x + 1.0f) / (float)W) + fx / (((float)W - 1.0f) / 2.0f);
                const float gyn = (-1.0f + (2.0f * y + 1.0f) / (float)H) + fy / (((float)H - 1.0f) / 2.0f);
                const float ix = ((gxn + 1.f) * (float)W - 1.f) / 2.f;
                const float iy = ((gyn + 1.f) * (float)H - 1.f) / 2.f;
                const float fx0 = floorf(ix), fy0 = floorf(iy);
                const int x0 = (int)fx0, y0 = (int)fy0, x1 = x0 + 1, y1 = y0 + 1;
                const float wx1 = ix - fx0, wx0 = 1.f - wx1, wy1 = iy - fy0, wy0 = 1.f - wy1;
                const bool vx0 = (unsigned)x0 < (unsigned)W, vx1 = (unsigned)x1 < (unsigned)W;
                const bool vy0 = (unsigned)y0 < (unsigned)H, vy1 = (unsigned)y1 < (unsigned)H;
                const float w00 = (vy0 && vx0) ? wy0 * wx0 : 0.f, w01 = (vy0 && vx1) ? wy0 * wx1 : 0.f;
                const float w10 = (vy1 && vx0) ? wy1 * wx0 : 0.f, w11 = (vy1 && vx1) ? wy1 * wx1 : 0.f;
                const float mask = (w00 + w01 + w10 + w11) > 0.999f ? 1.f : 0.f;
                float s00[8], s01[8], s10[8], s11[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) s00[j] = s01[j] = s10[j] = s11[j] = 0.f;
                if (w00 != 0.f) load8(sb + ((long long)y0 * W + x0) * a.second.ld + g * 8, s00);
                if (w01 != 0.f) load8(sb + ((long long)y0 * W + x1) * a.second.ld + g * 8, s01);
                if (w10 != 0.f) load8(sb + ((long long)y1 * W + x0) * a.second.ld + g * 8, s10);
                if (w11 != 0.f) load8(sb + ((long long)y1 * W + x1) * a.second.ld + g * 8, s11);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    float vv = 0.f;
                    if (w00 != 0.f) vv += w00 * s00[j];
                    if (w01 != 0.f) vv += w01 * s01[j];
                    if (w10 != 0.f) vv += w10 * s10[j];
                    if (w11 != 0.f) vv += w11 * s11[j];
                    v[j] = vv * mask;
                }
            }
            store8(wrp + ((y + 4) * BW + x + 4) * CP + g * 8, v);
        }
    }
    __syncthreads();
    // ---- correlation + LeakyReLU into D[c0 + d] ----
    T* dst = img_ptr<T>(a.D, pair);
    if constexpr (H >= 8) {
        // on MFMA: for output row y and displacement row dy, G[x][x'] = sum_c first[y][x][c] second[y+dy][x'][c]
        // over a 16-wide window of x' (the zero border supplies the out-of-frame columns and rows);
        // out[y][x][(dy+4)*9 + dx+4] = G[x][x+dx] / C.  H = 16: windows x' in [-4, 12) for x < 8 and [4, 20)
        // for x >= 8; H = 8: one window [-4, 12), accumulator rows x >= 8 unused.
        constexpr int NWIN = H == 16 ? 2 : 1, NKS = CP / 32;
        for (int job = wave; job < H * 9 * NWIN; job += NWV) {
            const int win = job % NWIN, dyi = (job / NWIN) % 9, y = job / (NWIN * 9);
            const int x0 = win * 8 - 4;                    // first window column
            const int ya = y + dyi - 4;                    // second-feature row (-4..H+3)
            f32x4_t acc = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < NKS; ++ks) {
                const bf16x8_t A = *(const bf16x8_t*)(fst + (y * W + (col < W ? col : 0)) * CP + ks * 32 + kgl * 8);
                const bf16x8_t B = *(const bf16x8_t*)(wrp + ((ya + 4) * BW + x0 + col + 4) * CP + ks * 32 + kgl * 8);
                acc = mfma16<T>(A, B, acc);
            }
            // lane (kgl, col): G[x = 4*kgl + r][x' = x0 + col]
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int x = 4 * kgl + r, dx = x0 + col - x;
                const bool mine = x < W && (NWIN == 1 || (win == 0) == (x < 8));
                if (mine && dx >= -4 && dx <= 4) {
                    float v = acc[r] / (float)C;
                    v = v > 0.f ? v : 0.1f * v;
                    elem<T>::st(dst + (long long)(y * W + x) * a.D.ld + dyi * 9 + dx + 4, v);
                }
            }
        }
    } else {
        constexpr int NS = NT / NPIX > 81 ? 81 : NT / NPIX;
        for (int i = t; i < NPIX * NS; i += NT) {
            const int q = i % NPIX, sl = i / NPIX;
            const int y = q / W, x = q % W;
            const T* fa = fst + q * CP;
            T* o = dst + (long long)q * a.D.ld;
            for (int d = sl; d < 81; d += NS) {
                const int dy = d / 9 - 4, dx = d % 9 - 4;
                const T* fb = wrp + ((y + 4 + dy) * BW + x + 4 + dx) * CP;
                float acc = 0.f;
#pragma unroll
                for (int c = 0; c < CP; c += 8) {
                    float va[8], vb[8];
                    load8(fa + c, va);
                    load8(fb + c, vb);
#pragma unroll
                    for (int j = 0; j < 8; ++j) acc = fmaf(va[j], vb[j], acc);
                }
                float v = acc / (float)C;
                v = v > 0.f ? v : 0.1f * v;
                elem<T>::st(o + d, v);
            }
        }
    }
    // ---- assembly of [first | upflow | upfeat] ----
    if constexpr (PREV) {
        constexpr int NC = C + 4;
        for (int i = t; i < NPIX * NC; i += NT) {
            const int q = i / NC, c = i % NC;
            const float v = c < C ? elem<T>::ld(fst + q * CP + c) : up[q * 4 + (c - C)];
            elem<T>::st(dst + (long long)q * a.D.ld + 81 + c, v);
        }
    }
}

// threads per block at the 16x16 level (level 2: one block per pair is the whole level's parallelism, 104 blocks
// for the bench's 104 pairs on the side lane's CUs, so the block takes 16 waves; level 3 (8x8) 8 waves, the
// coarser levels 4)
#ifndef DBSR_PREP_NT16
#define DBSR_PREP_NT16 1024
#endif
// the level shapes with a specialised kernel: (H, C, previous level) of the 64x64 pyramid (levels 6..2)
#define DBSR_PREP_LEVELS(X) X(1, 196, false) X(2, 128, true) X(4, 96, true) X(8, 64, true) X(16, 32, true)

}  // namespace (level prep)

extern "C" int dbsr_pwc_level_prep_supported(int h, int w, int c) {
#define DBSR_PREP_OK(HH, CC, PP) if (h == HH && w == HH && c == CC) return 1;
    DBSR_PREP_LEVELS(DBSR_PREP_OK)
#undef DBSR_PREP_OK
    return 0;
}

extern "C" int dbsr_pwc_level_prep(int P, int h, int w, int c, float scale, dbsr_tensor first, dbsr_tensor second,
                                   dbsr_tensor D, dbsr_tensor prev_D, int prev_cin, dbsr_tensor prev_flow,
                                   const float* w_upflow, const float* b_upflow, const void* w_upfeat,
                                   const float* b_upfeat, void* stream) {
    DBSR_CHECK_ARG(P > 0 && h > 0 && w > 0 && c > 0, "pwc_level_prep: bad sizes");
    DBSR_CHECK_ARG(dbsr_pwc_level_prep_supported(h, w, c), "pwc_level_prep: no kernel for a %dx%d level of %d channels "
                   "(dbsr_pwc_level_prep_supported)", h, w, c);
    DBSR_CHECK_ARG(first.ptr && second.ptr && D.ptr && first.map.fpg > 0 && second.map.fpg > 0 && D.map.fpg > 0,
                   "pwc_level_prep: null tensor");
    DBSR_CHECK_ARG((first.dtype == DBSR_BF16 || first.dtype == DBSR_F16) && second.dtype == first.dtype &&
                   D.dtype == first.dtype, "pwc_level_prep: 16-bit tensors of one dtype");
    const int cp = cpad_i(c);
    DBSR_CHECK_ARG(first.ld % 8 == 0 && first.c0 == 0 && second.ld % 8 == 0 && second.c0 == 0 && first.ld >= cp &&
                   second.ld >= cp, "pwc_level_prep: features must be aligned slices of >= %d channels", cp);
    const int has_prev = prev_D.ptr != nullptr;
    DBSR_CHECK_ARG(D.c0 + 81 + (has_prev ? c + 4 : 0) <= D.ld, "pwc_level_prep: D base slice exceeds ld");
    PrepArgs a;
    a.P = P; a.h = h; a.w = w; a.C = c; a.Cp = cp; a.scale = scale;
    a.first = first; a.second = second;
    a.D = D;
    a.D.ptr = (char*)D.ptr + (long long)D.c0 * 2;
    a.D.c0 = 0;
    a.has_prev = has_prev;
    a.pcin32 = 0;
    if (has_prev) {
        DBSR_CHECK_ARG(h % 2 == 0 && w % 2 == 0, "pwc_level_prep: level size must be twice the previous one");
        DBSR_CHECK_ARG(prev_D.dtype == first.dtype && prev_D.map.fpg > 0 && prev_D.c0 == 0 && prev_D.ld % 8 == 0,
                       "pwc_level_prep: bad previous D");
        DBSR_CHECK_ARG(prev_flow.ptr && prev_flow.dtype == DBSR_F32 && prev_flow.map.fpg > 0 && prev_flow.c0 == 0 &&
                       prev_flow.ld >= 8 && prev_flow.ld % 4 == 0, "pwc_level_prep: previous flow must be fp32, ld >= 8");
        DBSR_CHECK_ARG(w_upflow && b_upflow && w_upfeat && b_upfeat, "pwc_level_prep: null ConvT weights");
        a.pcin32 = (prev_cin + 31) / 32 * 32;
        DBSR_CHECK_ARG(a.pcin32 <= prev_D.ld, "pwc_level_prep: previous D has fewer than %d channels", a.pcin32);
    }
    a.pD = prev_D; a.pflow = prev_flow;
    a.wflow = w_upflow; a.bflow = b_upflow; a.wfeat = w_upfeat; a.bfeat = b_upfeat;
    hipStream_t s = (hipStream_t)stream;
    bool launched = false;
#define DBSR_PREP_LAUNCH(HH, CC, PP)                                                                           \
    if (!launched && h == HH && c == CC) {                                                                     \
        DBSR_CHECK_ARG(has_prev == PP, "pwc_level_prep: level %dx%d x %d %s a previous level", h, w, c,          \
                       PP ? "needs" : "takes no");                                                            \
        constexpr int NT = HH >= 16 ? DBSR_PREP_NT16 : HH == 8 ? 512 : 256;                                   \
        if (first.dtype == DBSR_BF16)                                                                          \
            hipLaunchKernelGGL((pwc_level_prep_kernel<bf16_t, HH, CC, PP, NT>), dim3(P), dim3(NT), 0, s, a);   \
        else                                                                                                   \
            hipLaunchKernelGGL((pwc_level_prep_kernel<f16_t, HH, CC, PP, NT>), dim3(P), dim3(NT), 0, s, a);    \
        launched = true;                                                                                       \
    }
    DBSR_PREP_LEVELS(DBSR_PREP_LAUNCH)
#undef DBSR_PREP_LAUNCH
    DBSR_LAUNCH_CHECK();
    return 0;
}
