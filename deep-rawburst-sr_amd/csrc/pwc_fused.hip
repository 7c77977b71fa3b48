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

inline int round_up_i(int a, int b) { return (a + b - 1) / b * b; }
inline int cpad_i(int c) { return c <= 16 ? round_up_i(c, 8) : round_up_i(c, 32); }
// LDS pixel stride of an image with c channels: the padded width (+8 above 16 channels, which spreads the
// 16 pixel rows of a B-fragment read over the banks)
inline int lds_ld(int c) { return cpad_i(c) <= 16 ? cpad_i(c) : cpad_i(c) + 8; }

constexpr int EXT_CONVS = 18;
constexpr int EXT_R0 = 66 * 66 * 8;                 // input frame, bordered, 8 channels
constexpr int EXT_R1 = 34 * 34 * 16;                // level-1 images, bordered, 16 channels
constexpr int EXT_ELEMS = EXT_R0 + 2 * EXT_R1;      // 143.7 KiB of 16-bit elements

struct ExtConv {
    const void* w;
    const float* bias;
    int Kp, CG, KG;          // packed row length, 8-channel groups per tap, real k-groups (9 * CG)
    int ks_lo, ks_hi;        // k-steps that contain an in-frame tap
    int mt, cout;            // 16-cout M tiles (padded width / 16), real couts
    int stride;
    int ih, iw, ild;         // input image (interior size) and its LDS pixel stride
    int oh, ow, old;         // output image
    int in_buf, out_buf;     // LDS images 0 (input frame), 1, 2
    int level;               // >= 0: also store to the level output tensor
};

struct ExtArgs {
    int F;
    dbsr_tensor rgb;         // [F][64][64][8]
    dbsr_tensor lv[6];       // level outputs [F][64 >> (l+1)]^2 [cpad(C_l)]
    ExtConv cv[EXT_CONVS];
};

template <typename T>
__global__ __launch_bounds__(512) void pwc_extract_kernel(ExtArgs a) {
    __shared__ __attribute__((aligned(16))) u32x4_t smem[EXT_ELEMS / 8];
    T* const base = (T*)smem;
    const int f = blockIdx.x;
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int kgl = lane >> 4, col = lane & 15;

    // the frame into image 0 (66x66, zero border)
    {
        const T* src = img_ptr<T>(a.rgb, f);
        for (int i = threadIdx.x; i < 66 * 66; i += 512) {
            const int y = i / 66 - 1, x = i - (i / 66) * 66 - 1;
            u32x4_t v = u32x4_t{0u, 0u, 0u, 0u};
            if ((unsigned)y < 64u && (unsigned)x < 64u) v = *(const u32x4_t*)(src + (y * 64 + x) * a.rgb.ld);
            *(u32x4_t*)(base + i * 8) = v;
        }
    }
    auto img = [&](int b) { return base + (b == 0 ? 0 : b == 1 ? EXT_R0 : EXT_R0 + EXT_R1); };

    for (int ci = 0; ci < EXT_CONVS; ++ci) {
        __syncthreads();                  // the previous conv's output is complete; its input is consumed
        const ExtConv& cv = a.cv[ci];
        const T* in = img(cv.in_buf);
        T* out = img(cv.out_buf);
        const int obw = cv.ow + 2, obh = cv.oh + 2, ibw = cv.iw + 2;
        // the output image's border (every channel slot) to zero: the buffer held another geometry before
        {
            const int s8 = cv.old / 8, nb = 2 * obw + 2 * cv.oh;
            for (int i = threadIdx.x; i < nb * s8; i += 512) {
                const int bp = i / s8, c = i - bp * s8;
                int y, x;
                if (bp < obw) { y = 0; x = bp; }
                else if (bp < 2 * obw) { y = obh - 1; x = bp - obw; }
                else { const int r = bp - 2 * obw; y = 1 + (r >> 1); x = (r & 1) ? obw - 1 : 0; }
                *(u32x4_t*)(out + (y * obw + x) * cv.old + c * 8) = u32x4_t{0u, 0u, 0u, 0u};
            }
        }
        const int npix = cv.oh * cv.ow;
        const int ntiles = (npix + 15) / 16;
        const int items = cv.mt * ntiles;
        const int nks = cv.ks_hi - cv.ks_lo;
        // epilogue of one (M tile m, N tile n) accumulator: lane (kgl, col) holds couts m*16 + 4*kgl .. +3 of
        // pixel n*16 + col
        auto store = [&](const f32x4_t& acc, int m, int n) {
            const int p = n * 16 + col;
            if (p >= npix) return;
            const int oy = p / cv.ow, ox = p - (p / cv.ow) * cv.ow;
            const int co = m * 16 + 4 * kgl;
            float v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float b = (cv.bias && co + r < cv.cout) ? cv.bias[co + r] : 0.f;
                const float t = acc[r] + b;
                v[r] = t > 0.f ? t : 0.1f * t;
            }
            uint2 q;
            q.x = H16<T>::pack(v[0], v[1]);
            q.y = H16<T>::pack(v[2], v[3]);
            *(uint2*)(out + ((oy + 1) * obw + ox + 1) * cv.old + co) = q;
            if (cv.level >= 0) {
                const dbsr_tensor& L = a.lv[cv.level];
                *(uint2*)(img_ptr<T>(L, f) + (long long)p * L.ld + co) = q;
            }
        };
        // the LDS offset of k-step j's B-fragment relative to a pixel's window origin (tap-major k-groups)
        auto b_off = [&](int j, bool& ok) {
            const int kg = (cv.ks_lo + j) * 4 + kgl;
            const int tap = kg / cv.CG, cg = kg - tap * cv.CG;
            ok = kg < cv.KG;
            const int ky = tap / 3, kx = tap - (tap / 3) * 3;
            return (ky * ibw + kx) * cv.ild + cg * 8;
        };
        auto origin = [&](int n) {          // window origin of this lane's pixel in tile n (pad slots: pixel 0)
            const int p = n * 16 + col;
            const int oy = p < npix ? p / cv.ow : 0, ox = p < npix ? p - (p / cv.ow) * cv.ow : 0;
            return in + ((oy * cv.stride) * ibw + ox * cv.stride) * cv.ild;
        };
        if (8 % cv.mt == 0 && nks <= 16) {
            // every item of this wave has M tile wave % mt: its A-fragments and B offsets load once, then the
            // wave walks its N tiles two at a time (two independent MFMA chains)
            const int m = wave % cv.mt, nstep = 8 / cv.mt;
            const T* wrow = (const T*)cv.w + (long long)(m * 16 + col) * cv.Kp + kgl * 8;
            bf16x8_t A[16];
            int bo[16];
            bool bv[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                A[j] = bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
                bv[j] = false;
                bo[j] = 0;
                if (j < nks) {
                    A[j] = *(const bf16x8_t*)(wrow + (cv.ks_lo + j) * 32);
                    bo[j] = b_off(j, bv[j]);
                }
            }
            for (int n = wave / cv.mt; n < ntiles; n += 2 * nstep) {
                const int n2 = n + nstep;
                const T* b1 = origin(n);
                const T* b2 = origin(n2 < ntiles ? n2 : n);
                f32x4_t acc1 = f32x4_t{0.f, 0.f, 0.f, 0.f}, acc2 = acc1;
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    if (j < nks) {
                        const bf16x8_t z = bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
                        const bf16x8_t B1 = bv[j] ? *(const bf16x8_t*)(b1 + bo[j]) : z;
                        const bf16x8_t B2 = bv[j] ? *(const bf16x8_t*)(b2 + bo[j]) : z;
                        acc1 = mfma16<T>(A[j], B1, acc1);
                        acc2 = mfma16<T>(A[j], B2, acc2);
                    }
                }
                store(acc1, m, n);
                if (n2 < ntiles) store(acc2, m, n2);
            }
            continue;
        }
        for (int it = wave; it < items; it += 8) {
            const int m = it % cv.mt, n = it / cv.mt;
            const T* bin = origin(n);
            const T* wrow = (const T*)cv.w + (long long)(m * 16 + col) * cv.Kp + kgl * 8;
            f32x4_t acc = f32x4_t{0.f, 0.f, 0.f, 0.f};
            for (int k0 = 0; k0 < nks; k0 += 8) {
                bf16x8_t A[8], B[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const bool ok = k0 + j < nks;
                    A[j] = *(const bf16x8_t*)(wrow + (cv.ks_lo + (ok ? k0 + j : 0)) * 32);
                    bool live;
                    const int off = b_off(ok ? k0 + j : 0, live);
                    B[j] = (ok && live) ? *(const bf16x8_t*)(bin + off) : bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
                }
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    if (k0 + j < nks) acc = mfma16<T>(A[j], B[j], acc);
            }
            store(acc, m, n);
        }
    }
}

}  // namespace

extern "C" int dbsr_pwc_extract_supported(int Hp, int Wp) { return Hp == 64 && Wp == 64 ? 1 : 0; }

extern "C" int dbsr_pwc_extract(int F, int Hp, int Wp, dbsr_tensor rgb, const dbsr_pwc_ext_conv* convs,
                                const dbsr_tensor* levels, void* stream) {
    static const int CH[7] = {3, 16, 32, 64, 96, 128, 196};    // pwcnet.py:49-100
    DBSR_CHECK_ARG(convs && levels && rgb.ptr && rgb.map.fpg > 0, "pwc_extract: null argument");
    DBSR_CHECK_ARG(dbsr_pwc_extract_supported(Hp, Wp), "pwc_extract: needs a 64x64 frame (got %dx%d)", Hp, Wp);
    DBSR_CHECK_ARG(rgb.dtype == DBSR_BF16 || rgb.dtype == DBSR_F16, "pwc_extract: 16-bit activations only");
    DBSR_CHECK_ARG(rgb.ld == 8 && rgb.c0 == 0, "pwc_extract: rgb must be the 8-channel packed frame");
    DBSR_CHECK_ARG(F > 0, "pwc_extract: no frames");
    ExtArgs a;
    a.F = F;
    a.rgb = rgb;
    int in_buf = 0, ih = 64;
    for (int l = 0; l < 6; ++l) {
        const dbsr_tensor& L = levels[l];
        DBSR_CHECK_ARG(L.ptr && L.dtype == rgb.dtype && L.map.fpg > 0 && L.c0 == 0 && L.ld == cpad_i(CH[l + 1]),
                       "pwc_extract: level %d output must be a %d-channel slice of ld %d", l + 1, CH[l + 1],
                       cpad_i(CH[l + 1]));
        a.lv[l] = L;
        for (int j = 0; j < 3; ++j) {
            const int i = 3 * l + j;
            const dbsr_pwc_ext_conv& c = convs[i];
            const int cin = j == 0 ? CH[l] : CH[l + 1], cout = CH[l + 1], s = j == 0 ? 2 : 1;
            DBSR_CHECK_ARG(c.w && c.cin == cin && c.cout == cout && c.stride == s,
                           "pwc_extract: conv %d must be %d -> %d, stride %d", i, cin, cout, s);
            ExtConv& e = a.cv[i];
            e.w = c.w;
            e.bias = c.bias;
            e.CG = cpad_i(cin) / 8;
            e.KG = 9 * e.CG;
            e.Kp = round_up_i(e.KG, 4) * 8;
            e.mt = cpad_i(cout) / 16;
            e.cout = cout;
            e.stride = s;
            e.ih = e.iw = ih;
            e.oh = e.ow = (ih + 2 - 3) / s + 1;
            e.ild = i == 0 ? 8 : lds_ld(cin);
            e.old = lds_ld(cout);
            // taps with an in-frame input pixel for some output pixel (pad 1)
            int tlo = 9, thi = -1;
            for (int ky = 0; ky < 3; ++ky)
                for (int kx = 0; kx < 3; ++kx) {
                    bool yok = false, xok = false;
                    for (int o = 0; o < e.oh; ++o) yok |= (unsigned)(o * s - 1 + ky) < (unsigned)ih;
                    for (int o = 0; o < e.ow; ++o) xok |= (unsigned)(o * s - 1 + kx) < (unsigned)ih;
                    if (yok && xok) {
                        tlo = std::min(tlo, ky * 3 + kx);
                        thi = std::max(thi, ky * 3 + kx);
                    }
                }
            e.ks_lo = (tlo * e.CG) / 4;
            e.ks_hi = std::min(((thi + 1) * e.CG + 3) / 4, e.Kp / 32);
            e.in_buf = in_buf;
            e.out_buf = in_buf == 1 ? 2 : 1;
            e.level = j == 2 ? l : -1;
            const int cap = e.out_buf == 0 ? EXT_R0 : EXT_R1;
            DBSR_CHECK_ARG((e.oh + 2) * (e.ow + 2) * e.old <= cap, "pwc_extract: level %d image exceeds its LDS buffer",
                           l + 1);
            in_buf = e.out_buf;
            ih = e.oh;
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

template <typename T>
__global__ __launch_bounds__(256) void pwc_level_prep_kernel(PrepArgs a) {
    __shared__ __attribute__((aligned(16))) unsigned char smem[PREP_LDS_BYTES];
    const int pair = blockIdx.x, h = a.h, w = a.w, npix = h * w, Cp = a.Cp, c8 = Cp / 8;
    const int bw = w + 8, bh = h + 8;
    float* up = (float*)smem;                          // [npix][4]: upflow x, y, upfeat 0, 1
    T* fst = (T*)(smem + npix * 16);                   // [npix][Cp]
    T* wrp = fst + npix * Cp;                          // [(h+8) x (w+8)][Cp], 4-pixel zero border
    const int t = threadIdx.x;

    // ---- upflow / upfeat (ConvTranspose2d k4 s2 p1) of the previous level ----
    // upfeat: every (tap, cout) contribution of every previous-level pixel as one small GEMM on MFMA,
    // part[in_px][(ky*4+kx)*2+co] = sum_ci D_prev[in_px][ci] * w[ky][kx][co][ci] (M = 32 rows, N = the previous
    // level's pixels, K = its channels), then each output pixel sums its <= 4 (input pixel, tap) terms.  The
    // 2-channel upflow keeps the scalar form (convt_k4s2_kernel's arithmetic).
    float* part = (float*)(smem + npix * 16);         // [npix / 4][32] (before the first-feature image exists)
    if (a.has_prev) {
        const int pw = w / 2, pnp = npix / 4;
        const int lane = t & 63, wave = t >> 6, kgl = lane >> 4, col = lane & 15;
        const int ntn = (pnp + 15) / 16, nks = a.pcin32 / 32;
        const T* pd = img_ptr<T>(a.pD, pair);
        for (int item = wave; item < 2 * ntn; item += 4) {
            const int mt = item & 1, nt = item >> 1;
            const int q = nt * 16 + col;
            const T* brow = pd + (long long)(q < pnp ? q : 0) * a.pD.ld + kgl * 8;
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
            if (q < pnp) {
#pragma unroll
                for (int r = 0; r < 4; ++r) part[q * 32 + mt * 16 + 4 * kgl + r] = acc[r];
            }
        }
        __syncthreads();
        for (int q = t; q < npix; q += 256) {
            const int oy = q / w, ox = q - (q / w) * w;
            float af[2];
            convt_px<float>(a, a.pflow, pair, 8, a.wflow, oy, ox, 0, 1, af);
            float ad0 = 0.f, ad1 = 0.f;
            const int ky0 = (oy + 1) & 1, kx0 = (ox + 1) & 1;
            for (int aa = 0; aa < 2; ++aa) {
                const int ky = ky0 + 2 * aa, iy = (oy + 1 - ky) >> 1;
                if (iy < 0 || iy >= h / 2) continue;
                for (int bq = 0; bq < 2; ++bq) {
                    const int kx = kx0 + 2 * bq, ix = (ox + 1 - kx) >> 1;
                    if (ix < 0 || ix >= pw) continue;
                    const float* pp = part + (iy * pw + ix) * 32 + (ky * 4 + kx) * 2;
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
        for (int i = t; i < npix * c8; i += 256) {
            const int q = i / c8, c = i - q * c8;
            *(u32x4_t*)(fst + q * Cp + c * 8) = *(const u32x4_t*)(f1 + (long long)q * a.first.ld + c * 8);
        }
        for (int i = t; i < bh * bw * c8; i += 256) {
            const int q = i / c8, c = i - q * c8;
            const int y = q / bw - 4, x = q - (q / bw) * bw - 4;
            if ((unsigned)y >= (unsigned)h || (unsigned)x >= (unsigned)w)
                *(u32x4_t*)(wrp + q * Cp + c * 8) = u32x4_t{0u, 0u, 0u, 0u};
        }
    }
    __syncthreads();                                   // upflow ready
    // ---- backwarp of the second features (backwarp_kernel's arithmetic) into the bordered image ----
    {
        const T* sb = img_ptr<T>(a.second, pair);
        for (int i = t; i < npix * c8; i += 256) {
            const int q = i / c8, g = i - q * c8;
            const int y = q / w, x = q - (q / w) * w;
            float v[8];
            if (!a.has_prev) {
                load8(sb + (long long)q * a.second.ld + g * 8, v);
            } else {
                const float fx = up[q * 4 + 0] * a.scale, fy = up[q * 4 + 1] * a.scale;
                const float gxn = (-1.0f + (2.0f * x + 1.0f) / (float)w) + fx / (((float)w - 1.0f) / 2.0f);
                const float gyn = (-1.0f + (2.0f * y + 1.0f) / (float)h) + fy / (((float)h - 1.0f) / 2.0f);
                const float ix = ((gxn + 1.f) * (float)w - 1.f) / 2.f;
                const float iy = ((gyn + 1.f) * (float)h - 1.f) / 2.f;
                const float fx0 = floorf(ix), fy0 = floorf(iy);
                const int x0 = (int)fx0, y0 = (int)fy0, x1 = x0 + 1, y1 = y0 + 1;
                const float wx1 = ix - fx0, wx0 = 1.f - wx1, wy1 = iy - fy0, wy0 = 1.f - wy1;
                const bool vx0 = (unsigned)x0 < (unsigned)w, vx1 = (unsigned)x1 < (unsigned)w;
                const bool vy0 = (unsigned)y0 < (unsigned)h, vy1 = (unsigned)y1 < (unsigned)h;
                const float w00 = (vy0 && vx0) ? wy0 * wx0 : 0.f, w01 = (vy0 && vx1) ? wy0 * wx1 : 0.f;
                const float w10 = (vy1 && vx0) ? wy1 * wx0 : 0.f, w11 = (vy1 && vx1) ? wy1 * wx1 : 0.f;
                const float mask = (w00 + w01 + w10 + w11) > 0.999f ? 1.f : 0.f;
                float s00[8], s01[8], s10[8], s11[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) s00[j] = s01[j] = s10[j] = s11[j] = 0.f;
                if (w00 != 0.f) load8(sb + ((long long)y0 * w + x0) * a.second.ld + g * 8, s00);
                if (w01 != 0.f) load8(sb + ((long long)y0 * w + x1) * a.second.ld + g * 8, s01);
                if (w10 != 0.f) load8(sb + ((long long)y1 * w + x0) * a.second.ld + g * 8, s10);
                if (w11 != 0.f) load8(sb + ((long long)y1 * w + x1) * a.second.ld + g * 8, s11);
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
            store8(wrp + ((y + 4) * bw + x + 4) * Cp + g * 8, v);
        }
    }
    __syncthreads();
    // ---- correlation + LeakyReLU into D[c0 + d]; assembly of [first | upflow | upfeat] ----
    T* dst = img_ptr<T>(a.D, pair);
    {
        const int ns = 256 / npix > 81 ? 81 : (256 / npix > 0 ? 256 / npix : 1);
        for (int i = t; i < npix * ns; i += 256) {
            const int q = i % npix, sl = i / npix;
            const int y = q / w, x = q - (q / w) * w;
            const T* fa = fst + q * Cp;
            T* o = dst + (long long)q * a.D.ld;
            for (int d = sl; d < 81; d += ns) {
                const int dy = d / 9 - 4, dx = d - (d / 9) * 9 - 4;
                const T* fb = wrp + ((y + 4 + dy) * bw + x + 4 + dx) * Cp;
                float acc = 0.f;
                for (int c = 0; c < Cp; c += 8) {
                    float va[8], vb[8];
                    load8(fa + c, va);
                    load8(fb + c, vb);
#pragma unroll
                    for (int j = 0; j < 8; ++j) acc = fmaf(va[j], vb[j], acc);
                }
                float v = acc / (float)a.C;
                v = v > 0.f ? v : 0.1f * v;
                elem<T>::st(o + d, v);
            }
        }
    }
    if (a.has_prev) {
        const int nc = a.C + 4;
        for (int i = t; i < npix * nc; i += 256) {
            const int q = i / nc, c = i - q * nc;
            const float v = c < a.C ? elem<T>::ld(fst + q * Cp + c) : up[q * 4 + (c - a.C)];
            elem<T>::st(dst + (long long)q * a.D.ld + 81 + c, v);
        }
    }
}

}  // namespace (level prep)

extern "C" int dbsr_pwc_level_prep_supported(int h, int w, int c) {
    const int cp = cpad_i(c);
    const int part = (h * w / 4) * 32 * 4;              // upfeat partials (reuse the first-feature region)
    const int img = std::max(h * w * cp * 2 + (h + 8) * (w + 8) * cp * 2, part);
    return h * w * 16 + img <= PREP_LDS_BYTES && h * w <= 256 ? 1 : 0;
}

extern "C" int dbsr_pwc_level_prep(int P, int h, int w, int c, float scale, dbsr_tensor first, dbsr_tensor second,
                                   dbsr_tensor D, dbsr_tensor prev_D, int prev_cin, dbsr_tensor prev_flow,
                                   const float* w_upflow, const float* b_upflow, const void* w_upfeat,
                                   const float* b_upfeat, void* stream) {
    DBSR_CHECK_ARG(P > 0 && h > 0 && w > 0 && c > 0, "pwc_level_prep: bad sizes");
    DBSR_CHECK_ARG(dbsr_pwc_level_prep_supported(h, w, c), "pwc_level_prep: %dx%d x %d channels exceed the LDS tile",
                   h, w, c);
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
    if (first.dtype == DBSR_BF16)
        hipLaunchKernelGGL(pwc_level_prep_kernel<bf16_t>, dim3(P), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL(pwc_level_prep_kernel<f16_t>, dim3(P), dim3(256), 0, s, a);
    DBSR_LAUNCH_CHECK();
    return 0;
}
