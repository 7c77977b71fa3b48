// The DBSR warp fused with the weight predictor's feature projection of the warped frames (dbsr_warp_project).
//
// Reference: oth_feat = warp(feat, offsets) (models/dbsr/encoders.py:80, models/layers/warp.py: bilinear grid_sample,
// zero padding), then the projection all_feat_proj = ReLU(conv1x1(all_feat) + b) (models/dbsr/merging.py:34-36,75)
// of the same warped embeddings.  Unfused, the warp writes the 512-channel warped frames (245 MB at the bench shape)
// and the 1x1 conv reads them all back; here the projection consumes them in registers as the warp computes them.
//
// A wave owns 16 pixels at a time and lane l computes pixel l & 15: its 4 taps' addresses and weights, then for each
// of the 16 k-steps (32 channels) the 8 channels 32 s + 8 (l >> 4) .. + 7 -- exactly the MFMA 16x16x32 B fragment of
// that k-step, so the warped values go from the bilinear sum straight into the MFMAs (4 output blocks of 16 channels)
// and to `out`, with no LDS round trip and no barrier.  The packed projection weights (64 x 512, 64 KiB) sit in the LDS
// in A-fragment order, loaded once per persistent block; the tap loads of the next DBSR_WP_PD k-steps are in flight
// while a k-step is combined.  The bilinear sums are warp512_bf16_kernel's arithmetic (fp32, taps in order), so
// `out` is bitwise dbsr_warp_bilinear's.
#include "common.hpp"

#include <algorithm>
#include <type_traits>

using namespace dbsr;

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bfv8_t;
typedef __attribute__((ext_vector_type(8))) _Float16 hv8_t;

template <typename T>
__device__ __forceinline__ f32x4_t mma16(u32x4_t a, u32x4_t b, f32x4_t c) {
    if constexpr (std::is_same<T, bf16_t>::value)
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bfv8_t, a), __builtin_bit_cast(bfv8_t, b), c,
                                                       0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(hv8_t, a), __builtin_bit_cast(hv8_t, b), c, 0,
                                                      0, 0);
}

constexpr int WP_C = 512;                  // embedding channels (the warp512 layout)
constexpr int WP_KS = WP_C / 32;           // k-steps of the projection
constexpr int WP_MB = 4;                   // 16-channel output blocks (proj_cout <= 64)
#ifndef DBSR_WP_PD
#define DBSR_WP_PD 4                       // k-steps of tap loads in flight ahead of the one being combined
#endif
#ifndef DBSR_WP_WAVES
#define DBSR_WP_WAVES 8                    // waves per block (all share the block's LDS copy of the weights)
#endif
#ifndef DBSR_WP_BPC
#define DBSR_WP_BPC 2                      // blocks per CU (64 KiB of LDS each)
#endif
constexpr int WP_PD = DBSR_WP_PD;

template <typename T>
__global__ __launch_bounds__(64 * DBSR_WP_WAVES) void warp_proj_kernel(
    int n, int h, int w, dbsr_tensor feat, const float* __restrict__ flow, long long fis, dbsr_tensor out,
    const T* __restrict__ pw, int pw_ld, const float* __restrict__ pb, int pcout, dbsr_tensor pout, int ntiles) {
    __shared__ __attribute__((aligned(16))) u32x4_t lA[WP_MB * WP_KS * 64];     // [block][k-step][lane]
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g = lane >> 4, col = lane & 15;
    const int nmb = pcout / 16;
    // the weights in A-fragment order: block m, k-step s, lane l = W[16 m + (l & 15)][32 s + 8 (l >> 4) .. + 7]
    for (int i = threadIdx.x; i < nmb * WP_KS * 64; i += 64 * DBSR_WP_WAVES) {
        const int l = i & 63, ms = i >> 6, m = ms / WP_KS, ks = ms - m * WP_KS;
        lA[i] = *(const u32x4_t*)(pw + (long long)(16 * m + (l & 15)) * pw_ld + 32 * ks + 8 * (l >> 4));
    }
    float bias[WP_MB][4];
#pragma unroll
    for (int m = 0; m < WP_MB; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r) bias[m][r] = (pb && m < nmb) ? pb[16 * m + 4 * g + r] : 0.f;
    __syncthreads();
    // the block's contiguous range of tiles (an XCD's blocks on adjacent ranges), its waves interleaved over it
    const unsigned b = blockIdx.x, nb = gridDim.x, xcd = b & 7, q8 = nb >> 3, r8 = nb & 7;
    const unsigned lb = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
    const int per = (ntiles + (int)nb - 1) / (int)nb;
    const int t_lo = (int)lb * per, t_hi = min(ntiles, t_lo + per);
    const int hw = h * w;
    const unsigned total = (unsigned)n * hw;
    for (int tile = t_lo + wave; tile < t_hi; tile += DBSR_WP_WAVES) {
        // this lane's pixel: grid = pixel centre + flow, normalised, grid_sample align_corners=False (warp.py:30-44)
        const unsigned pix = (unsigned)tile * 16 + col;
        const bool live = pix < total;
        const unsigned pc = live ? pix : 0;
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
        const T* tp[4];
        float tw[4];
        const T* fb = img_ptr<T>(feat, p) + 8 * g;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int xx = x0 + (t & 1), yy = y0 + (t >> 1);
            const bool ok = (unsigned)xx < (unsigned)w && (unsigned)yy < (unsigned)h;
            tw[t] = ok ? ((t & 1) ? wx1 : wx0) * ((t >> 1) ? wy1 : wy0) : 0.f;
            tp[t] = fb + (ok ? (long long)(yy * w + xx) * feat.ld : 0);     // clamped: in-bounds address, weight 0
        }
        T* ob = img_ptr<T>(out, p) + (long long)rr * out.ld + 8 * g;
        f32x4_t acc[WP_MB];
#pragma unroll
        for (int m = 0; m < WP_MB; ++m) acc[m] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        u32x4_t xr[WP_PD][4];
#pragma unroll
        for (int d = 0; d < WP_PD; ++d)
#pragma unroll
            for (int t = 0; t < 4; ++t) xr[d][t] = *(const u32x4_t*)(tp[t] + 32 * d);
#pragma unroll
        for (int ks = 0; ks < WP_KS; ++ks) {
            u32x4_t v[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) v[t] = xr[ks % WP_PD][t];
            if (ks + WP_PD < WP_KS) {
#pragma unroll
                for (int t = 0; t < 4; ++t) xr[ks % WP_PD][t] = *(const u32x4_t*)(tp[t] + 32 * (ks + WP_PD));
            }
            f32x2_t a2[4] = {{0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}};
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const f32x2_t w2 = {tw[t], tw[t]};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const f32x2_t x2 = {H16<T>::lo(v[t][e]), H16<T>::hi(v[t][e])};
                    a2[e] = __builtin_elementwise_fma(w2, x2, a2[e]);
                }
            }
            u32x4_t o;
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = H16<T>::pack(a2[e][0], a2[e][1]);
            if (live) *(u32x4_t*)(ob + 32 * ks) = o;
#pragma unroll
            for (int m = 0; m < WP_MB; ++m)
                if (m < nmb) acc[m] = mma16<T>(lA[(m * WP_KS + ks) * 64 + lane], o, acc[m]);
        }
        // D row 4 g + r of block m = output channel 16 m + 4 g + r, column = this lane's pixel... of lane col: the
        // accumulator's column is pixel tile*16 + (lane & 15), the same pixel this lane warped
        if (live) {
            T* po = img_ptr<T>(pout, p) + (long long)rr * pout.ld + 4 * g;
#pragma unroll
            for (int m = 0; m < WP_MB; ++m) {
                if (m >= nmb) continue;
                float q[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) q[r] = fmaxf(acc[m][r] + bias[m][r], 0.f);
                *(u32x2_t*)(po + 16 * m) = u32x2_t{H16<T>::pack(q[0], q[1]), H16<T>::pack(q[2], q[3])};
            }
        }
    }
}

int warp_proj_cus() {
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (cus <= 0) cus = 256;
    }
    return cus;
}

}  // namespace

extern "C" int dbsr_warp_project(int n, int h, int w, int c, dbsr_tensor feat, const float* flow,
                                 long long flow_img_stride, dbsr_tensor out, const void* proj_w, const float* proj_b,
                                 int proj_cout, dbsr_tensor proj_out, void* stream) {
    DBSR_CHECK_ARG(feat.ptr && feat.map.fpg > 0 && out.ptr && out.map.fpg > 0 && proj_out.ptr &&
                   proj_out.map.fpg > 0 && flow && proj_w, "warp_project: null tensor");
    DBSR_CHECK_ARG(feat.dtype == out.dtype && proj_out.dtype == feat.dtype &&
                   (feat.dtype == DBSR_F16 || feat.dtype == DBSR_BF16), "warp_project: 16-bit tensors of one dtype");
    DBSR_CHECK_ARG(c == WP_C, "warp_project: c must be %d (got %d)", WP_C, c);
    DBSR_CHECK_ARG(n > 0 && h > 0 && w > 0 && (long long)n * h * w < (1LL << 31), "warp_project: sizes");
    DBSR_CHECK_ARG(feat.ld % 8 == 0 && feat.c0 % 8 == 0 && out.ld % 8 == 0 && out.c0 % 8 == 0,
                   "warp_project: feat / out ld and c0 must be multiples of 8");
    DBSR_CHECK_ARG(proj_cout > 0 && proj_cout % 16 == 0 && proj_cout <= 64, "warp_project: proj_cout in {16,32,48,64}");
    DBSR_CHECK_ARG(proj_out.ld % 4 == 0 && proj_out.c0 % 4 == 0 && proj_out.c0 + proj_cout <= proj_out.ld,
                   "warp_project: proj_out ld / c0 multiples of 4 with c0 + proj_cout <= ld");
    const int ntiles = (int)(((long long)n * h * w + 15) / 16);
    // persistent: DBSR_WP_BPC blocks per CU (64 KiB of LDS each); at least 8 (surplus blocks find an empty tile range)
    const int grid = std::max(8, std::min((ntiles + DBSR_WP_WAVES - 1) / DBSR_WP_WAVES, DBSR_WP_BPC * warp_proj_cus()));
    // packed 1x1 weights (dbsr_conv_pack_weights, cin = 512): rows of kgp * 8 = 512 elements
    const int pw_ld = WP_C;
    hipStream_t s = (hipStream_t)stream;
    if (feat.dtype == DBSR_F16)
        hipLaunchKernelGGL(warp_proj_kernel<f16_t>, dim3(grid), dim3(64 * DBSR_WP_WAVES), 0, s, n, h, w, feat, flow, flow_img_stride,
                           out, (const f16_t*)proj_w, pw_ld, proj_b, proj_cout, proj_out, ntiles);
    else
        hipLaunchKernelGGL(warp_proj_kernel<bf16_t>, dim3(grid), dim3(64 * DBSR_WP_WAVES), 0, s, n, h, w, feat, flow, flow_img_stride,
                           out, (const bf16_t*)proj_w, pw_ld, proj_b, proj_cout, proj_out, ntiles);
    DBSR_LAUNCH_CHECK();
    return 0;
}
