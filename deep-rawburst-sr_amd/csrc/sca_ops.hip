// BurstSR scoring path: spatial + colour alignment of a prediction to its ground
// truth before the masked PSNR, models/loss/spatial_color_alignment.py:23-108.  The PWC flow and the
// bilinear warps run on the engine / warp kernels; this file holds the rest: PyTorch-semantics bilinear
// resampling (the x1/8 flow and ground-truth downsampling, :96-101), the reflect-padded Gaussian
// smoothing (filtering.py:56-63), the per-image 3x3 least-squares colour fit (:36-44; normal equations
// in fp64, the unique least-squares solution torch.lstsq returns for a full-rank system) and the colour
// transform + validity mask at the prediction's resolution (:45-67).  fp32 NCHW images.
#include "common.hpp"

using namespace dbsr;

namespace {

// F.interpolate(mode='bilinear', align_corners=False) with an explicit scale_factor: source coordinate
// (dst + 0.5) * r - 0.5 clamped at 0, r = 1 / scale_factor (PyTorch's area_pixel_compute_source_index
// and compute_scales_value), taps floor(src) and +1 clamped to the last row / column; times `mul`
__global__ __launch_bounds__(256) void resize_bilinear_kernel(int planes, int ih, int iw, const float* __restrict__ in,
                                                              int oh, int ow, float rh, float rw, float mul,
                                                              float* __restrict__ out) {
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long long)planes * oh * ow) return;
    const int x = (int)(idx % ow);
    const long long t = idx / ow;
    const int y = (int)(t % oh), p = (int)(t / oh);
    const float sy = fmaxf(rh * ((float)y + 0.5f) - 0.5f, 0.f), sx = fmaxf(rw * ((float)x + 0.5f) - 0.5f, 0.f);
    const int y0 = (int)sy, x0 = (int)sx;
    const int y1 = y0 + (y0 < ih - 1 ? 1 : 0), x1 = x0 + (x0 < iw - 1 ? 1 : 0);
    const float ly = sy - (float)y0, lx = sx - (float)x0;
    const float* src = in + (long long)p * ih * iw;
    const float v = (1.f - ly) * ((1.f - lx) * src[y0 * iw + x0] + lx * src[y0 * iw + x1]) +
                    ly * ((1.f - lx) * src[y1 * iw + x0] + lx * src[y1 * iw + x1]);
    out[idx] = v * mul;
}

struct Kern { float k[81]; };

// apply_kernel (filtering.py:56-63): F.pad(reflect, ksz // 2) then a ksz x ksz cross-correlation, per plane
__global__ __launch_bounds__(256) void gauss_reflect_kernel(int planes, int h, int w, int ksz, Kern kern,
                                                            const float* __restrict__ in, float* __restrict__ out) {
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long long)planes * h * w) return;
    const int x = (int)(idx % w);
    const long long t = idx / w;
    const int y = (int)(t % h), p = (int)(t / h);
    const int r = ksz / 2;
    const float* src = in + (long long)p * h * w;
    auto refl = [](int i, int n) { return i < 0 ? -i : (i >= n ? 2 * n - 2 - i : i); };
    float acc = 0.f;
    for (int dy = 0; dy < ksz; ++dy) {
        const int yy = refl(y + dy - r, h);
        for (int dx = 0; dx < ksz; ++dx) acc = fmaf(kern.k[dy * ksz + dx], src[yy * w + refl(x + dx - r, w)], acc);
    }
    out[idx] = acc;
}

// One block per image: normal equations of min_C || Q C - R ||  (Q, R: [pixels of the crop] x 3) in
// fp64, solved by Gaussian elimination with partial pivoting; C[k][j] maps input channel k to output j
__global__ __launch_bounds__(256) void color_fit_kernel(int h, int w, int bi, const float* __restrict__ ref,
                                                        const float* __restrict__ q, float* __restrict__ cmat) {
    const int b = blockIdx.x;
    const long long hw = (long long)h * w;
    const float* R = ref + b * 3 * hw;
    const float* Q = q + b * 3 * hw;
    double s[15];                                   // QtQ (6: 00 01 02 11 12 22) + QtR (9: k*3+j)
    for (int i = 0; i < 15; ++i) s[i] = 0.0;
    const int ch = h - 2 * bi, cw = w - 2 * bi;
    for (int i = threadIdx.x; i < ch * cw; i += blockDim.x) {
        const int y = bi + i / cw, x = bi + i % cw;
        const long long o = (long long)y * w + x;
        const double q0 = Q[o], q1 = Q[o + hw], q2 = Q[o + 2 * hw];
        const double r0 = R[o], r1 = R[o + hw], r2 = R[o + 2 * hw];
        s[0] += q0 * q0; s[1] += q0 * q1; s[2] += q0 * q2; s[3] += q1 * q1; s[4] += q1 * q2; s[5] += q2 * q2;
        s[6] += q0 * r0; s[7] += q0 * r1; s[8] += q0 * r2;
        s[9] += q1 * r0; s[10] += q1 * r1; s[11] += q1 * r2;
        s[12] += q2 * r0; s[13] += q2 * r1; s[14] += q2 * r2;
    }
    __shared__ double red[15][256];
    for (int i = 0; i < 15; ++i) red[i][threadIdx.x] = s[i];
    __syncthreads();
    for (int st = blockDim.x / 2; st > 0; st >>= 1) {
        if ((int)threadIdx.x < st)
            for (int i = 0; i < 15; ++i) red[i][threadIdx.x] += red[i][threadIdx.x + st];
        __syncthreads();
    }
    if (threadIdx.x != 0) return;
    double A[3][6];                                 // [QtQ | QtR], reduced to [I | C]
    auto g = [&](int i) { return red[i][0]; };
    A[0][0] = g(0); A[0][1] = g(1); A[0][2] = g(2);
    A[1][0] = g(1); A[1][1] = g(3); A[1][2] = g(4);
    A[2][0] = g(2); A[2][1] = g(4); A[2][2] = g(5);
    for (int k = 0; k < 3; ++k)
        for (int j = 0; j < 3; ++j) A[k][3 + j] = g(6 + k * 3 + j);
    for (int c = 0; c < 3; ++c) {
        int piv = c;
        for (int r = c + 1; r < 3; ++r)
            if (fabs(A[r][c]) > fabs(A[piv][c])) piv = r;
        if (piv != c)
            for (int j = 0; j < 6; ++j) { const double tmp = A[c][j]; A[c][j] = A[piv][j]; A[piv][j] = tmp; }
        const double d = A[c][c];
        for (int r = 0; r < 3; ++r) {
            if (r == c) continue;
            const double f = d != 0.0 ? A[r][c] / d : 0.0;
            for (int j = c; j < 6; ++j) A[r][j] -= f * A[c][j];
        }
    }
    for (int k = 0; k < 3; ++k)
        for (int j = 0; j < 3; ++j) cmat[b * 9 + k * 3 + j] = (float)(A[k][k] != 0.0 ? A[k][3 + j] / A[k][k] : 0.0);
}

// Colour transform of the test image (:64-67) and the validity mask (:48-61): the low-resolution mask
// err = ||(Q C - R) * 255||_2 < thresh on the crop [bi, h-bi) (zero outside: F.pad), upsampled by
// bilinear interpolation (rh, rw = 1 / upsample_factor, the caller's scale) and thresholded > 0.9
__global__ __launch_bounds__(256) void color_apply_kernel(int n, int h, int w, int bi, const float* __restrict__ ref,
                                                          const float* __restrict__ q, const float* __restrict__ cmat,
                                                          float thresh, const float* __restrict__ test, int oh,
                                                          int ow, float rh, float rw, float* __restrict__ out,
                                                          unsigned char* __restrict__ valid) {
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long long)n * oh * ow) return;
    const int x = (int)(idx % ow);
    const long long t = idx / ow;
    const int y = (int)(t % oh), b = (int)(t / oh);
    float c[9];
    for (int i = 0; i < 9; ++i) c[i] = cmat[b * 9 + i];
    const long long ohw = (long long)oh * ow, o = (long long)y * ow + x;
    const float* T = test + b * 3 * ohw;
    const float t0 = T[o], t1 = T[o + ohw], t2 = T[o + 2 * ohw];
    float* O = out + b * 3 * ohw;
    for (int j = 0; j < 3; ++j) O[o + j * ohw] = t0 * c[j] + t1 * c[3 + j] + t2 * c[6 + j];

    const long long hw = (long long)h * w;
    const float* R = ref + b * 3 * hw;
    const float* Q = q + b * 3 * hw;
    auto vlr = [&](int yy, int xx) -> float {
        if (yy < bi || yy >= h - bi || xx < bi || xx >= w - bi) return 0.f;
        const long long p = (long long)yy * w + xx;
        const float q0 = Q[p], q1 = Q[p + hw], q2 = Q[p + 2 * hw];
        float e2 = 0.f;
        for (int j = 0; j < 3; ++j) {
            const float d = ((q0 * c[j] + q1 * c[3 + j] + q2 * c[6 + j]) - R[p + j * hw]) * 255.0f;
            e2 += d * d;
        }
        return sqrtf(e2) < thresh ? 1.f : 0.f;
    };
    const float sy = fmaxf(rh * ((float)y + 0.5f) - 0.5f, 0.f), sx = fmaxf(rw * ((float)x + 0.5f) - 0.5f, 0.f);
    const int y0 = (int)sy, x0 = (int)sx;
    const int y1 = y0 + (y0 < h - 1 ? 1 : 0), x1 = x0 + (x0 < w - 1 ? 1 : 0);
    const float ly = sy - (float)y0, lx = sx - (float)x0;
    const float v = (1.f - ly) * ((1.f - lx) * vlr(y0, x0) + lx * vlr(y0, x1)) + ly * ((1.f - lx) * vlr(y1, x0) + lx * vlr(y1, x1));
    valid[idx] = v > 0.9f ? 1 : 0;
}

inline unsigned nblk(long long n) { return (unsigned)((n + 255) / 256); }

}  // namespace

extern "C" int dbsr_resize_bilinear(int planes, int ih, int iw, const float* in, int oh, int ow, float rh, float rw,
                                    float mul, float* out, void* stream) {
    DBSR_CHECK_ARG(in && out && planes > 0 && ih > 0 && iw > 0 && oh > 0 && ow > 0, "resize_bilinear: bad arguments");
    hipLaunchKernelGGL(resize_bilinear_kernel, dim3(nblk((long long)planes * oh * ow)), dim3(256), 0,
                       (hipStream_t)stream, planes, ih, iw, in, oh, ow, rh, rw, mul, out);
    DBSR_LAUNCH_CHECK();
    return 0;
}

extern "C" int dbsr_gauss_reflect(int planes, int h, int w, int ksz, const float* k_host, const float* in, float* out,
                                  void* stream) {
    DBSR_CHECK_ARG(in && out && k_host && planes > 0, "gauss_reflect: bad arguments");
    DBSR_CHECK_ARG(ksz >= 1 && ksz <= 9 && ksz % 2 == 1, "gauss_reflect: ksz must be odd and <= 9");
    DBSR_CHECK_ARG(h > ksz / 2 && w > ksz / 2, "gauss_reflect: reflect padding needs h, w > ksz / 2 (F.pad)");
    Kern kern;
    for (int i = 0; i < ksz * ksz; ++i) kern.k[i] = k_host[i];
    hipLaunchKernelGGL(gauss_reflect_kernel, dim3(nblk((long long)planes * h * w)), dim3(256), 0, (hipStream_t)stream,
                       planes, h, w, ksz, kern, in, out);
    DBSR_LAUNCH_CHECK();
    return 0;
}

extern "C" int dbsr_color_fit(int n, int h, int w, int bi, const float* ref, const float* q, float* c_mat,
                              void* stream) {
    DBSR_CHECK_ARG(ref && q && c_mat && n > 0, "color_fit: bad arguments");
    DBSR_CHECK_ARG(bi >= 0 && h - 2 * bi >= 3 && w - 2 * bi >= 1, "color_fit: crop too small");
    hipLaunchKernelGGL(color_fit_kernel, dim3(n), dim3(256), 0, (hipStream_t)stream, h, w, bi, ref, q, c_mat);
    DBSR_LAUNCH_CHECK();
    return 0;
}

extern "C" int dbsr_color_apply(int n, int h, int w, int bi, const float* ref, const float* q, const float* c_mat,
                                float thresh, const float* test, int oh, int ow, float rh, float rw, float* out,
                                unsigned char* valid, void* stream) {
    DBSR_CHECK_ARG(ref && q && c_mat && test && out && valid && n > 0 && oh > 0 && ow > 0, "color_apply: bad arguments");
    hipLaunchKernelGGL(color_apply_kernel, dim3(nblk((long long)n * oh * ow)), dim3(256), 0, (hipStream_t)stream, n, h,
                       w, bi, ref, q, c_mat, thresh, test, oh, ow, rh, rw, out, valid);
    DBSR_LAUNCH_CHECK();
    return 0;
}
