// PWC-Net specific kernels: cost volume, backwarp, transposed-conv upsampling, decoder input assembly,
// input packing/resizing and the final flow upsampling.  All activations NHWC (see dbsr_hip.h).
#include "common.hpp"

using namespace dbsr;

namespace {

// ------------------------------------------------------------------------------------------------
// Cost volume (correlation.py:35-103): out[p,(dy+4)*9+(dx+4),y,x] = sum_c f1[p,c,y,x]*f2[p,c,y+dy,x+dx]/C
// zero outside the image (rbot zero padding, :281-282), then LeakyReLU(0.1) (pwcnet.py:161,169).
// One thread per (pixel, displacement); 8-wide channel loads; fp32 accumulation.
// ------------------------------------------------------------------------------------------------
template <typename T>
__global__ void correlation_kernel(int n, int h, int w, int C, dbsr_tensor f1, dbsr_tensor f2, dbsr_tensor out,
                                   int leaky, int vec) {
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long total = (long long)n * h * w * 81;
    if (idx >= total) return;
    const int d = (int)(idx % 81);
    const long long pix = idx / 81;
    const int p = (int)(pix / (h * w));
    const int rr = (int)(pix - (long long)p * h * w);
    const int y = rr / w, x = rr - y * w;
    const int dy = d / 9 - 4, dx = d % 9 - 4;
    const int y2 = y + dy, x2 = x + dx;
    float acc = 0.f;
    if ((unsigned)y2 < (unsigned)h && (unsigned)x2 < (unsigned)w) {
        const T* a = img_ptr<T>(f1, p) + (long long)rr * f1.ld;
        const T* b = img_ptr<T>(f2, p) + ((long long)y2 * w + x2) * f2.ld;
        int c = 0;
        if (vec) {
            for (; c + 8 <= C; c += 8) {
                float va[8], vb[8];
                load8(a + c, va);
                load8(b + c, vb);
#pragma unroll
                for (int j = 0; j < 8; ++j) acc = fmaf(va[j], vb[j], acc);
            }
        }
        for (; c < C; ++c) acc = fmaf(elem<T>::ld(a + c), elem<T>::ld(b + c), acc);
    }
    float v = acc / (float)C;
    if (leaky) v = v > 0.f ? v : 0.1f * v;
    elem<T>::st(img_ptr<T>(out, p) + (long long)rr * out.ld + d, v);
}

// Cost-volume backward (correlation.py:105-233, K3/K4: updateGradFirst / updateGradSecond), with the
// callers' LeakyReLU(0.1) folded in when leaky != 0 (slope from the sign of the forward output):
//   g[d](y,x)     = gout[d](y,x) * (leaky && out[d](y,x) <= 0 ? 0.1 : 1)
//   dfirst(y,x)   = 1/C sum_d g[d](y,x) * second(y+dy, x+dx)
//   dsecond(y,x)  = 1/C sum_d g[d](y-dy,x-dx) * first(y-dy, x-dx)
// both as gathers (no atomics): one thread per (pair, pixel, 8-channel group).
template <typename T>
__global__ void correlation_bwd_kernel(int n, int h, int w, int C, dbsr_tensor f1, dbsr_tensor f2, dbsr_tensor out,
                                       dbsr_tensor gout, int leaky, dbsr_tensor d1, dbsr_tensor d2) {
    const int groups = (C + 7) / 8;
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long long)n * h * w * groups) return;
    const int g = (int)(idx % groups);
    const long long pix = idx / groups;
    const int p = (int)(pix / (h * w)), rr = (int)(pix - (long long)p * h * w);
    const int y = rr / w, x = rr - y * w;
    const int c0 = g * 8, nc = min(8, C - c0);
    float a1[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, a2[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    auto grad_at = [&](int yy, int xx, int d) {
        const long long o = (long long)(yy * w + xx);
        float gv = elem<T>::ld(img_ptr<T>(gout, p) + o * gout.ld + d);
        if (leaky && elem<T>::ld(img_ptr<T>(out, p) + o * out.ld + d) <= 0.f) gv *= 0.1f;
        return gv;
    };
    for (int d = 0; d < 81; ++d) {
        const int dy = d / 9 - 4, dx = d % 9 - 4;
        // dfirst: second at (y+dy, x+dx)
        const int y2 = y + dy, x2 = x + dx;
        if ((unsigned)y2 < (unsigned)h && (unsigned)x2 < (unsigned)w) {
            const float gv = grad_at(y, x, d);
            const T* b = img_ptr<T>(f2, p) + ((long long)y2 * w + x2) * f2.ld + c0;
            for (int j = 0; j < nc; ++j) a1[j] = fmaf(gv, elem<T>::ld(b + j), a1[j]);
        }
        // dsecond: output pixel (y-dy, x-dx) used this pixel of `second` at displacement d
        const int y1 = y - dy, x1 = x - dx;
        if ((unsigned)y1 < (unsigned)h && (unsigned)x1 < (unsigned)w) {
            const float gv = grad_at(y1, x1, d);
            const T* a = img_ptr<T>(f1, p) + ((long long)y1 * w + x1) * f1.ld + c0;
            for (int j = 0; j < nc; ++j) a2[j] = fmaf(gv, elem<T>::ld(a + j), a2[j]);
        }
    }
    const float inv = 1.0f / (float)C;
    T* o1 = img_ptr<T>(d1, p) + (long long)rr * d1.ld + c0;
    T* o2 = img_ptr<T>(d2, p) + (long long)rr * d2.ld + c0;
    for (int j = 0; j < nc; ++j) {
        elem<T>::st(o1 + j, a1[j] * inv);
        elem<T>::st(o2 + j, a2[j] * inv);
    }
}

// ------------------------------------------------------------------------------------------------
// backwarp (pwcnet.py:16-38): grid = linspace(-1+1/W, 1-1/W) + flow/((W-1)/2), grid_sample bilinear
// zeros align_corners=False, then mask = (sampled ones-channel > 0.999).  The ones-channel is the
// sum of the in-bounds bilinear weights, computed inline (no extra channel).
// ------------------------------------------------------------------------------------------------
template <typename T>
__global__ void backwarp_kernel(int n, int h, int w, int C, dbsr_tensor in, dbsr_tensor flow, float scale,
                                dbsr_tensor out) {
    const int groups = (C + 7) / 8;
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long total = (long long)n * h * w * groups;
    if (idx >= total) return;
    const int g = (int)(idx % groups);
    const long long pix = idx / groups;
    const int p = (int)(pix / (h * w));
    const int rr = (int)(pix - (long long)p * h * w);
    const int y = rr / w, x = rr - y * w;
    const float* fl = img_ptr<float>(flow, p) + (long long)rr * flow.ld;
    const float fx = fl[0] * scale, fy = fl[1] * scale;
    // grid value (normalised) then grid_sample's unnormalisation ((g + 1) * size - 1) / 2
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
    const float mass = w00 + w01 + w10 + w11;
    const float mask = mass > 0.999f ? 1.f : 0.f;
    const T* base = img_ptr<T>(in, p);
    T* o = img_ptr<T>(out, p) + (long long)rr * out.ld;
    const int c_end = min(C, g * 8 + 8);
    for (int c = g * 8; c < c_end; ++c) {
        float v = 0.f;
        if (w00 != 0.f) v += w00 * elem<T>::ld(base + ((long long)y0 * w + x0) * in.ld + c);
        if (w01 != 0.f) v += w01 * elem<T>::ld(base + ((long long)y0 * w + x1) * in.ld + c);
        if (w10 != 0.f) v += w10 * elem<T>::ld(base + ((long long)y1 * w + x0) * in.ld + c);
        if (w11 != 0.f) v += w11 * elem<T>::ld(base + ((long long)y1 * w + x1) * in.ld + c);
        elem<T>::st(o + c, v * mask);
    }
}

// ------------------------------------------------------------------------------------------------
// ConvTranspose2d(k=4, s=2, p=1) (pwcnet.py:119-120): out[oy,ox,co] = b[co] + sum over the 2x2 input
// pixels iy=(oy+1-ky)/2, ix=(ox+1-kx)/2 and all ci of in[iy,ix,ci]*w[ci,co,ky,kx].
// Weights repacked as [ky][kx][co][cin8] (zero-padded to a multiple of 8 channels) so a lane group
// reads them contiguously.  SG lanes per output pixel (lane = 8-channel group, shuffle reduction over
// the group): SG = 1 for the 2-channel upflow (a thread per pixel, no idle lanes), 32 for the ~70
// groups of the upfeat inputs (two pixels per wave, ~2 groups per lane).
// ------------------------------------------------------------------------------------------------
template <typename T, int SG>
__global__ __launch_bounds__(256) void convt_k4s2_kernel(int n, int h, int w, int cin8, int cout, dbsr_tensor in,
                                                         const float* __restrict__ wgt, const float* __restrict__ bias,
                                                         dbsr_tensor out, int vec) {
    const int sl = threadIdx.x & (SG - 1);
    const long long opix = (long long)blockIdx.x * (256 / SG) + threadIdx.x / SG;
    const int H2 = 2 * h, W2 = 2 * w;
    // whole lane groups leave together (the shuffle below stays within a group)
    if (opix >= (long long)n * H2 * W2) return;
    const int p = (int)(opix / (H2 * W2));
    const int rr = (int)(opix - (long long)p * H2 * W2);
    const int oy = rr / W2, ox = rr - oy * W2;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    const T* base = img_ptr<T>(in, p);
    const int ky0 = (oy + 1) & 1, kx0 = (ox + 1) & 1;
    const int ngroups = cin8 / 8;
    for (int a = 0; a < 2; ++a) {
        const int ky = ky0 + 2 * a, iy = (oy + 1 - ky) >> 1;
        if (iy < 0 || iy >= h) continue;
        for (int bq = 0; bq < 2; ++bq) {
            const int kx = kx0 + 2 * bq, ix = (ox + 1 - kx) >> 1;
            if (ix < 0 || ix >= w) continue;
            const T* src = base + ((long long)iy * w + ix) * in.ld;
            const float* wt = wgt + (long long)((ky * 4 + kx) * cout) * cin8;
            for (int cgi = sl; cgi < ngroups; cgi += SG) {
                float v[8];
                if (vec) {
                    load8(src + cgi * 8, v);
                } else {
#pragma unroll
                    for (int j = 0; j < 8; ++j) v[j] = elem<T>::ld(src + cgi * 8 + j);
                }
#pragma unroll
                for (int co = 0; co < 4; ++co) {
                    if (co < cout) {
                        float wv[8];
                        load8(wt + (long long)co * cin8 + cgi * 8, wv);
#pragma unroll
                        for (int j = 0; j < 8; ++j) acc[co] = fmaf(v[j], wv[j], acc[co]);
                    }
                }
            }
        }
    }
#pragma unroll
    for (int co = 0; co < 4; ++co) {
        float v = acc[co];
#pragma unroll
        for (int off = SG / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
        acc[co] = v;
    }
    if (sl == 0) {
        float* o = img_ptr<float>(out, p) + (long long)rr * out.ld;
        for (int co = 0; co < cout; ++co) o[co] = acc[co] + (bias ? bias[co] : 0.f);
    }
}

// ------------------------------------------------------------------------------------------------
// Decoder input assembly (pwcnet.py:171): [vol | first | flow | feat] -> writes first/flow/feat.
// ------------------------------------------------------------------------------------------------
template <typename T>
__global__ void pwc_assemble_kernel(int n, int hw, int C, dbsr_tensor first, dbsr_tensor flow, dbsr_tensor feat,
                                    dbsr_tensor out) {
    const int nc = C + 4;
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long long)n * hw * nc) return;
    const int c = (int)(idx % nc);
    const long long pix = idx / nc;
    const int p = (int)(pix / hw), rr = (int)(pix - (long long)p * hw);
    float v;
    if (c < C)
        v = elem<T>::ld(img_ptr<T>(first, p) + (long long)rr * first.ld + c);
    else if (c < C + 2)
        v = img_ptr<float>(flow, p)[(long long)rr * flow.ld + (c - C)];
    else
        v = img_ptr<float>(feat, p)[(long long)rr * feat.ld + (c - C - 2)];
    elem<T>::st(img_ptr<T>(out, p) + (long long)rr * out.ld + 81 + c, v);
}

// bilinear, align_corners=False source index (PyTorch area_pixel_compute_source_index + the
// upsample_bilinear2d neighbour/lambda computation)
struct Lin {
    int i0, i1;
    float l0, l1;
};
__device__ __forceinline__ Lin lin_index(int dst, int in_size, int out_size) {
    const float scale = (float)in_size / (float)out_size;
    float src = scale * ((float)dst + 0.5f) - 0.5f;
    if (src < 0.f) src = 0.f;
    Lin r;
    r.i0 = (int)src;
    if (r.i0 > in_size - 1) r.i0 = in_size - 1;
    r.i1 = r.i0 + ((r.i0 < in_size - 1) ? 1 : 0);
    r.l1 = src - (float)r.i0;
    r.l0 = 1.f - r.l1;
    return r;
}

// ------------------------------------------------------------------------------------------------
// Burst packing (encoders.py:52-54, pwcnet.py:262-271): raw NHWC frames + resized x_rgb.
// ------------------------------------------------------------------------------------------------
template <typename T>
__global__ void pack_raw_kernel(int F, int H, int W, const float* __restrict__ burst, dbsr_tensor raw) {
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long long)F * H * W) return;
    const int f = (int)(idx / (H * W)), rr = (int)(idx - (long long)f * H * W);
    const float* src = burst + (long long)f * 4 * H * W + rr;
    T* o = img_ptr<T>(raw, f) + (long long)rr * raw.ld;
#pragma unroll
    for (int c = 0; c < 4; ++c) elem<T>::st(o + c, src[(long long)c * H * W]);
}

__device__ __forceinline__ void rgb_at(const float* fr, int HW, int off, float& r, float& g, float& b) {
    r = fr[off];
    g = (fr[HW + off] + fr[2 * HW + off]) / 2.0f;     // x[:, :, 1:3].mean(dim=2)
    b = fr[3 * HW + off];
}

template <typename T>
__global__ void pack_rgb_kernel(int F, int H, int W, int Hp, int Wp, const float* __restrict__ burst,
                                dbsr_tensor rgb) {
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long long)F * Hp * Wp) return;
    const int f = (int)(idx / (Hp * Wp)), rr = (int)(idx - (long long)f * Hp * Wp);
    const int Y = rr / Wp, X = rr - Y * Wp;
    const float* fr = burst + (long long)f * 4 * H * W;
    const Lin ly = lin_index(Y, H, Hp), lx = lin_index(X, W, Wp);
    float c00[3], c01[3], c10[3], c11[3];
    rgb_at(fr, H * W, ly.i0 * W + lx.i0, c00[0], c00[1], c00[2]);
    rgb_at(fr, H * W, ly.i0 * W + lx.i1, c01[0], c01[1], c01[2]);
    rgb_at(fr, H * W, ly.i1 * W + lx.i0, c10[0], c10[1], c10[2]);
    rgb_at(fr, H * W, ly.i1 * W + lx.i1, c11[0], c11[1], c11[2]);
    T* o = img_ptr<T>(rgb, f) + (long long)rr * rgb.ld;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float v = ly.l0 * (lx.l0 * c00[c] + lx.l1 * c01[c]) + ly.l1 * (lx.l0 * c10[c] + lx.l1 * c11[c]);
        elem<T>::st(o + c, v);
    }
}

// ------------------------------------------------------------------------------------------------
// Flow finalisation (pwcnet.py:274-279) + offsets_all % modulo (merging.py:98-105).
// ------------------------------------------------------------------------------------------------
template <typename T>
__global__ void flow_finalize_kernel(int B, int N, int hf, int wf, dbsr_tensor flow, int H, int W, float sx, float sy,
                                     float* __restrict__ offsets, float modulo, dbsr_tensor om) {
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long long)B * N * H * W) return;
    const int f = (int)(idx / (H * W)), rr = (int)(idx - (long long)f * H * W);
    const int b = f / N, nn = f - b * N;
    if (nn == 0) {
        if (om.ptr) {
            T* o = img_ptr<T>(om, f) + (long long)rr * om.ld;
            elem<T>::st(o, 0.f);
            elem<T>::st(o + 1, 0.f);
        }
        return;
    }
    const int p = b * (N - 1) + nn - 1;
    const int y = rr / W, x = rr - y * W;
    const Lin ly = lin_index(y, hf, H), lx = lin_index(x, wf, W);
    const float* fl = img_ptr<float>(flow, p);
    float v[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const float a00 = fl[((long long)ly.i0 * wf + lx.i0) * flow.ld + c];
        const float a01 = fl[((long long)ly.i0 * wf + lx.i1) * flow.ld + c];
        const float a10 = fl[((long long)ly.i1 * wf + lx.i0) * flow.ld + c];
        const float a11 = fl[((long long)ly.i1 * wf + lx.i1) * flow.ld + c];
        const float up = ly.l0 * (lx.l0 * a00 + lx.l1 * a01) + ly.l1 * (lx.l0 * a10 + lx.l1 * a11);
        v[c] = (20.0f * up) * (c == 0 ? sx : sy);
    }
    float* op = offsets + (long long)p * 2 * H * W + rr;
    op[0] = v[0];
    op[(long long)H * W] = v[1];
    if (om.ptr) {
        T* o = img_ptr<T>(om, f) + (long long)rr * om.ld;
#pragma unroll
        for (int c = 0; c < 2; ++c) {     // torch.remainder: fmod, then shift into the divisor's sign
            float m = v[c];
            if (modulo != 0.f) {          // (0: offset_modulo None, merging.py:101-102 skips the remainder)
                m = fmodf(v[c], modulo);
                if (m != 0.f && ((m < 0.f) != (modulo < 0.f))) m += modulo;
            }
            elem<T>::st(o + c, m);
        }
    }
}

inline unsigned nblocks(long long total, int bs) { return (unsigned)((total + bs - 1) / bs); }

template <typename F>
int by_dtype(int dtype, F&& f) {
    if (dtype == DBSR_BF16) return f((bf16_t*)nullptr);
    if (dtype == DBSR_F16) return f((f16_t*)nullptr);
    if (dtype == DBSR_F32) return f((float*)nullptr);
    dbsr_set_error("unsupported dtype %d", dtype);
    return DBSR_E_ARG;
}

bool map_ok(const dbsr_tensor& t) { return t.ptr && t.map.fpg > 0; }

}  // namespace

extern "C" int dbsr_correlation(int n, int h, int w, int c, dbsr_tensor first, dbsr_tensor second, dbsr_tensor out,
                                int leaky, void* stream) {
    DBSR_CHECK_ARG(map_ok(first) && map_ok(second) && map_ok(out), "correlation: bad tensor");
    DBSR_CHECK_ARG(first.dtype == second.dtype && first.dtype == out.dtype, "correlation: dtype mismatch");
    DBSR_CHECK_ARG(n > 0 && h > 0 && w > 0 && c > 0 && out.c0 + 81 <= out.ld, "correlation: bad sizes");
    const int vec = (first.ld % 8 == 0 && first.c0 % 8 == 0 && second.ld % 8 == 0 && second.c0 % 8 == 0);
    const long long total = (long long)n * h * w * 81;
    return by_dtype(first.dtype, [&](auto* tag) {
        using T = std::remove_pointer_t<decltype(tag)>;
        hipLaunchKernelGGL(correlation_kernel<T>, dim3(nblocks(total, 256)), dim3(256), 0, (hipStream_t)stream, n, h,
                           w, c, first, second, out, leaky, vec);
        DBSR_LAUNCH_CHECK();
        return 0;
    });
}

extern "C" int dbsr_correlation_backward(int n, int h, int w, int c, dbsr_tensor first, dbsr_tensor second,
                                         dbsr_tensor out, dbsr_tensor gout, int leaky, dbsr_tensor dfirst,
                                         dbsr_tensor dsecond, void* stream) {
    DBSR_CHECK_ARG(map_ok(first) && map_ok(second) && map_ok(gout) && map_ok(dfirst) && map_ok(dsecond) &&
                   (!leaky || map_ok(out)), "correlation_backward: bad tensor");
    DBSR_CHECK_ARG(first.dtype == second.dtype && gout.dtype == first.dtype && dfirst.dtype == first.dtype &&
                   dsecond.dtype == first.dtype && (!leaky || out.dtype == first.dtype), "correlation_backward: dtype");
    DBSR_CHECK_ARG(n > 0 && h > 0 && w > 0 && c > 0 && gout.c0 + 81 <= gout.ld, "correlation_backward: sizes");
    const long long total = (long long)n * h * w * ((c + 7) / 8);
    return by_dtype(first.dtype, [&](auto* tag) {
        using T = std::remove_pointer_t<decltype(tag)>;
        hipLaunchKernelGGL(correlation_bwd_kernel<T>, dim3(nblocks(total, 256)), dim3(256), 0, (hipStream_t)stream, n,
                           h, w, c, first, second, out, gout, leaky, dfirst, dsecond);
        DBSR_LAUNCH_CHECK();
        return 0;
    });
}

extern "C" int dbsr_backwarp(int n, int h, int w, int c, dbsr_tensor in, dbsr_tensor flow, float scale,
                             dbsr_tensor out, void* stream) {
    DBSR_CHECK_ARG(map_ok(in) && map_ok(flow) && map_ok(out), "backwarp: bad tensor");
    DBSR_CHECK_ARG(in.dtype == out.dtype && flow.dtype == DBSR_F32, "backwarp: dtype mismatch");
    DBSR_CHECK_ARG(n > 0 && h > 0 && w > 0 && c > 0, "backwarp: bad sizes");
    const long long total = (long long)n * h * w * ((c + 7) / 8);
    return by_dtype(in.dtype, [&](auto* tag) {
        using T = std::remove_pointer_t<decltype(tag)>;
        hipLaunchKernelGGL(backwarp_kernel<T>, dim3(nblocks(total, 256)), dim3(256), 0, (hipStream_t)stream, n, h, w,
                           c, in, flow, scale, out);
        DBSR_LAUNCH_CHECK();
        return 0;
    });
}

extern "C" int dbsr_conv_transpose_k4s2(int n, int h, int w, int cin, int cout, dbsr_tensor in, const float* wgt,
                                        const float* bias, dbsr_tensor out, void* stream) {
    DBSR_CHECK_ARG(map_ok(in) && map_ok(out) && wgt, "conv_transpose: bad tensor");
    DBSR_CHECK_ARG(out.dtype == DBSR_F32 && cout >= 1 && cout <= 4 && cin > 0, "conv_transpose: out f32, cout<=4");
    const int cin8 = (cin + 7) / 8 * 8;
    DBSR_CHECK_ARG(in.c0 + cin8 <= in.ld, "conv_transpose: input slice [c0, c0+round_up(cin,8)) exceeds ld");
    const int vec = in.ld % 8 == 0 && in.c0 % 8 == 0;
    const long long opix = (long long)n * 4 * h * w;
    return by_dtype(in.dtype, [&](auto* tag) {
        using T = std::remove_pointer_t<decltype(tag)>;
        const int ng = cin8 / 8;
#define DBSR_CONVT(SG)                                                                                              \
    hipLaunchKernelGGL((convt_k4s2_kernel<T, SG>), dim3(nblocks(opix, 256 / SG)), dim3(256), 0, (hipStream_t)stream, \
                       n, h, w, cin8, cout, in, wgt, bias, out, vec)
        if (ng <= 1) DBSR_CONVT(1);
        else if (ng <= 8) DBSR_CONVT(4);
        else if (ng <= 24) DBSR_CONVT(8);
        else if (ng <= 96) DBSR_CONVT(32);
        else DBSR_CONVT(64);
#undef DBSR_CONVT
        DBSR_LAUNCH_CHECK();
        return 0;
    });
}

extern "C" int dbsr_pwc_assemble(int n, int h, int w, int c, dbsr_tensor first, dbsr_tensor flow, dbsr_tensor feat,
                                 dbsr_tensor out, void* stream) {
    DBSR_CHECK_ARG(map_ok(first) && map_ok(flow) && map_ok(feat) && map_ok(out), "pwc_assemble: bad tensor");
    DBSR_CHECK_ARG(first.dtype == out.dtype && flow.dtype == DBSR_F32 && feat.dtype == DBSR_F32, "pwc_assemble: dtype");
    DBSR_CHECK_ARG(out.c0 + 81 + c + 4 <= out.ld, "pwc_assemble: output slice exceeds ld");
    const long long total = (long long)n * h * w * (c + 4);
    return by_dtype(out.dtype, [&](auto* tag) {
        using T = std::remove_pointer_t<decltype(tag)>;
        hipLaunchKernelGGL(pwc_assemble_kernel<T>, dim3(nblocks(total, 256)), dim3(256), 0, (hipStream_t)stream, n,
                           h * w, c, first, flow, feat, out);
        DBSR_LAUNCH_CHECK();
        return 0;
    });
}

extern "C" int dbsr_pack_burst(int B, int N, int H, int W, const float* burst, dbsr_tensor raw, int Hp, int Wp,
                               dbsr_tensor rgb, void* stream) {
    DBSR_CHECK_ARG(burst && B > 0 && N > 0 && H > 0 && W > 0, "pack_burst: bad args");
    const int F = B * N;
    if (raw.ptr) {
        DBSR_CHECK_ARG(map_ok(raw) && raw.c0 + 4 <= raw.ld, "pack_burst: bad raw tensor");
        int rc = by_dtype(raw.dtype, [&](auto* tag) {
            using T = std::remove_pointer_t<decltype(tag)>;
            hipLaunchKernelGGL(pack_raw_kernel<T>, dim3(nblocks((long long)F * H * W, 256)), dim3(256), 0,
                               (hipStream_t)stream, F, H, W, burst, raw);
            DBSR_LAUNCH_CHECK();
            return 0;
        });
        if (rc) return rc;
    }
    if (rgb.ptr) {
        DBSR_CHECK_ARG(map_ok(rgb) && rgb.c0 + 3 <= rgb.ld && Hp > 0 && Wp > 0, "pack_burst: bad rgb tensor");
        return by_dtype(rgb.dtype, [&](auto* tag) {
            using T = std::remove_pointer_t<decltype(tag)>;
            hipLaunchKernelGGL(pack_rgb_kernel<T>, dim3(nblocks((long long)F * Hp * Wp, 256)), dim3(256), 0,
                               (hipStream_t)stream, F, H, W, Hp, Wp, burst, rgb);
            DBSR_LAUNCH_CHECK();
            return 0;
        });
    }
    return 0;
}

extern "C" int dbsr_flow_finalize(int B, int N, int hf, int wf, dbsr_tensor flow, int H, int W, int Hp, int Wp,
                                  float* offsets, float modulo, dbsr_tensor offs_mod, void* stream) {
    DBSR_CHECK_ARG(map_ok(flow) && flow.dtype == DBSR_F32 && offsets, "flow_finalize: bad flow/offsets");
    DBSR_CHECK_ARG(B > 0 && N > 1 && hf > 0 && wf > 0 && H > 0 && W > 0 && Hp > 0 && Wp > 0, "flow_finalize: sizes");
    if (offs_mod.ptr) DBSR_CHECK_ARG(map_ok(offs_mod) && offs_mod.c0 + 2 <= offs_mod.ld, "flow_finalize: bad offs_mod");
    const float sx = (float)W / (float)Wp, sy = (float)H / (float)Hp;
    const int dt = offs_mod.ptr ? offs_mod.dtype : DBSR_F32;
    return by_dtype(dt, [&](auto* tag) {
        using T = std::remove_pointer_t<decltype(tag)>;
        hipLaunchKernelGGL(flow_finalize_kernel<T>, dim3(nblocks((long long)B * N * H * W, 256)), dim3(256), 0,
                           (hipStream_t)stream, B, N, hf, wf, flow, H, W, sx, sy, offsets, modulo, offs_mod);
        DBSR_LAUNCH_CHECK();
        return 0;
    });
}

extern "C" int dbsr_zero(void* ptr, size_t bytes, void* stream) {
    DBSR_CHECK_ARG(ptr || bytes == 0, "zero: null pointer");
    hipError_t e = hipMemsetAsync(ptr, 0, bytes, (hipStream_t)stream);
    if (e != hipSuccess) {
        dbsr_set_error("hipMemsetAsync: %s", hipGetErrorString(e));
        return (int)e;
    }
    return 0;
}
