// Error-diffusion rounding of conv weights to the 16-bit compute dtype (dbsr_weights_round_diffuse).
//
// Rounding every weight to its nearest fp16 value leaves per output channel a sum of rounding errors that grows
// like sqrt(K) ulps; the ReLU activations a conv sees share a large common mean, so that sum acts on them as a
// coherent bias error, and it was the largest part of the fp16 forward's error against the fp32 reference
// (tools/precision_attrib.py: rounding the decoder post-ResBlocks' weights alone was half of the error^2).  Here
// each output channel's K weights (taps x input channels, the packed order) are rounded in sequence with the
// running error carried into the next: q_k = round(w_k - e_k), e_{k+1} = e_k + (q_k - w_k).  The carried error stays
// within half an ulp of the channel's largest weight, so every q_k is within one such ulp of w_k and a channel's
// error sum within half of one.
#include "common.hpp"

using namespace dbsr;

namespace {

constexpr int MAX_K = 9 * 1152;      // taps x input channels per output channel (LDS staging)

template <typename T>
__device__ __forceinline__ float round16(float v);
template <>
__device__ __forceinline__ float round16<f16_t>(float v) { return (float)(f16_t)v; }
template <>
__device__ __forceinline__ float round16<bf16_t>(float v) { return bf2f(f2bf(v)); }

// one wave per output channel: the row is staged in the LDS in K order (coalesced loads), lane 0 runs the carried
// rounding, and the wave writes the row back in the torch layout
template <typename T>
__global__ __launch_bounds__(64) void diffuse_round_kernel(const float* __restrict__ w, int cin, int taps,
                                                           float* __restrict__ out) {
    __shared__ float row[MAX_K];
    const int co = blockIdx.x, K = cin * taps;
    const float* src = w + (long long)co * K;                     // torch [cout][cin][kh][kw]: index c * taps + tap
    for (int i = threadIdx.x; i < K; i += 64) {
        const int c = i / taps, tap = i - c * taps;
        row[tap * cin + c] = src[i];                               // K order: tap-major, then channel
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float e = 0.f;
        for (int k = 0; k < K; ++k) {
            const float v = row[k];
            const float q = round16<T>(v - e);
            e += q - v;
            row[k] = q;
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < K; i += 64) {
        const int c = i / taps, tap = i - c * taps;
        out[(long long)co * K + i] = row[tap * cin + c];
    }
}

}  // namespace

extern "C" int dbsr_weights_round_diffuse(const float* w, int cout, int cin, int kh, int kw, int dtype, float* w_out,
                                          void* stream) {
    DBSR_CHECK_ARG(w && w_out, "weights_round_diffuse: null pointer");
    DBSR_CHECK_ARG(cout > 0 && cin > 0 && kh > 0 && kw > 0, "weights_round_diffuse: bad shape");
    DBSR_CHECK_ARG((long long)cin * kh * kw <= MAX_K, "weights_round_diffuse: K = %d exceeds %d", cin * kh * kw, MAX_K);
    DBSR_CHECK_ARG(dtype == DBSR_F16 || dtype == DBSR_BF16, "weights_round_diffuse: dtype must be 16-bit");
    DBSR_CHECK_ARG(w != w_out, "weights_round_diffuse: out must not alias w");
    hipStream_t s = (hipStream_t)stream;
    if (dtype == DBSR_F16)
        hipLaunchKernelGGL(diffuse_round_kernel<f16_t>, dim3(cout), dim3(64), 0, s, w, cin, kh * kw, w_out);
    else
        hipLaunchKernelGGL(diffuse_round_kernel<bf16_t>, dim3(cout), dim3(64), 0, s, w, cin, kh * kw, w_out);
    DBSR_LAUNCH_CHECK();
    return 0;
}
