// Shared pieces of the implicit-GEMM conv kernels (conv2d.hip) and the fused 64-channel ResBlock (resblock64.hip):
// the kernel argument block, the MFMA fragment types, the halo swizzle and the ResBlock kernels' tile order.
#pragma once
#include "common.hpp"

#include <vector>

namespace dbsr {

inline int round_up(int a, int b) { return (a + b - 1) / b * b; }
// channel padding of the packed K dimension (dbsr_hip.h): 8 for cin <= 16, else 32, so every
// conv with cin > 16 is a whole number of 32-channel MFMA chunks per tap
inline int cin_pad(int cin) { return cin <= 16 ? round_up(cin, 8) : round_up(cin, 32); }


inline bool is16(int dtype) { return dtype == DBSR_BF16 || dtype == DBSR_F16; }   // 16-bit activations
inline int esize(int dtype) { return is16(dtype) ? 2 : 4; }   // dbsr_set_conv_algo: 0 generic only, 1 LDS-tiled where applicable, 2 + pipelined


struct ConvK {
    const void* x; long long x_is; int x_ld; dbsr_frame_map xm; int in_h, in_w;
    const void* w; const float* bias; int Kp, KG, KGp, CG, kw, stride, pad, dil, cout;
    void* y; int y_f32; long long y_is; int y_ld, y_c0; dbsr_frame_map ym; int out_h, out_w;
    int act;
    const void* r; long long r_is; int r_ld, r_c0; dbsr_frame_map rm; int post_act;
    const void* gt; long long g_is; int g_ld, g_c0; dbsr_frame_map gm;   // gate (ReLU backward): out *= (gate > 0)
    int out_mode, shuffle, cps;
    int npix;
    int vec_store;
    int ksplit;        // K slices (generic kernel); > 1: fp32 partials to ws, summed by conv_splitk_finalize
    float* ws;         // [ksplit][npix][cw] fp32
    int cw;            // round_up(cout, 4)
    const void* w_pipe;  // chunk-major weight copy (3x3, cin > 16): [cout/16][chunk][tap][4 k-groups][16 co][8]
    int max_blocks;      // persistent kernel: workgroup cap (0 = one per CU)
    const float* head_w; // fused 1x1 head (pipelined kernel, EPI 4): fp32 [head_cout][cout], bias [head_cout]
    const float* head_b;
    int head_cout;       // y is then the head's fp32 NCHW output (y_is = image stride)
    int stage_epi;       // generic kernel, MT == 4: LDS-staged 16-B-row epilogue (set by launch_conv)
};

template <typename T> struct Frag;
template <> struct Frag<bf16_t> {
    bf16x8_t v;
    __device__ __forceinline__ void load(const bf16_t* p) { v = *(const bf16x8_t*)p; }
    __device__ __forceinline__ void zero() { v = bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0}; }
};
template <> struct Frag<f16_t> {
    bf16x8_t v;                                                 // raw fp16 bits
    __device__ __forceinline__ void load(const f16_t* p) { v = *(const bf16x8_t*)p; }
    __device__ __forceinline__ void zero() { v = bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0}; }
};
template <> struct Frag<float> {
    float4 a, b;
    __device__ __forceinline__ void load(const float* p) { a = *(const float4*)p; b = *(const float4*)(p + 4); }
    __device__ __forceinline__ void load(const bf16_t* p) {      // bf16 activations, fp32 ("precise") math
        const u32x4_t q = *(const u32x4_t*)p;
        a = make_float4(__uint_as_float(q[0] << 16), __uint_as_float(q[0] & 0xffff0000u),
                        __uint_as_float(q[1] << 16), __uint_as_float(q[1] & 0xffff0000u));
        b = make_float4(__uint_as_float(q[2] << 16), __uint_as_float(q[2] & 0xffff0000u),
                        __uint_as_float(q[3] << 16), __uint_as_float(q[3] & 0xffff0000u));
    }
    __device__ __forceinline__ void load(const f16_t* p) {       // fp16 activations, fp32 ("precise") math
        const u32x4_t q = *(const u32x4_t*)p;
        a = make_float4(H16<f16_t>::lo(q[0]), H16<f16_t>::hi(q[0]), H16<f16_t>::lo(q[1]), H16<f16_t>::hi(q[1]));
        b = make_float4(H16<f16_t>::lo(q[2]), H16<f16_t>::hi(q[2]), H16<f16_t>::lo(q[3]), H16<f16_t>::hi(q[3]));
    }
    __device__ __forceinline__ void zero() { a = make_float4(0, 0, 0, 0); b = a; }
};

__device__ __forceinline__ f32x4_t mma(const Frag<bf16_t>& A, const Frag<bf16_t>& B, f32x4_t c) {
    typedef __attribute__((ext_vector_type(8))) __bf16 bfv;
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bfv, A.v), __builtin_bit_cast(bfv, B.v), c,
                                                   0, 0, 0);
}
__device__ __forceinline__ f32x4_t mma(const Frag<f16_t>& A, const Frag<f16_t>& B, f32x4_t c) {
    typedef __attribute__((ext_vector_type(8))) _Float16 hv;
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(hv, A.v), __builtin_bit_cast(hv, B.v), c, 0, 0, 0);
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


// ReLU of two packed 16-bit floats (bf16 or fp16) on their bit patterns: a signed 16-bit max with 0 zeroes every
// negative value and -0, so relu16x2(pack(x)) == pack(max(x, 0)) bitwise
__device__ __forceinline__ unsigned relu16x2(unsigned v) {
    typedef short s16x2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(unsigned, __builtin_elementwise_max(__builtin_bit_cast(s16x2, v), s16x2{0, 0}));
}
__device__ __forceinline__ int halo_phys(int p, int g) { return 2 * (g & 1) + ((g >> 1) ^ ((p >> 2) & 1)); }


// tile of block b's round i (blocks b < ntiles % nb take one round more): a full round of 256 tiles goes to the
// 256 blocks so that XCD b % 8 takes 32 consecutive tiles; a partial last round in block order (its tiles exist
// only for b < ntiles % nb -- applied to it, the XCD order addressed tiles past the last frame)
__host__ __device__ __forceinline__ int rb_tile(int i, int b, int nb, int ntiles) {
    if (nb == 256 && (i + 1) * 256 <= ntiles) return i * 256 + (b & 7) * 32 + (b >> 3);
    return i * nb + b;
}


// every (block, round) of a launch maps to a distinct tile below ntiles (checked on the host before each launch)
inline bool rb_mapping_ok(int nb, int ntiles) {
    std::vector<unsigned char> seen(ntiles, 0);
    for (int b = 0; b < nb; ++b) {
        const int my = ntiles / nb + (b < ntiles % nb ? 1 : 0);
        for (int i = 0; i < my; ++i) {
            const int t = rb_tile(i, b, nb, ntiles);
            if (t < 0 || t >= ntiles || seen[t]) return false;
            seen[t] = 1;
        }
    }
    return true;
}

// launch of the fused 64-channel ResBlock (resblock64.hip): grid = min(cap or CUs, tiles) persistent blocks
int resblock64_launch(const ConvK& k1, const ConvK& k2, int n_frames, bool f16, int max_blocks, int cus,
                      hipStream_t s);
namespace rb64 {
constexpr int TW = 16, TH = 8;                                // output tile (frames must be multiples)
}  // namespace rb64

// launch of the K-split weight-stationary 128 -> 128 conv (conv128.hip); epi: the pipelined kernel's epilogue codes
// (0 run-time act / residual / post-act, 1 bias + ReLU, 2 bias + residual then ReLU, 3 bias, 5 as 0 + the gate)
int ks128_launch(const ConvK& k, int n_frames, bool f16, int epi, int max_blocks, int cus, hipStream_t s);
namespace ks128 {
constexpr int TW = 16, TH = 8;                                // output tile (frames must be multiples)
}  // namespace ks128

}  // namespace dbsr
