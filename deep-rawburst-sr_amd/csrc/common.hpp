// Shared device helpers for the gfx950 DBSR kernels.
#pragma once
#include <type_traits>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/dbsr_hip.h"

namespace dbsr {

typedef uint16_t bf16_t;                                            // bf16 storage type
typedef _Float16 f16_t;                                             // fp16 storage type (configs[4])
typedef __attribute__((ext_vector_type(8))) short bf16x8_t;        // MFMA 16-bit operand (8 elems, raw bits)
typedef __attribute__((ext_vector_type(4))) float f32x4_t;          // 16x16 MFMA accumulator
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2_t;

// The LDS-DMA-staged MFMA conv kernels (pipelined, weight-stationary, two-barrier tiled) claim the whole VGPR
// file of their SIMDs (v255 marked live -> 256 VGPRs per wave; their 2 waves per SIMD then fill its 512), so no
// wave of another kernel is ever co-resident with them.  This is a WORKAROUND FOR AN UNEXPLAINED RACE, not a
// fix ('The two-lane race'): with another stream's kernels sharing their CUs, waves of those kernels
// computed wrong values from correct inputs (an instrumented PWC backwarp wave read the right flow and
// produced a wrong bilinear mass); exclusive SIMDs remove it.  Ruled out so far: stray writes, kernargs,
// stream order, split-K workspace aliasing, and -- by the static ISA audit of the shipped code objects
// (tools/isa_audit.py, tests/test_capi.py) -- under-declared VGPR/AGPR counts, LDS-DMA without M0 set in the
// same basic block, and LDS use beyond the declared group segment.  The audit also fails any future LDS-DMA
// kernel that does not claim its SIMDs.  Costs nothing at 2 waves per SIMD (their occupancy is already 2).
#ifndef DBSR_NO_OWN_SIMDS
#define DBSR_OWN_SIMDS() asm volatile("" ::: "v255")
#else
#define DBSR_OWN_SIMDS() do { } while (0)     // (experiment build: LDS-DMA kernels may share their SIMDs)
#endif

// Barrier after LDS-DMA (buffer/global_load ... lds): every wave first drains its own vector-memory queue, so
// the pieces it DMA'd have landed before any wave reads them.  __syncthreads() alone does not guarantee this:
// its workgroup fence needs no vmcnt(0), and the s_waitcnt the compiler puts before a barrier is sized for
// the LDS reads of THIS wave that it can see alias the DMA (tools/isa_audit.py checks every barrier).
// The wait is the s_waitcnt builtin rather than inline asm so that the compiler's own wait insertion knows
// the queue is empty afterwards (it does not read inline asm) and emits no conservative waits later on.
__device__ __forceinline__ void vm_drain() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0x0F70);           // vmcnt(0), expcnt / lgkmcnt unconstrained (gfx9 encoding)
    asm volatile("" ::: "memory");
}
__device__ __forceinline__ void dma_barrier() {
    vm_drain();
    __syncthreads();
}
// s_waitcnt vmcnt(n), n < 64 (gfx9 encoding: vmcnt bits [3:0] and [15:14])
#define DBSR_VM_WAIT(n) do { asm volatile("" ::: "memory"); \
    __builtin_amdgcn_s_waitcnt(0x0F70 | ((n) & 15) | (((n) >> 4) << 14)); asm volatile("" ::: "memory"); } while (0)

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((unsigned)v) << 16); }

// fp32 -> bf16, round-to-nearest-even, NaN kept NaN: the plain cast lowers to the hardware
// v_cvt_pk_bf16_f32 (MI355X_MICROARCH.md correctness table), one VALU op per two values instead of
// the ~7-op integer rounding sequence (which made the warp kernel VALU-bound)
typedef __attribute__((ext_vector_type(2))) float f32x2_t;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
__device__ __forceinline__ unsigned pack_bf16x2(float lo, float hi) {
    return __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2_t{lo, hi}, bf16x2_t));
}
__device__ __forceinline__ bf16_t f2bf(float f) { return __builtin_bit_cast(unsigned short, (__bf16)f); }
typedef __attribute__((ext_vector_type(2))) _Float16 f16x2_t;

// Two 16-bit values per dword (bf16 or fp16 storage): unpack to fp32 / pack from fp32 (round to nearest
// even, hardware v_cvt_pk_* conversions)
template <typename T> struct H16;
template <> struct H16<bf16_t> {
    static __device__ __forceinline__ float lo(unsigned u) { return __uint_as_float(u << 16); }
    static __device__ __forceinline__ float hi(unsigned u) { return __uint_as_float(u & 0xffff0000u); }
    static __device__ __forceinline__ unsigned pack(float a, float b) { return pack_bf16x2(a, b); }
};
template <> struct H16<f16_t> {
    static __device__ __forceinline__ float lo(unsigned u) { return (float)__builtin_bit_cast(f16x2_t, u)[0]; }
    static __device__ __forceinline__ float hi(unsigned u) { return (float)__builtin_bit_cast(f16x2_t, u)[1]; }
    static __device__ __forceinline__ unsigned pack(float a, float b) {
        return __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2_t{a, b}, f16x2_t));
    }
};

template <typename T> struct elem;
template <> struct elem<float> {
    static __device__ __forceinline__ float ld(const float* p) { return *p; }
    static __device__ __forceinline__ void st(float* p, float v) { *p = v; }
};
template <> struct elem<f16_t> {
    static __device__ __forceinline__ float ld(const f16_t* p) { return (float)*p; }
    static __device__ __forceinline__ void st(f16_t* p, float v) { *p = (f16_t)v; }
};
template <> struct elem<bf16_t> {
    static __device__ __forceinline__ float ld(const bf16_t* p) { return bf2f(*p); }
    static __device__ __forceinline__ void st(bf16_t* p, float v) { *p = f2bf(v); }
};

// load 8 consecutive elements as fp32
__device__ __forceinline__ void load8(const float* p, float (&v)[8]) {
    float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
template <typename T>
__device__ __forceinline__ void load8(const T* p, float (&v)[8]) {      // 16-bit storage (bf16 / fp16)
    u32x4_t q = *(const u32x4_t*)p;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        v[2 * i] = H16<T>::lo(q[i]);
        v[2 * i + 1] = H16<T>::hi(q[i]);
    }
}
__device__ __forceinline__ void store8(float* p, const float (&v)[8]) {
    *(float4*)p = make_float4(v[0], v[1], v[2], v[3]);
    *(float4*)(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}
template <typename T>
__device__ __forceinline__ void store8(T* p, const float (&v)[8]) {     // 16-bit storage (bf16 / fp16)
    u32x4_t q;
#pragma unroll
    for (int i = 0; i < 4; ++i) q[i] = H16<T>::pack(v[2 * i], v[2 * i + 1]);
    *(u32x4_t*)p = q;
}

__device__ __forceinline__ long long map_frame(const dbsr_frame_map& m, int f) {
    return (long long)(f / m.fpg) * m.group_stride + m.group_offset + (long long)(f % m.fpg) * m.inner_stride;
}

template <typename T>
__device__ __forceinline__ T* img_ptr(const dbsr_tensor& t, int f) {
    return (T*)t.ptr + map_frame(t.map, f) * t.img_stride + t.c0;
}

__device__ __forceinline__ float apply_act(float v, int act) {
    if (act == DBSR_ACT_RELU) return v > 0.f ? v : 0.f;
    if (act == DBSR_ACT_LRELU) return v > 0.f ? v : 0.1f * v;
    return v;
}

// Buffer-resource LDS-DMA (buffer_load_dwordx4 ... lds): a lane whose byte offset lies past the
// resource's num_records gets zeros written to LDS, so halo pixels outside the frame need neither a
// zero page nor a per-lane pointer select; soffset carries the wave-uniform part of the address.
constexpr int BUF_OOB = (int)0x80000000u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, unsigned bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ void blds16(__amdgpu_buffer_rsrc_t r, int voff, int soff, u32x4_t* lds_piece) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_piece, 16, voff, soff, 0, 0);
}

// 3x3 Gaussian blur (upsampling.py:24-29, 59-65) as a separable pair -- the reference's kernel is the normalised
// outer product of a 1-D Gaussian -- horizontal taps kh, vertical taps kv.  Every blur kernel of the library sums
// in this order (blur_row, then blur_col), so their outputs are bitwise equal to one another.
struct Blur3 {
    float kh[3], kv[3];
};
// k9 (row-major 3x3) -> kh = its middle row, kv = its middle column / k[4]; false unless k9 = kv kh^T to 1e-6
inline bool blur_separable(const float* k9, Blur3& b) {
    if (!(k9[4] > 0.f)) return false;
    float mx = 0.f;
    for (int i = 0; i < 9; ++i) mx = k9[i] > mx ? k9[i] : (-k9[i] > mx ? -k9[i] : mx);
    for (int j = 0; j < 3; ++j) b.kh[j] = k9[3 + j];
    for (int i = 0; i < 3; ++i) b.kv[i] = k9[3 * i + 1] / k9[4];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            const float d = k9[3 * i + j] - b.kv[i] * b.kh[j];
            if (d > 1e-6f * mx || -d > 1e-6f * mx) return false;
        }
    return true;
}
// horizontal pass over one row of 8 channels: x0, x1, x2 = columns -1, 0, +1 (16-bit, raw).  Channel pairs run as
// packed fp32 ops (v_pk_mul_f32 / v_pk_fma_f32: each component is the scalar mul / fma, so the sums are bitwise the
// scalar ones) -- half the VALU issue of the blur, which bounds the fused upsampler
template <typename T>
__device__ __forceinline__ void blur_row(const Blur3& b, const u32x4_t& x0, const u32x4_t& x1, const u32x4_t& x2,
                                         float (&h)[8]) {
    const f32x2_t k0 = {b.kh[0], b.kh[0]}, k1 = {b.kh[1], b.kh[1]}, k2 = {b.kh[2], b.kh[2]};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const f32x2_t v0 = {H16<T>::lo(x0[q]), H16<T>::hi(x0[q])};
        const f32x2_t v1 = {H16<T>::lo(x1[q]), H16<T>::hi(x1[q])};
        const f32x2_t v2 = {H16<T>::lo(x2[q]), H16<T>::hi(x2[q])};
        const f32x2_t r = __builtin_elementwise_fma(k2, v2, __builtin_elementwise_fma(k1, v1, k0 * v0));
        h[2 * q] = r.x;
        h[2 * q + 1] = r.y;
    }
}
// vertical pass: rows -1, 0, +1 of horizontal sums
__device__ __forceinline__ void blur_col(const Blur3& b, const float (&h0)[8], const float (&h1)[8], const float (&h2)[8],
                                         float (&o)[8]) {
    const f32x2_t k0 = {b.kv[0], b.kv[0]}, k1 = {b.kv[1], b.kv[1]}, k2 = {b.kv[2], b.kv[2]};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const f32x2_t a0 = {h0[2 * q], h0[2 * q + 1]}, a1 = {h1[2 * q], h1[2 * q + 1]}, a2 = {h2[2 * q], h2[2 * q + 1]};
        const f32x2_t r = __builtin_elementwise_fma(k2, a2, __builtin_elementwise_fma(k1, a1, k0 * a0));
        o[2 * q] = r.x;
        o[2 * q + 1] = r.y;
    }
}

// compile-time loop: f(std::integral_constant<int, I>) for I in [I0, I1) (register arrays indexed by I stay
// in registers whatever the unroller decides)
template <int I0, int I1>
struct StaticFor {
    template <class F>
    __device__ __forceinline__ static void run(F&& f) {
        if constexpr (I0 < I1) {
            f(std::integral_constant<int, I0>{});
            StaticFor<I0 + 1, I1>::run(f);
        }
    }
};

// One 1-KiB LDS-DMA piece issued from inline asm (as conv_wgrad_dma_kernel does): the compiler's wait insertion
// does not see it, so it neither drains every outstanding piece before the fragment reads (it cannot tell the
// ring stage being read from the stages being filled) nor at every __syncthreads; the kernel counts its own
// pieces (vmcnt is in order, so the compiler's own waits only get stricter).  rsrc words: base, stride 0,
// num_records, raw-buffer flags.
__device__ __forceinline__ void lds_dma16(const void* base, unsigned bytes, int voff, int soff, unsigned lds_addr) {
    const unsigned long long a = (unsigned long long)base;
    typedef int i32x4_t __attribute__((ext_vector_type(4)));
    const i32x4_t r = {(int)(unsigned)a, (int)((unsigned)(a >> 32) & 0xffffu), (int)bytes, 0x00020000};
    asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dwordx4 %0, %1, %3 offen lds" ::"v"(voff), "s"(r), "s"(lds_addr),
                 "s"(soff)
                 : "memory", "m0");
}

}  // namespace dbsr

// ---------------- host-side helpers ----------------
void dbsr_set_error(const char* fmt, ...);
#define DBSR_CHECK_ARG(cond, ...)                 \
    do {                                          \
        if (!(cond)) {                            \
            dbsr_set_error(__VA_ARGS__);          \
            return DBSR_E_ARG;                    \
        }                                         \
    } while (0)
#define DBSR_LAUNCH_CHECK()                                               \
    do {                                                                  \
        hipError_t e_ = hipGetLastError();                                \
        if (e_ != hipSuccess) {                                           \
            dbsr_set_error("HIP launch error: %s", hipGetErrorString(e_)); \
            return (int)e_;                                               \
        }                                                                 \
    } while (0)
