// Backward-pass and optimizer kernels for the DBSR training step (BASELINE configs[3]; SURVEY §8e/§8f
// rank 3).  The reference trains with autograd over cuDNN/ATen (trainers/simple_trainer.py:78-81,
// actors/dbsr_actors.py:27-47): L1 loss on the boundary-cropped prediction, loss.backward(), Adam.
// Here every backward op is a hand-written HIP kernel; conv dgrad reuses the forward implicit-GEMM conv
// (dbsr_conv2d with dgrad-packed weights and the gate epilogue), conv wgrad is the MFMA kernel below.
// All activations NHWC (dbsr_hip.h); gradients of trainable parameters are fp32 in torch layout.
#include "common.hpp"

#include <algorithm>
#include <type_traits>

using namespace dbsr;

namespace {

inline unsigned nblocks(long long total, int bs) { return (unsigned)((total + bs - 1) / bs); }
bool map_ok(const dbsr_tensor& t) { return t.ptr && t.map.fpg > 0; }
__host__ __device__ inline bool vec_ok(const dbsr_tensor& t, int v) { return t.ld % v == 0 && t.c0 % v == 0; }

template <typename F>
int by_dtype(int dtype, F&& f) {
    if (dtype == DBSR_BF16) return f((bf16_t*)nullptr);
    if (dtype == DBSR_F16) return f((f16_t*)nullptr);
    if (dtype == DBSR_F32) return f((float*)nullptr);
    dbsr_set_error("unsupported dtype %d", dtype);
    return DBSR_E_ARG;
}

// ------------------------------------------------------------------------------------------------
// Conv weight gradient (nn.Conv2d backward w.r.t. weight, k = 1 or 3, stride 1, pad k/2):
//   dW[co][ci][ky][kx] = sum over pixels p of dY[p][co] * X[p + (ky-1, kx-1)][ci]
// a GEMM whose reduction axis is the pixel.  Work unit: a tile of 8 rows x 16 columns of one frame
// (128 output pixels = 4 MFMA k-steps of 32).  A block owns a 64-cout x 64-cin slice and a contiguous
// range of tiles; per tile it stages dY [128 px][64 co] and the (10 x 18)-pixel X halo [180 px][64 ci]
// in LDS (rows of 64 channels, 16-B loads, zeros outside the frame / channel range), then
//   3x3: wave t (9 waves) accumulates tap t: B rows are the halo pixels shifted by the tap;
//   1x1: wave w (4 waves) accumulates k-step w of every tile.
// bf16 MFMA 16x16x32 takes 8 consecutive pixels per lane for one channel: both operands are read from
// the pixel-major tiles with the gfx950 transposed LDS read ds_read_b64_tr_b16 (two 4-row reads per
// operand; cdna_hip_programming.md T10).  fp32 runs v_mfma_f32_16x16x4_f32 on plain reads (one pixel
// per lane per MFMA).  Each wave's 64x64 accumulator block is written to its own fp32 partial slot
// [block][wave][co][ci]; wgrad_reduce sums the slots in a fixed order (deterministic).
// 1x1 stages the X tile itself (no halo).  The conv's bias gradient db[co] = sum over pixels of dY[co] rides
// along in the ci-block-0 blocks (bpart != NULL): every thread's dY pieces are one fixed 16-B channel group,
// summed in fp32 as they go to the LDS, then reduced per block into bpart[block][cout] (fixed order).
// ------------------------------------------------------------------------------------------------
constexpr int WG_TH = 8, WG_TW = 16, WG_PX = WG_TH * WG_TW;             // output tile
// blocks over all (co, ci) tiles, each one fp32 partial slot: one per CU for 64-channel blocks (160+ VGPRs x 9
// waves), two for 32-channel blocks (97 VGPRs)
inline int wg_blocks(int cb) { return cb == 32 ? 512 : 256; }
constexpr int WG_HH = WG_TH + 2, WG_HW = WG_TW + 2, WG_HPX = WG_HH * WG_HW;   // halo

// a pixel row of CB channels in the LDS: CB elements + 16 B skew
template <typename T, int CB> struct WgCfg { static constexpr int ROWB = CB * (int)sizeof(T) + 16; };

typedef short v4s_t __attribute__((ext_vector_type(4)));
struct FragB { bf16x8_t v; };
template <typename T>
__device__ __forceinline__ f32x4_t mma16(const FragB& a, const FragB& b, f32x4_t c) {
    if constexpr (std::is_same_v<T, f16_t>) {
        typedef __attribute__((ext_vector_type(8))) _Float16 hv;
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(hv, a.v), __builtin_bit_cast(hv, b.v), c, 0, 0, 0);
    } else {
        typedef __attribute__((ext_vector_type(8))) __bf16 bfv;
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bfv, a.v), __builtin_bit_cast(bfv, b.v), c, 0, 0, 0);
    }
}

__device__ __forceinline__ v4s_t tr16(const unsigned char* lds_byte) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s_t*)lds_byte);
}

// CB: the (co, ci) block edge, 64 or 32 (32: the 32-channel convs, whose few MFMAs per tile leave the loop
// latency-bound -- two tiles are prefetched and the smaller accumulator set leaves room for them)
template <typename T, int K, int CB>
__global__ __launch_bounds__(K == 3 ? 576 : 256) void conv_wgrad_kernel(
        int n_frames, int h, int w, dbsr_tensor x, int cin, dbsr_tensor dy, int cout, long long n_units,
        float* __restrict__ partial, float* __restrict__ bpart) {
    constexpr int NW = K == 3 ? 9 : 4;
    constexpr int NB = CB / 16;                        // 16-channel MFMA blocks per edge
    constexpr int ROWB = WgCfg<T, CB>::ROWB;
    constexpr int XW = K == 3 ? WG_HW : WG_TW;         // X tile: the 3x3 halo, or the output tile itself
    constexpr int XPX = K == 3 ? WG_HPX : WG_PX;
    __shared__ __attribute__((aligned(16))) unsigned char lds[(WG_PX + XPX) * ROWB];
    unsigned char* ldy = lds;                          // [128 px][CB co]
    unsigned char* lx = lds + WG_PX * ROWB;            // [XPX px][CB ci]
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int co0 = blockIdx.y * CB, ci0 = blockIdx.z * CB;
    const int tiles_x = (w + WG_TW - 1) / WG_TW, tiles_y = (h + WG_TH - 1) / WG_TH;
    const long long u0 = n_units * blockIdx.x / gridDim.x, u1 = n_units * (blockIdx.x + 1) / gridDim.x;
    const int ky = K == 3 ? wave / 3 : 0, kx = K == 3 ? wave % 3 : 0;   // 1x1: the tile itself
    f32x4_t acc[NB][NB];
#pragma unroll
    for (int i = 0; i < NB; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    constexpr int EPP = 16 / (int)sizeof(T);           // elements per 16-B piece
    constexpr int PPR = CB / EPP;                      // pieces per CB-channel row
    constexpr int PIECES = (WG_PX + XPX) * PPR;
    constexpr int PT = (PIECES + NW * 64 - 1) / (NW * 64);   // pieces per thread per tile
    static_assert((NW * 64) % PPR == 0, "a thread's dY pieces must be one channel group");
    static_assert(NW * 64 * EPP * 4 <= (WG_PX + XPX) * ROWB, "bias reduction must fit the LDS tile");
    const bool do_bias = bpart != nullptr && blockIdx.z == 0;   // block-uniform
    float bs[EPP];
#pragma unroll
    for (int e = 0; e < EPP; ++e) bs[e] = 0.f;
    // the next tile's dY / X pieces are loaded into registers while this tile's MFMAs run (software pipeline),
    // then written to the LDS after the barrier that ends them
    constexpr int DIST = CB == 32 ? 2 : 1;             // prefetch distance in tiles (register budget)
    u32x4_t pre[DIST][PT];
    auto fetch = [&](long long u, u32x4_t (&dst)[PT]) {
        const int tx = (int)(u % tiles_x);
        const long long r = u / tiles_x;
        const int ty = (int)(r % tiles_y);
        const int f = (int)(r / tiles_y);
        const int y0 = ty * WG_TH, x0 = tx * WG_TW;
        const T* dyf = img_ptr<T>(dy, f);
        const T* xf = img_ptr<T>(x, f);
#pragma unroll
        for (int k = 0; k < PT; ++k) {
            const int it = threadIdx.x + k * NW * 64;
            const int row = it / PPR, pc = it % PPR;
            u32x4_t v = {0u, 0u, 0u, 0u};
            if (row < WG_PX) {
                const int yy = y0 + row / WG_TW, xx = x0 + row % WG_TW, c = co0 + pc * EPP;
                if (yy < h && xx < w && c < cout) v = *(const u32x4_t*)(dyf + ((long long)yy * w + xx) * dy.ld + c);
            } else if (it < PIECES) {
                const int hr = row - WG_PX, o = K == 3 ? 1 : 0;
                const int yy = y0 - o + hr / XW, xx = x0 - o + hr % XW, c = ci0 + pc * EPP;
                if ((unsigned)yy < (unsigned)h && (unsigned)xx < (unsigned)w && c < cin)
                    v = *(const u32x4_t*)(xf + ((long long)yy * w + xx) * x.ld + c);
            }
            dst[k] = v;
        }
    };
    auto put = [&](const u32x4_t (&src)[PT]) {
#pragma unroll
        for (int k = 0; k < PT; ++k) {
            const int it = threadIdx.x + k * NW * 64;
            if (it >= PIECES) break;
            const int row = it / PPR, pc = it % PPR;
            *(u32x4_t*)(lds + row * ROWB + pc * 16) = src[k];   // ldy rows, then the lx rows right after them
            if (do_bias && row < WG_PX) {
                if constexpr (sizeof(T) == 2) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        bs[2 * q] += H16<T>::lo(src[k][q]);
                        bs[2 * q + 1] += H16<T>::hi(src[k][q]);
                    }
                } else {
#pragma unroll
                    for (int q = 0; q < 4; ++q) bs[q] += __uint_as_float(src[k][q]);
                }
            }
        }
    };
    // every 16-channel block of the slice is computed (blocks past cout / cin multiply the zeros the staging
    // loads there), so the MFMAs issue back to back
    auto compute = [&]() {
        // ---- MFMAs ---- (k-steps not unrolled: one k-step's fragments live at a time)
#pragma unroll 1
        for (int s = 0; s < 4; ++s) {
            if (K == 1 && s != wave) continue;
            if constexpr (sizeof(T) == 2) {
                // lane (g = lane>>4, q = (lane>>2)&3, p = lane&3): rows k = 8g+q (+4) of this k-step,
                // channels 4p..4p+3 of each 16-channel block
                const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
                FragB a[NB], b[NB];
#pragma unroll
                for (int half = 0; half < 2; ++half) {
                    const int kk = 8 * g + 4 * half + q;             // pixel of the k-step, 0..31
                    const int ty_ = 2 * s + kk / 16, tx_ = kk % 16;
                    const unsigned char* arow = ldy + (ty_ * WG_TW + tx_) * ROWB;
                    const unsigned char* brow = lx + ((ty_ + ky) * XW + tx_ + kx) * ROWB;
#pragma unroll
                    for (int i = 0; i < NB; ++i) {
                        const v4s_t va = tr16(arow + (i * 16 + 4 * p) * 2);
                        const v4s_t vb = tr16(brow + (i * 16 + 4 * p) * 2);
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            a[i].v[4 * half + e] = va[e];
                            b[i].v[4 * half + e] = vb[e];
                        }
                    }
                }
#pragma unroll
                for (int i = 0; i < NB; ++i)
#pragma unroll
                    for (int j = 0; j < NB; ++j)
                        acc[i][j] = mma16<T>(a[i], b[j], acc[i][j]);
            } else {
                // fp32: 8 MFMAs of k = 4 pixels; lane (kq = lane>>4, m = lane&15)
                const int kq = lane >> 4, m = lane & 15;
#pragma unroll
                for (int k4 = 0; k4 < 8; ++k4) {
                    const int kk = k4 * 4 + kq;
                    const int ty_ = 2 * s + kk / 16, tx_ = kk % 16;
                    const float* arow = (const float*)(ldy + (ty_ * WG_TW + tx_) * ROWB);
                    const float* brow = (const float*)(lx + ((ty_ + ky) * XW + tx_ + kx) * ROWB);
                    float av[NB], bv[NB];
#pragma unroll
                    for (int i = 0; i < NB; ++i) {
                        av[i] = arow[i * 16 + m];
                        bv[i] = brow[i * 16 + m];
                    }
#pragma unroll
                    for (int i = 0; i < NB; ++i)
#pragma unroll
                        for (int j = 0; j < NB; ++j)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[j], acc[i][j], 0, 0, 0);
                }
            }
        }
    };
#pragma unroll
    for (int d = 0; d < DIST; ++d)
        if (u0 + d < u1) fetch(u0 + d, pre[d]);
    for (long long u = u0; u < u1; u += DIST) {
#pragma unroll
        for (int d = 0; d < DIST; ++d) {
            if (u + d >= u1) break;
            put(pre[d]);
            __syncthreads();
            if (u + d + DIST < u1) fetch(u + d + DIST, pre[d]);
            compute();
            __syncthreads();
        }
    }
    if (do_bias) {
        // the loop's last barrier has freed the LDS: thread t's EPP sums of channel group t % PPR, then channel c
        // adds the threads of its group in thread order
        float* red = (float*)lds;
#pragma unroll
        for (int e = 0; e < EPP; ++e) red[threadIdx.x * EPP + e] = bs[e];
        __syncthreads();
        if ((int)threadIdx.x < CB && co0 + (int)threadIdx.x < cout) {
            const int c = threadIdx.x, g = c / EPP, e = c % EPP;
            float t = 0.f;
            for (int th = g; th < NW * 64; th += PPR) t += red[th * EPP + e];
            bpart[(long long)blockIdx.x * cout + co0 + c] = t;
        }
    }
    // ---- this wave's partial: C[m = co][n = ci], lane holds co 4(lane>>4)+r of block i, ci lane&15 of block j
    float* out = partial + ((long long)blockIdx.x * gridDim.y * gridDim.z + blockIdx.y * gridDim.z + blockIdx.z) *
                               (NW * CB * CB) + wave * CB * CB;
#pragma unroll
    for (int i = 0; i < NB; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                out[(i * 16 + 4 * (lane >> 4) + r) * CB + j * 16 + (lane & 15)] = acc[i][j][r];
}

// 16-bit wgrad with LDS-DMA staging (conv_wgrad_kernel above stays for fp32): the same work split and partial
// slots, but the dY tile and the X tile go global -> LDS by buffer_load ... lds into a 3-stage ring, two tiles
// ahead, with one barrier per tile (conv_wgrad_kernel's register staging leaves one tile of compute to hide
// each tile's load latency, and two barriers).  LDS rows of CB channels are unpadded and the 3x3 halo rows sit
// at a pitch of XP = 24 pixels; each row's 16-B chunks are XOR-swizzled by a key taken
// from row bits (0, 1, 3) (CB 64) / 3 (CB 32), which makes a lane's key the same for every k-step (and,
// for the halo, depend only on the half), so the fragment addresses are per-lane bases plus immediates, and
// the transposed reads (16 rows x 32 B) stay at the 2-cycle minimum.  A tile's barrier is passed with the next
// tile's DMAs in flight: they target the ring stage after this one, and the stage the DMAs issued after the
// barrier overwrite was last read before it (tools/isa_audit.py: RING_KERNELS).
// The bias gradient rides along in the ci-block-0 blocks: the tap-5 wave (3x3; a SIMD with two waves) or every
// wave (1x1) also sums its dY fragments (lane: 8 pixels of one channel) in fp32, db[co] = sum over pixels of
// dY[co]; the four lanes of a channel and the bias waves are added in a fixed order at the end.
template <int K, int CB> struct WgdCfg {
    static constexpr int NW = K == 3 ? 9 : 4;
    static constexpr int RB = CB * 2;                    // row bytes
    static constexpr int CPR = RB / 16;                  // 16-B chunks per row
    static constexpr int XP = K == 3 ? 24 : WG_TW;      // X row pitch (pixels)
    static constexpr int XROWS = K == 3 ? WG_HH * XP : WG_PX;          // X rows in the LDS
    static constexpr int DY_PIECES = WG_PX * CPR / 64;   // the dY rows fill whole 1-KiB pieces
    static constexpr int PIECES = ((WG_PX + XROWS) * CPR + 63) / 64;
    static constexpr int PER = (PIECES + NW - 1) / NW;   // pieces per wave per tile (surplus: re-issue the last)
    static constexpr int STAGE_U4 = PIECES * 64;
    static_assert(WG_PX * CPR % 64 == 0, "dY rows must fill whole pieces");
    static_assert(PER < 16, "vmcnt immediate");
    static_assert(3 * STAGE_U4 * 16 <= 160 * 1024, "ring must fit the LDS");
};
// One 1-KiB LDS-DMA piece issued from inline asm: the compiler's wait insertion does not see it, so it neither
// drains the ring before every fragment read (it cannot tell the stage being read from the stage being filled)
// nor at every barrier; the kernel counts its own DMAs (vmcnt is in order, so the compiler's own waits only get
// stricter).  rsrc: the buffer resource words (base, stride 0, num_records, raw-buffer flags).
__device__ __forceinline__ void wgd_dma(const void* base, unsigned bytes, int voff, unsigned lds_addr) {
    const unsigned long long a = (unsigned long long)base;
    typedef int i32x4_t __attribute__((ext_vector_type(4)));
    const i32x4_t r = {(int)(unsigned)a, (int)((unsigned)(a >> 32) & 0xffffu), (int)bytes, 0x00020000};
    asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(r), "s"(lds_addr)
                 : "memory", "m0");
}
// CB 32: a 64-B row is a quarter of the 64 banks, so the rows x + q and x + 8 + q that one 32-lane half of a
// transposed read takes (lane groups g, g + 1) share a bank quarter: their 32-B windows must sit in opposite
// halves of the row -- key bit 1 (the window) is row bit 3, which no k-step's row step (32 for dY, 2 x 24 for X)
// changes.  (The earlier key, row bits 4, 3, put both windows in one half: a 2-way conflict on every A and B
// read, SQ_LDS_BANK_CONFLICT = half of SQ_LDS_IDX_ACTIVE at the decoder's 32-channel wgrads, r06 PMC; it also
// needed an X pitch of 32 pixels, whose 84-KB ring let only one of the two blocks per CU in at a time.)
template <int CB> __device__ __forceinline__ int wgd_swz(int row) {
    return CB == 64 ? ((row & 3) | (((row >> 3) & 1) << 2)) : (((row >> 3) & 1) << 1);
}

template <typename T, int K, int CB>
__global__ __launch_bounds__(K == 3 ? 576 : 256) void conv_wgrad_dma_kernel(
        int n_frames, int h, int w, dbsr_tensor x, int cin, dbsr_tensor dy, int cout, long long n_units,
        float* __restrict__ partial, float* __restrict__ bpart) {
    using C = WgdCfg<K, CB>;
    constexpr int NW = C::NW, NB = CB / 16, RB = C::RB;
    __shared__ __attribute__((aligned(16))) u32x4_t lds[3 * C::STAGE_U4];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int co0 = blockIdx.y * CB, ci0 = blockIdx.z * CB;
    const int tiles_x = (w + WG_TW - 1) / WG_TW, tiles_y = (h + WG_TH - 1) / WG_TH;
    const long long u0 = n_units * blockIdx.x / gridDim.x, u1 = n_units * (blockIdx.x + 1) / gridDim.x;
    const int ky = K == 3 ? wave / 3 : 0, kx = K == 3 ? wave % 3 : 0;
    const bool do_bias = bpart != nullptr && blockIdx.z == 0;          // block-uniform
    const bool bias_wave = do_bias && (K == 1 || wave == 5);

    // the lane's chunk of each of its pieces, relative to the tile, packed: pixel (ry + 2, rx + 2) and the
    // channel offset; a chunk of the pitch padding / past the X tile gets the channel field 0xff, which no
    // 16-bit slice reaches (CB <= 64 channels per block: c < 64), so its DMA always lands zeros
    int p_geo[C::PER];
#pragma unroll
    for (int it = 0; it < C::PER; ++it) {
        const int piece = min(wave + NW * it, C::PIECES - 1);
        const int sc = piece * 64 + lane, row = sc / C::CPR, cp = sc % C::CPR;
        int ry, rx, c;
        if (piece < C::DY_PIECES) {
            ry = row / WG_TW; rx = row % WG_TW; c = (cp ^ wgd_swz<CB>(row)) * 8;
        } else {
            const int xr = row - WG_PX, o = K == 3 ? 1 : 0;
            ry = xr / C::XP - o; rx = xr % C::XP - o; c = (cp ^ wgd_swz<CB>(xr)) * 8;
            if (xr >= C::XROWS || rx >= (K == 3 ? WG_HW - 1 : WG_TW)) c = 0xff;   // pitch padding / past the tile
        }
        p_geo[it] = ((ry + 2) << 16) | ((rx + 2) << 8) | c;
    }
    const unsigned dy_bytes = (unsigned)((long long)h * w * dy.ld * 2), x_bytes = (unsigned)((long long)h * w * x.ld * 2);
    const unsigned lds0 = (unsigned)(unsigned long long)(__attribute__((address_space(3))) u32x4_t*)lds;
    auto issue = [&](long long u, int stage) {
        // 32-bit unsigned (wave-uniform, scalar) division: the host checks n_units < 2^31
        const unsigned uu = (unsigned)u, txs = (unsigned)tiles_x, tys = (unsigned)tiles_y;
        const unsigned r = uu / txs;
        const int tx = (int)(uu - r * txs);
        const int f = (int)(r / tys), ty = (int)(r - (unsigned)f * tys);
        const int y0 = ty * WG_TH - 2, x0 = tx * WG_TW - 2;
        const T* dyf = img_ptr<T>(dy, f);
        const T* xf = img_ptr<T>(x, f);
#pragma unroll
        for (int it = 0; it < C::PER; ++it) {
            const int piece = min(wave + NW * it, C::PIECES - 1);
            const bool isdy = piece < C::DY_PIECES;                    // wave-uniform
            const int geo = p_geo[it];
            const int yy = y0 + (geo >> 16), xx = x0 + ((geo >> 8) & 0xff);
            const int c = (isdy ? co0 : ci0) + (geo & 0xff);
            const bool ok = (geo & 0xff) != 0xff && (unsigned)yy < (unsigned)h && (unsigned)xx < (unsigned)w &&
                            c < (isdy ? cout : cin);
            const int off = ok ? ((yy * w + xx) * (isdy ? dy.ld : x.ld) + c) * 2 : BUF_OOB;
            wgd_dma(isdy ? (const void*)dyf : (const void*)xf, isdy ? dy_bytes : x_bytes, off,
                    lds0 + (unsigned)((stage * C::STAGE_U4 + piece * 64) * 16));
        }
    };

    f32x4_t acc[NB][NB];
    float accb[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        accb[i] = 0.f;
#pragma unroll
        for (int j = 0; j < NB; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    }
    // lane (g, q, p): rows k = 8g + q (+4 for the second half) of a k-step, channels 4p..4p+3 of each 16-channel
    // block.  Row of k-step s, half hf: A (dY) ar0 + 32 s + 4 hf, B (X) br0 + 2 s XP + 4 hf; the swizzle keys
    // do not change with s (nor, for A, with hf)
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int ar0 = 16 * (g >> 1) + 8 * (g & 1) + q;
    const int br0 = ((g >> 1) + ky) * C::XP + 8 * (g & 1) + q + kx;
    int offa[NB], offb[2][NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const int cl = 2 * i + (p >> 1);
        offa[i] = ar0 * RB + ((cl ^ wgd_swz<CB>(ar0)) << 4) + 8 * (p & 1);
#pragma unroll
        for (int hf = 0; hf < 2; ++hf)
            offb[hf][i] = WG_PX * RB + (br0 + 4 * hf) * RB + ((cl ^ wgd_swz<CB>(br0 + 4 * hf)) << 4) + 8 * (p & 1);
    }
    // every 16-channel block of the slice is computed (blocks past cout / cin multiply the zeros their DMAs
    // land), so the MFMAs issue back to back
    auto compute = [&](const unsigned char* st) {
        // k-steps not unrolled: the fragments of one k-step live at a time (three waves per SIMD interleave)
#pragma unroll 1
        for (int s = 0; s < 4; ++s) {
            if (K == 1 && s != wave) continue;
            FragB a[NB], b[NB];
#pragma unroll
            for (int hf = 0; hf < 2; ++hf) {
#pragma unroll
                for (int i = 0; i < NB; ++i) {
                    const v4s_t va = tr16(st + offa[i] + (32 * s + 4 * hf) * RB);
                    const v4s_t vb = tr16(st + offb[hf][i] + 2 * s * C::XP * RB);
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        a[i].v[4 * hf + e] = va[e];
                        b[i].v[4 * hf + e] = vb[e];
                    }
                }
            }
#pragma unroll
            for (int i = 0; i < NB; ++i)
#pragma unroll
                for (int j = 0; j < NB; ++j)
                    acc[i][j] = mma16<T>(a[i], b[j], acc[i][j]);
            if (bias_wave) {
#pragma unroll
                for (int i = 0; i < NB; ++i) {
                    float t = 0.f;
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const unsigned u = (unsigned short)a[i].v[2 * e] | ((unsigned)(unsigned short)a[i].v[2 * e + 1] << 16);
                        t += H16<T>::lo(u) + H16<T>::hi(u);
                    }
                    accb[i] += t;
                }
            }
        }
    };

    const long long nt = u1 - u0;
    if (nt > 0) issue(u0, 0);
    if (nt > 1) issue(u0 + 1, 1);
    for (long long t = 0; t < nt; ++t) {
        // this wave's pieces of tile t landed (tile t + 1's, issued after them, may still be in flight) ...
        if (t + 1 < nt) DBSR_VM_WAIT(C::PER);
        else DBSR_VM_WAIT(0);
        __syncthreads();                // ... and everyone's; every wave is done with tile t - 1's stage
        if (t + 2 < nt) issue(u0 + t + 2, (int)((t + 2) % 3));
        compute((const unsigned char*)(lds + (int)(t % 3) * C::STAGE_U4));
    }
    float* out = partial + ((long long)blockIdx.x * gridDim.y * gridDim.z + blockIdx.y * gridDim.z + blockIdx.z) *
                               (NW * CB * CB) + wave * CB * CB;
#pragma unroll
    for (int i = 0; i < NB; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                out[(i * 16 + 4 * (lane >> 4) + r) * CB + j * 16 + (lane & 15)] = acc[i][j][r];
    if (do_bias) {
        constexpr int NBW = K == 3 ? 1 : 4;            // bias waves, summed in wave order
        DBSR_VM_WAIT(0);                // (no DMA is in flight after the last tile; explicit for the ISA audit)
        __syncthreads();                // every wave is done with the ring
        float* red = (float*)lds;       // [bias wave][lane group g][CB]
        if (bias_wave) {
            const int bw = K == 3 ? 0 : wave;
#pragma unroll
            for (int i = 0; i < NB; ++i) red[(bw * 4 + g) * CB + i * 16 + (lane & 15)] = accb[i];
        }
        __syncthreads();
        if ((int)threadIdx.x < CB && co0 + (int)threadIdx.x < cout) {
            float t = 0.f;
#pragma unroll
            for (int bw = 0; bw < NBW; ++bw)
                t += ((red[(bw * 4) * CB + threadIdx.x] + red[(bw * 4 + 1) * CB + threadIdx.x]) +
                      red[(bw * 4 + 2) * CB + threadIdx.x]) + red[(bw * 4 + 3) * CB + threadIdx.x];
            bpart[(long long)blockIdx.x * cout + co0 + threadIdx.x] = t;
        }
    }
}

// dW[co][ci][tap] (+)= sum over blocks (and, for 1x1, over the 4 waves) of the partial slots.  A block owns
// (co, tap, 64 consecutive ci) and splits the blocks bx over 4 waves (each wave's loads: 64 consecutive
// floats); the 4 wave sums are added in a fixed order (deterministic).
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(int nbx, int nty, int ntz, int nw, int taps, int cout,
                                                           int cin, int cb, const float* __restrict__ partial,
                                                           float* __restrict__ dw, int accumulate) {
    const int nci64 = (cin + 63) / 64;
    int b = blockIdx.x;
    const int cib = b % nci64;
    b /= nci64;
    const int tap = b % taps, co = b / taps;
    const int il = threadIdx.x & 63, sl = threadIdx.x >> 6;
    const int ci = cib * 64 + il;
    const int by = co / cb, cl = co % cb, bz = ci / cb, il_ = ci % cb;
    const int wsz = cb * cb;
    float s = 0.f;
    if (ci < cin) {
        const long long slot = (long long)nw * wsz;
        const float* base = partial + ((long long)by * ntz + bz) * slot + cl * cb + il_;
#pragma unroll 8
        for (int bx = sl; bx < nbx; bx += 4) {
            const float* blk = base + (long long)bx * nty * ntz * slot;
            if (taps == 1) {
                for (int wv = 0; wv < nw; ++wv) s += blk[wv * wsz];
            } else {
                s += blk[tap * wsz];
            }
        }
    }
    __shared__ float red[4][64];
    red[sl][il] = s;
    __syncthreads();
    if (sl == 0 && ci < cin) {
        const float t = ((red[0][il] + red[1][il]) + red[2][il]) + red[3][il];
        const long long idx = ((long long)co * cin + ci) * taps + tap;
        dw[idx] = accumulate ? dw[idx] + t : t;
    }
}

// ------------------------------------------------------------------------------------------------
// Per-channel sum over all pixels (conv bias gradient, db[c] = sum_p dY[p][c]): block = (64 channels,
// pixel range), partials [nblk][c], reduced in block order.
// ------------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void chan_sum_kernel(int n, int hw, int c, dbsr_tensor t, int px_per_block,
                                                       float* __restrict__ partial) {
    const int cl = threadIdx.x & 63, sub = threadIdx.x >> 6;
    const int ch = blockIdx.y * 64 + cl;
    const long long total = (long long)n * hw;
    const long long p0 = (long long)blockIdx.x * px_per_block, p1 = std::min<long long>(p0 + px_per_block, total);
    float s = 0.f;
    if (ch < c)
        for (long long p = p0 + sub; p < p1; p += 4) {
            const int f = (int)(p / hw), rr = (int)(p - (long long)f * hw);
            s += elem<T>::ld(img_ptr<T>(t, f) + (long long)rr * t.ld + ch);
        }
    __shared__ float red[4][64];
    red[sub][cl] = s;
    __syncthreads();
    if (sub == 0 && ch < c) partial[(long long)blockIdx.x * c + ch] = red[0][cl] + red[1][cl] + red[2][cl] + red[3][cl];
}

// 16-B version: TPP threads cover a pixel's channel groups of 8 (TPP a power of two >= ceil(c/8)), 256/TPP
// pixels per block step, four pixel loads in flight per thread; partials [nblk][c] as chan_sum_kernel
template <typename T, int TPP>
__global__ __launch_bounds__(256) void chan_sum16_kernel(int n, int hw, int c, dbsr_tensor t, int px_per_block,
                                                         float* __restrict__ partial) {
    constexpr int PPI = 256 / TPP;
    const int cg = threadIdx.x % TPP, row = threadIdx.x / TPP;
    const bool live = cg * 8 < c;
    const long long total = (long long)n * hw;
    const long long p0 = (long long)blockIdx.x * px_per_block, p1 = std::min<long long>(p0 + px_per_block, total);
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (live) {
        for (long long p = p0 + row; p < p1; p += 4 * PPI) {
            float v[4][8];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const long long q = p + (long long)u * PPI;
                if (q < p1) {
                    const int f = (int)(q / hw), rr = (int)(q - (long long)f * hw);
                    load8(img_ptr<T>(t, f) + (long long)rr * t.ld + cg * 8, v[u]);
                } else {
#pragma unroll
                    for (int j = 0; j < 8; ++j) v[u][j] = 0.f;
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int j = 0; j < 8; ++j) s[j] += v[u][j];
        }
    }
    __shared__ float red[PPI][TPP * 8 + 1];
#pragma unroll
    for (int j = 0; j < 8; ++j) red[row][cg * 8 + j] = s[j];
    __syncthreads();
    for (int ch = threadIdx.x; ch < c; ch += 256) {
        float a = 0.f;
        for (int r = 0; r < PPI; ++r) a += red[r][ch];
        partial[(long long)blockIdx.x * c + ch] = a;
    }
}

// out[ch] (+)= scale * sum over rows of partial[row][ch]: a block per 64 channels, the rows split over 4 waves
// (loads of 64 consecutive floats), the 4 wave sums added in a fixed order (deterministic)
__global__ __launch_bounds__(256) void sum_rows_kernel(int rows, int c, const float* __restrict__ partial,
                                                       float* __restrict__ out, int accumulate, float scale) {
    const int il = threadIdx.x & 63, sl = threadIdx.x >> 6;
    const int ch = blockIdx.x * 64 + il;
    float s = 0.f;
    if (ch < c) {
#pragma unroll 8
        for (int r = sl; r < rows; r += 4) s += partial[(long long)r * c + ch];
    }
    __shared__ float red[4][64];
    red[sl][il] = s;
    __syncthreads();
    if (sl == 0 && ch < c) {
        const float t = (((red[0][il] + red[1][il]) + red[2][il]) + red[3][il]) * scale;
        out[ch] = accumulate ? out[ch] + t : t;
    }
}

// *out = scale * sum of n partials (one block; strided per-thread sums, then a fixed-order tree)
__global__ __launch_bounds__(256) void sum_all_kernel(int n, const float* __restrict__ partial, float* __restrict__ out,
                                                      float scale) {
    float s = 0.f;
#pragma unroll 8
    for (int i = threadIdx.x; i < n; i += 256) s += partial[i];
    __shared__ float red[256];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int st = 128; st > 0; st >>= 1) {
        if ((int)threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
        __syncthreads();
    }
    if (threadIdx.x == 0) *out = red[0] * scale;
}

// ------------------------------------------------------------------------------------------------
// The decoder's RGB predictor (decoders.py:61: 1x1 conv 32 -> HC, ReLU; HC = 3) on its own in the training
// step, where the last post-ResBlock's output h must be kept for the backward (the inference forward fuses
// the predictor into that conv instead: dbsr_conv2d_head).  A thread per pixel, grid-stride:
//   forward:  out[f][c][r] = ReLU(sum_i w[c][i] h[p][i] + b[c])                (fp32 NCHW)
//   backward: dh[p][i] = [h[p][i] > 0] * sum_c w[c][i] dp[p][c]                (dgrad, gated by h's ReLU)
//             dw[c][i] = sum_p dp[p][c] h[p][i], db[c] = sum_p dp[p][c]        (one pass over dp and h)
// The weight/bias sums are fp32 per thread, then a butterfly per wave, the 4 waves in order per block, and
// the blocks in order (sum_rows_kernel): deterministic.  Memory-bound: h is read once, dh written once.
// ------------------------------------------------------------------------------------------------
constexpr int HEAD_CIN = 32;
inline int head_blocks(long long npix) {
    return (int)std::min<long long>(1024, std::max<long long>(1, (npix + 255) / 256));
}

template <typename T, int HC>
__global__ __launch_bounds__(256) void head_fwd_kernel(int n, int hw, dbsr_tensor h, const float* __restrict__ w,
                                                       const float* __restrict__ b, float* __restrict__ out) {
    __shared__ float sw[HC * HEAD_CIN + HC];
    for (int i = threadIdx.x; i < HC * HEAD_CIN; i += 256) sw[i] = w[i];
    if ((int)threadIdx.x < HC) sw[HC * HEAD_CIN + threadIdx.x] = b ? b[threadIdx.x] : 0.f;
    __syncthreads();
    const long long total = (long long)n * hw;
    for (long long p = blockIdx.x * 256LL + threadIdx.x; p < total; p += (long long)gridDim.x * 256) {
        const int f = (int)(p / hw), r = (int)(p - (long long)f * hw);
        const T* hp = img_ptr<T>(h, f) + (long long)r * h.ld;
        float v[4][8];
#pragma unroll
        for (int g = 0; g < 4; ++g) load8(hp + 8 * g, v[g]);
        float a[HC];
#pragma unroll
        for (int c = 0; c < HC; ++c) a[c] = sw[HC * HEAD_CIN + c];
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
            for (int j = 0; j < 8; ++j)
#pragma unroll
                for (int c = 0; c < HC; ++c) a[c] += sw[c * HEAD_CIN + 8 * g + j] * v[g][j];
#pragma unroll
        for (int c = 0; c < HC; ++c) out[((long long)f * HC + c) * hw + r] = fmaxf(a[c], 0.f);
    }
}

template <typename T, int HC>
__global__ __launch_bounds__(256) void head_bwd_kernel(int n, int hw, dbsr_tensor h, dbsr_tensor dp,
                                                       const float* __restrict__ w, dbsr_tensor dh,
                                                       float* __restrict__ pw, float* __restrict__ pb) {
    constexpr int NV = HC * HEAD_CIN + HC;             // dw then db
    __shared__ float sw[HC * HEAD_CIN];
    __shared__ float red[4][NV];
    for (int i = threadIdx.x; i < HC * HEAD_CIN; i += 256) sw[i] = w[i];
    __syncthreads();
    float aw[HC][HEAD_CIN], ab[HC];
#pragma unroll
    for (int c = 0; c < HC; ++c) {
        ab[c] = 0.f;
#pragma unroll
        for (int i = 0; i < HEAD_CIN; ++i) aw[c][i] = 0.f;
    }
    const long long total = (long long)n * hw;
    for (long long p = blockIdx.x * 256LL + threadIdx.x; p < total; p += (long long)gridDim.x * 256) {
        const int f = (int)(p / hw), r = (int)(p - (long long)f * hw);
        const T* hp = img_ptr<T>(h, f) + (long long)r * h.ld;
        T* op = img_ptr<T>(dh, f) + (long long)r * dh.ld;
        float d8[8], v[4][8];
        load8(img_ptr<T>(dp, f) + (long long)r * dp.ld, d8);
#pragma unroll
        for (int g = 0; g < 4; ++g) load8(hp + 8 * g, v[g]);
#pragma unroll
        for (int c = 0; c < HC; ++c) ab[c] += d8[c];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            float o[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int i = 8 * g + j;
                float sacc = 0.f;
#pragma unroll
                for (int c = 0; c < HC; ++c) {
                    sacc += sw[c * HEAD_CIN + i] * d8[c];
                    aw[c][i] += d8[c] * v[g][j];
                }
                o[j] = v[g][j] > 0.f ? sacc : 0.f;
            }
            store8(op + 8 * g, o);
        }
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        float x = k < HC * HEAD_CIN ? aw[k / HEAD_CIN][k % HEAD_CIN] : ab[k - HC * HEAD_CIN];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
        if (lane == 0) red[wave][k] = x;
    }
    __syncthreads();
    for (int k = threadIdx.x; k < NV; k += 256) {
        const float t = ((red[0][k] + red[1][k]) + red[2][k]) + red[3][k];
        if (k < HC * HEAD_CIN) pw[(long long)blockIdx.x * HC * HEAD_CIN + k] = t;
        else pb[(long long)blockIdx.x * HC + (k - HC * HEAD_CIN)] = t;
    }
}

// ------------------------------------------------------------------------------------------------
// L1 loss on the boundary-cropped prediction (models/loss/image_quality_v2.py:24-66, boundary_ignore
// 40, mean reduction) and its gradient through the predictor's ReLU (decoders.py:52, blocks.py:46):
//   d_pre[b,c,y,x] = [pred > 0] * sign(pred - gt) / count inside the crop, 0 outside
// written NHWC (ld >= 4, compute dtype) for the predictor's dgrad / wgrad; |pred - gt| partial sums
// per block into `partial` (the loss is their ordered sum / count).
// ------------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void l1_loss_bwd_kernel(int B, int C, int H, int W, int bi,
                                                          const float* __restrict__ pred, const float* __restrict__ gt,
                                                          float inv_count, dbsr_tensor dpre,
                                                          float* __restrict__ partial) {
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long total = (long long)B * H * W;
    float s = 0.f;
    if (idx < total) {
        const int b = (int)(idx / ((long long)H * W));
        const int rr = (int)(idx - (long long)b * H * W);
        const int y = rr / W, x = rr - y * W;
        const bool in = y >= bi && y < H - bi && x >= bi && x < W - bi;
        T* o = img_ptr<T>(dpre, b) + (long long)rr * dpre.ld;
        for (int c = 0; c < C; ++c) {
            const long long off = ((long long)b * C + c) * H * W + rr;
            const float d = pred[off] - gt[off];
            float gv = 0.f;
            if (in) {
                s += fabsf(d);
                gv = pred[off] > 0.f ? (d > 0.f ? inv_count : (d < 0.f ? -inv_count : 0.f)) : 0.f;
            }
            elem<T>::st(o + c, gv);
        }
    }
    __shared__ float red[256];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int st = 128; st > 0; st >>= 1) {
        if ((int)threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
        __syncthreads();
    }
    if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}

// Same, 16-bit dpre with exactly 8 channels per pixel (c0 0, C <= 8): 4 pixels per thread, one 16-B store
// per pixel (channels C..7 written as the zeros they hold), wave-shuffle partial sums
template <typename T>
__global__ __launch_bounds__(256) void l1_loss_bwd8_kernel(int B, int C, int H, int W, int bi,
                                                           const float* __restrict__ pred, const float* __restrict__ gt,
                                                           float inv_count, dbsr_tensor dpre,
                                                           float* __restrict__ partial) {
    const long long total = (long long)B * H * W;
    const long long hw = (long long)H * W;
    float s = 0.f;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const long long idx = ((long long)blockIdx.x * 4 + u) * 256 + threadIdx.x;
        if (idx >= total) break;
        const int b = (int)(idx / hw);
        const int rr = (int)(idx - (long long)b * hw);
        const int y = rr / W, x = rr - y * W;
        const bool in = y >= bi && y < H - bi && x >= bi && x < W - bi;
        float gv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        for (int c = 0; c < C; ++c) {
            const long long off = ((long long)b * C + c) * hw + rr;
            const float pv = pred[off], d = pv - gt[off];
            if (in) {
                s += fabsf(d);
                gv[c] = pv > 0.f ? (d > 0.f ? inv_count : (d < 0.f ? -inv_count : 0.f)) : 0.f;
            }
        }
        store8(img_ptr<T>(dpre, b) + (long long)rr * 8, gv);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    __shared__ float red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) partial[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// The predictor ReLU's backward from an arbitrary upstream gradient (autograd through DBSRNet.forward, any
// objective): dpre[b][y][x][c] = [pred > 0] * gout[b][c][y][x] (fp32 NCHW in, NHWC out in the compute dtype).
template <typename T>
__global__ __launch_bounds__(256) void relu_grad_kernel(int B, int C, int H, int W, const float* __restrict__ pred,
                                                        const float* __restrict__ gout, dbsr_tensor dpre) {
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long long)B * H * W) return;
    const int b = (int)(idx / ((long long)H * W));
    const int rr = (int)(idx - (long long)b * H * W);
    T* o = img_ptr<T>(dpre, b) + (long long)rr * dpre.ld;
    for (int c = 0; c < C; ++c) {
        const long long off = ((long long)b * C + c) * H * W + rr;
        elem<T>::st(o + c, pred[off] > 0.f ? gout[off] : 0.f);
    }
}

// ------------------------------------------------------------------------------------------------
// PixelShuffle(s) backward with the upsampler's ReLU (upsampling.py:51-58): the gradient of the
// shuffled, ReLU'd output dS [B][sH][sW][C] (and the forward output S itself as the gate) -> the conv's
// pre-activation gradient in torch channel order k = c*s^2 + i*s + j: dU[b][y][x][k] =
// dS[b][y*s+i][x*s+j][c] * [S > 0].
// ------------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void unshuffle_gate_kernel(int B, int H, int W, int s, int C, dbsr_tensor ds,
                                                             dbsr_tensor gate, dbsr_tensor du) {
    const int K = C * s * s;
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long long)B * H * W * K) return;
    const int k = (int)(idx % K);
    const long long pix = idx / K;
    const int b = (int)(pix / ((long long)H * W)), rr = (int)(pix - (long long)b * H * W);
    const int y = rr / W, x = rr - y * W;
    const int c = k / (s * s), sub = k - c * s * s, i = sub / s, j = sub - i * s;
    const long long hr = (long long)(y * s + i) * (W * s) + (x * s + j);
    const float g = elem<T>::ld(img_ptr<T>(gate, b) + hr * gate.ld + c);
    const float v = g > 0.f ? elem<T>::ld(img_ptr<T>(ds, b) + hr * ds.ld + c) : 0.f;
    elem<T>::st(img_ptr<T>(du, b) + (long long)rr * du.ld + k, v);
}

// 16-B version: a block per low-res pixel (looping), thread = (sub-pixel, 8-channel group): 16-B loads of dS
// and the gate, the block's K = C*s*s outputs transposed through the LDS into 16-B stores
template <typename T>
__global__ __launch_bounds__(256) void unshuffle_gate16_kernel(int B, int H, int W, int s, int C, dbsr_tensor ds,
                                                               dbsr_tensor gate, dbsr_tensor du) {
    extern __shared__ __attribute__((aligned(16))) unsigned char ush[];
    T* tile = (T*)ush;
    const int ss = s * s, K = C * ss, groups = C / 8, tasks = ss * groups;
    const long long npix = (long long)B * H * W;
    for (long long pix = blockIdx.x; pix < npix; pix += gridDim.x) {
        const int b = (int)(pix / ((long long)H * W)), rr = (int)(pix - (long long)b * H * W);
        const int y = rr / W, x = rr - y * W;
        for (int t = threadIdx.x; t < tasks; t += 256) {
            const int sub = t / groups, cg = t - sub * groups, i = sub / s, j = sub - i * s;
            const long long hr = (long long)(y * s + i) * (W * s) + (x * s + j);
            float d[8], g[8];
            load8(img_ptr<T>(ds, b) + hr * ds.ld + cg * 8, d);
            load8(img_ptr<T>(gate, b) + hr * gate.ld + cg * 8, g);
#pragma unroll
            for (int e = 0; e < 8; ++e) elem<T>::st(tile + (cg * 8 + e) * ss + sub, g[e] > 0.f ? d[e] : 0.f);
        }
        __syncthreads();
        T* o = img_ptr<T>(du, b) + (long long)rr * du.ld;
        for (int q = threadIdx.x; q < K / 8; q += 256) *(u32x4_t*)(o + q * 8) = *(const u32x4_t*)(tile + q * 8);
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------------------
// Softmax-fusion backward (merging.py:116-124): fused = sum_n w_n f_n, w = softmax_n(l) per channel.
//   dF_n = w_n * dfused;  dl_n = w_n * dfused * (f_n - fused)
// Frame (b, n): weights/logit-grad image b*N+n; feature n == 0 -> ref image b (map), n > 0 -> oth image
// b*(N-1)+n-1; dref: image b; doth: image b*(N-1)+n-1.  8 channels per thread.
// ------------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void fuse_bwd_kernel(int B, int N, int hw, int C, dbsr_tensor wts, dbsr_tensor ref,
                                                       dbsr_tensor oth, dbsr_tensor fused, dbsr_tensor dfused,
                                                       dbsr_tensor dlogits, dbsr_tensor dref, dbsr_tensor doth) {
    const int groups = C / 8;
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long long)B * hw * groups) return;
    // 32-bit index math (the host checks B * hw * groups < 2^31): 64-bit divisions cost ~100 VALU each
    const unsigned ui = (unsigned)idx, pix = ui / (unsigned)groups;
    const int g = (int)(ui - pix * (unsigned)groups);
    const int b = (int)(pix / (unsigned)hw), rr = (int)(pix - (unsigned)b * (unsigned)hw);
    const int c = g * 8;
    float fu[8], dfu[8];
    load8(img_ptr<T>(fused, b) + (long long)rr * fused.ld + c, fu);
    load8(img_ptr<T>(dfused, b) + (long long)rr * dfused.ld + c, dfu);
    // frames in chunks of FB: every load of a chunk is issued before its first store (the stores may alias the
    // inputs as far as the compiler knows, so a load after a store waits for it: one latency per frame before)
    constexpr int FB = 7;
    constexpr int RW = sizeof(T) == 2 ? 1 : 2;           // 16-B words per 8 elements
    for (int n0 = 0; n0 < N; n0 += FB) {
        u32x4_t wr[FB][RW], fr[FB][RW];                  // raw: converted when used (half the registers)
#pragma unroll
        for (int u = 0; u < FB; ++u) {
            const int n = n0 + u;
            if (n < N) {
                const T* wp = img_ptr<T>(wts, b * N + n) + (long long)rr * wts.ld + c;
                const T* fp = (n == 0 ? img_ptr<T>(ref, b) + (long long)rr * ref.ld
                                      : img_ptr<T>(oth, b * (N - 1) + n - 1) + (long long)rr * oth.ld) + c;
#pragma unroll
                for (int q4 = 0; q4 < RW; ++q4) {
                    wr[u][q4] = *(const u32x4_t*)(wp + q4 * (8 / RW));
                    fr[u][q4] = *(const u32x4_t*)(fp + q4 * (8 / RW));
                }
            }
        }
#pragma unroll
        for (int u = 0; u < FB; ++u) {
            const int n = n0 + u;
            if (n >= N) break;
            float wv[8], fv[8];
            if constexpr (sizeof(T) == 2) {
#pragma unroll
                for (int q4 = 0; q4 < 4; ++q4) {
                    wv[2 * q4] = H16<T>::lo(wr[u][0][q4]); wv[2 * q4 + 1] = H16<T>::hi(wr[u][0][q4]);
                    fv[2 * q4] = H16<T>::lo(fr[u][0][q4]); fv[2 * q4 + 1] = H16<T>::hi(fr[u][0][q4]);
                }
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    wv[j] = __uint_as_float(wr[u][j / 4][j % 4]);
                    fv[j] = __uint_as_float(fr[u][j / 4][j % 4]);
                }
            }
            float dl[8], df[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                df[j] = wv[j] * dfu[j];
                dl[j] = df[j] * (fv[j] - fu[j]);
            }
            store8(img_ptr<T>(dlogits, b * N + n) + (long long)rr * dlogits.ld + c, dl);
            T* dp = n == 0 ? img_ptr<T>(dref, b) + (long long)rr * dref.ld
                           : img_ptr<T>(doth, b * (N - 1) + n - 1) + (long long)rr * doth.ld;
            store8(dp + c, df);
        }
    }
}

// ------------------------------------------------------------------------------------------------
// merge-prep backward (merging.py:79-89) + the projection's ReLU: weight-predictor input gradient
// dwp [b*N+n][base(c) | diff(c) | ...] ->
//   d_proj[b,0] = sum_n d_base[b,n] - sum_{n>=1} d_diff[b,n];  d_proj[b,n>=1] = d_diff[b,n]
// times [proj > 0], into dproj (images b*N+n).
// ------------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void merge_prep_bwd_kernel(int B, int N, int hw, int C, dbsr_tensor dwp,
                                                             dbsr_tensor proj, dbsr_tensor dproj) {
    const int groups = C / 8;
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long long)B * N * hw * groups) return;
    const int g = (int)(idx % groups);
    const long long pix = idx / groups;
    const int f = (int)(pix / hw), rr = (int)(pix - (long long)f * hw);
    const int b = f / N, n = f - b * N;
    const int c = g * 8;
    float d[8];
    if (n > 0) {
        load8(img_ptr<T>(dwp, f) + (long long)rr * dwp.ld + C + c, d);
    } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) d[j] = 0.f;
        for (int m = 0; m < N; ++m) {
            float db[8], dd[8];
            load8(img_ptr<T>(dwp, b * N + m) + (long long)rr * dwp.ld + c, db);
            load8(img_ptr<T>(dwp, b * N + m) + (long long)rr * dwp.ld + C + c, dd);
#pragma unroll
            for (int j = 0; j < 8; ++j) d[j] += db[j] - (m > 0 ? dd[j] : 0.f);
        }
    }
    float pv[8];
    load8(img_ptr<T>(proj, f) + (long long)rr * proj.ld + c, pv);
#pragma unroll
    for (int j = 0; j < 8; ++j) d[j] = pv[j] > 0.f ? d[j] : 0.f;
    store8(img_ptr<T>(dproj, f) + (long long)rr * dproj.ld + c, d);
}

// ------------------------------------------------------------------------------------------------
// warp backward w.r.t. the features (models/layers/warp.py:19-46 = grid_sample bilinear, zeros,
// align_corners=False at (x + fx, y + fy)): dfeat[src] += w_tap * dout[p] for the 4 taps of every
// output pixel -- fp32 atomics into dfeat32 (the scatter has no gather form for arbitrary flow), 8
// channels per thread.
// ------------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void warp_bwd_kernel(int n, int h, int w, int C, dbsr_tensor dout,
                                                       const float* __restrict__ flow, long long fis,
                                                       float* __restrict__ dfeat32, dbsr_frame_map fmap,
                                                       long long df_img_stride) {
    const int groups = C / 8;
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long long)n * h * w * groups) return;
    const int g = (int)(idx % groups);
    const long long pix = idx / groups;
    const int hw = h * w;
    const int p = (int)(pix / hw), rr = (int)(pix - (long long)p * hw);
    const int y = rr / w, x = rr - y * w;
    const float* fl = flow + (long long)p * fis + rr;
    const float gx = ((float)x + 0.5f) + fl[0], gy = ((float)y + 0.5f) + fl[hw];
    const float gxn = 2.0f * gx / (float)w - 1.0f, gyn = 2.0f * gy / (float)h - 1.0f;
    const float ix = ((gxn + 1.f) * (float)w - 1.f) / 2.f, iy = ((gyn + 1.f) * (float)h - 1.f) / 2.f;
    const float fx0 = floorf(ix), fy0 = floorf(iy);
    const int x0 = (int)fx0, y0 = (int)fy0;
    const float wx1 = ix - fx0, wx0 = 1.f - wx1, wy1 = iy - fy0, wy0 = 1.f - wy1;
    float d[8];
    load8(img_ptr<T>(dout, p) + (long long)rr * dout.ld + g * 8, d);
    float* base = dfeat32 + map_frame(fmap, p) * df_img_stride + g * 8;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int xx = x0 + (t & 1), yy = y0 + (t >> 1);
        if ((unsigned)xx >= (unsigned)w || (unsigned)yy >= (unsigned)h) continue;
        const float wt = ((t & 1) ? wx1 : wx0) * ((t >> 1) ? wy1 : wy0);
        float* o = base + ((long long)yy * w + xx) * C;
#pragma unroll
        for (int j = 0; j < 8; ++j) atomicAdd(o + j, wt * d[j]);
    }
}

// ------------------------------------------------------------------------------------------------
// warp backward as an owner-computes gather (no atomics on features, no fp32 scratch image).  The
// contributions -- (output pixel p, bilinear weight) for each in-frame tap q of p -- are binned per
// destination pixel q by a counting sort (wb_count: per-pixel counts; wb_scan: offsets per pair; wb_scatter:
// 8-B records {p, weight}), then wb_gather runs one wave per destination pixel: lanes own 8 channels each
// (16-B loads of dout[p]), the pixel's few contributions (4 on average) are summed in registers in record
// order and the result is written once, gated by the encoder output's ReLU (encoders.py:66-72):
// dfeat[q] = [gate[q] > 0] * sum_p w(p, q) dout[p].  Any flow field costs the same per contribution.  The
// scatter's atomics place a pixel's records in arbitrary order, so the gather sums them sorted by source pixel
// (unique within a destination: a source's four taps hit four different pixels): the gradients are bitwise
// reproducible run to run.
// ------------------------------------------------------------------------------------------------
struct WarpTaps { int x0, y0; float wx1, wy1; };
// bilinear taps of output pixel (x, y) (grid_sample, zeros, align_corners=False; as warp_kernel)
__device__ __forceinline__ WarpTaps warp_taps(int x, int y, int w, int h, float fx, float fy) {
    const float gx = ((float)x + 0.5f) + fx, gy = ((float)y + 0.5f) + fy;
    const float gxn = 2.0f * gx / (float)w - 1.0f, gyn = 2.0f * gy / (float)h - 1.0f;
    const float ix = ((gxn + 1.f) * (float)w - 1.f) / 2.f, iy = ((gyn + 1.f) * (float)h - 1.f) / 2.f;
    const float fx0 = floorf(ix), fy0 = floorf(iy);
    WarpTaps t;
    // far-away / non-finite coordinates: no tap in the frame (x0 = -2 keeps both columns out)
    const bool ok = fx0 >= -1.f && fx0 < (float)w && fy0 >= -1.f && fy0 < (float)h;
    t.x0 = ok ? (int)fx0 : -2;
    t.y0 = ok ? (int)fy0 : -2;
    t.wx1 = ix - fx0;
    t.wy1 = iy - fy0;
    return t;
}

__global__ __launch_bounds__(256) void wb_count_kernel(int n, int h, int w, const float* __restrict__ flow,
                                                       long long fis, int* __restrict__ counts) {
    const int hw = h * w;
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long long)n * hw) return;
    const int p = (int)((unsigned)idx / (unsigned)hw), rr = (int)((unsigned)idx - (unsigned)p * (unsigned)hw);   // n*hw < 2^31
    const float* fl = flow + (long long)p * fis;
    const WarpTaps t = warp_taps(rr % w, rr / w, w, h, fl[rr], fl[hw + rr]);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int xx = t.x0 + (k & 1), yy = t.y0 + (k >> 1);
        if ((unsigned)xx < (unsigned)w && (unsigned)yy < (unsigned)h)
            atomicAdd(&counts[(long long)p * hw + yy * w + xx], 1);
    }
}

// per pair: exclusive prefix sum of the per-pixel counts -> offsets and scatter cursors.  One block per pair;
// thread t scans 16 consecutive pixels serially, the block scans the 1024 thread totals, chunk by chunk.
__global__ __launch_bounds__(1024) void wb_scan_kernel(int hw, const int* __restrict__ counts,
                                                       int* __restrict__ offsets, int* __restrict__ cursor) {
    constexpr int PER = 16;
    const long long base_p = (long long)blockIdx.x * hw;
    __shared__ int part[1024];
    __shared__ int carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (int base = 0; base < hw; base += 1024 * PER) {
        const int i0 = base + (int)threadIdx.x * PER;
        int v[PER], tot = 0;
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            v[j] = i0 + j < hw ? counts[base_p + i0 + j] : 0;
            tot += v[j];
        }
        part[threadIdx.x] = tot;
        __syncthreads();
        for (int o = 1; o < 1024; o <<= 1) {                // Hillis-Steele inclusive scan of the totals
            const int a = (int)threadIdx.x >= o ? part[threadIdx.x - o] : 0;
            __syncthreads();
            part[threadIdx.x] += a;
            __syncthreads();
        }
        int ex = carry + part[threadIdx.x] - tot;
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            if (i0 + j < hw) {
                offsets[base_p + i0 + j] = ex;
                cursor[base_p + i0 + j] = ex;
            }
            ex += v[j];
        }
        __syncthreads();
        if (threadIdx.x == 1023) carry += part[1023];
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void wb_scatter_kernel(int n, int h, int w, const float* __restrict__ flow,
                                                         long long fis, int* __restrict__ cursor,
                                                         int2* __restrict__ records) {
    const int hw = h * w;
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long long)n * hw) return;
    const int p = (int)((unsigned)idx / (unsigned)hw), rr = (int)((unsigned)idx - (unsigned)p * (unsigned)hw);   // n*hw < 2^31
    const float* fl = flow + (long long)p * fis;
    const WarpTaps t = warp_taps(rr % w, rr / w, w, h, fl[rr], fl[hw + rr]);
    int2* rec = records + (long long)p * 4 * hw;             // the pair's region: <= 4 records per pixel
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int xx = t.x0 + (k & 1), yy = t.y0 + (k >> 1);
        if ((unsigned)xx >= (unsigned)w || (unsigned)yy >= (unsigned)h) continue;
        const float wt = ((k & 1) ? t.wx1 : 1.f - t.wx1) * ((k >> 1) ? t.wy1 : 1.f - t.wy1);
        const int pos = atomicAdd(&cursor[(long long)p * hw + yy * w + xx], 1);
        rec[pos] = int2{rr, __float_as_int(wt)};
    }
}

// one wave per destination pixel; lanes = 8-channel groups (16-B loads), channel passes of 512
template <typename T>
__global__ __launch_bounds__(256) void wb_gather_kernel(int n, int h, int w, int C, dbsr_tensor dout,
                                                        const int* __restrict__ counts, const int* __restrict__ offsets,
                                                        const int2* __restrict__ records, dbsr_tensor gate,
                                                        dbsr_tensor dfeat) {
    __shared__ int2 sorted[4][64];
    const int hw = h * w;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const long long q = (long long)blockIdx.x * 4 + wv;
    if (q >= (long long)n * hw) return;
    const int p = (int)((unsigned)q / (unsigned)hw), rr = (int)((unsigned)q - (unsigned)p * (unsigned)hw);   // n*hw < 2^31
    const int cnt = counts[q];
    const int2* rec = records + (long long)p * 4 * hw + offsets[q];
    const T* src = img_ptr<T>(dout, p);
    T* dst = img_ptr<T>(dfeat, p) + (long long)rr * dfeat.ld;
    const T* gp = gate.ptr ? img_ptr<T>(gate, p) + (long long)rr * gate.ld : nullptr;
    if (cnt <= 64) {
        // rank of each record by source pixel (lane e holds record e), then the records in that order in the LDS
        const int2 mine = lane < cnt ? rec[lane] : int2{0x7fffffff, 0};
        int rank = 0;
        for (int j = 0; j < cnt; ++j) rank += __shfl(mine.x, j) < mine.x;
        if (lane < cnt) sorted[wv][rank] = mine;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    // record e in source-pixel order: from the LDS, or (more than 64 contributions: strongly converging flows)
    // the e-th smallest source found by a wave-wide minimum over the pixel's records
    int last = -1;
    auto record = [&](int e) -> int2 {
        if (cnt <= 64) return sorted[wv][e];
        int bx = 0x7fffffff, by = 0;
        for (int i = lane; i < cnt; i += 64) {
            const int2 r = rec[i];
            if (r.x > last && r.x < bx) { bx = r.x; by = r.y; }
        }
        for (int o = 32; o >= 1; o >>= 1) {
            const int ox = __shfl_xor(bx, o), oy = __shfl_xor(by, o);
            if (ox < bx) { bx = ox; by = oy; }
        }
        last = bx;
        return int2{bx, by};
    };
    for (int c0 = 0; c0 < C; c0 += 512) {
        const int c = c0 + lane * 8;
        const bool on = c < C;              // (lanes past C stay in the loop: record() may need the whole wave)
        float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        last = -1;
        for (int e0 = 0; e0 < cnt; e0 += 4) {
            float d[4][8];
            float wt[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if (e0 + u < cnt) {
                    const int2 r = record(e0 + u);
                    wt[u] = __int_as_float(r.y);
                    if (on) {
                        load8(src + (long long)r.x * dout.ld + c, d[u]);
                    } else {
#pragma unroll
                        for (int j = 0; j < 8; ++j) d[u][j] = 0.f;
                    }
                } else {
                    wt[u] = 0.f;
#pragma unroll
                    for (int j = 0; j < 8; ++j) d[u][j] = 0.f;
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int j = 0; j < 8; ++j) a[j] = fmaf(wt[u], d[u][j], a[j]);
        }
        if (!on) continue;
        if (gp) {
            float g[8];
            load8(gp + c, g);
#pragma unroll
            for (int j = 0; j < 8; ++j) a[j] = g[j] > 0.f ? a[j] : 0.f;
        }
        store8(dst + c, a);
    }
}

__global__ void zero_ints_kernel(long long n, int* __restrict__ p) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = 0;
}

// out[f] = [gate[f] > 0] * in[f] over n images of c channels (8 per thread, 16-B accesses)
template <typename T>
__global__ __launch_bounds__(256) void gate_copy_kernel(int n, int hw, int c, dbsr_tensor in, dbsr_tensor gate,
                                                        dbsr_tensor out) {
    const int groups = c / 8;
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long long)n * hw * groups) return;
    const int g = (int)(idx % groups);
    const long long pix = idx / groups;
    const int f = (int)(pix / hw), rr = (int)(pix - (long long)f * hw);
    float d[8], e[8];
    load8(img_ptr<T>(in, f) + (long long)rr * in.ld + g * 8, d);
    load8(img_ptr<T>(gate, f) + (long long)rr * gate.ld + g * 8, e);
#pragma unroll
    for (int j = 0; j < 8; ++j) d[j] = e[j] > 0.f ? d[j] : 0.f;
    store8(img_ptr<T>(out, f) + (long long)rr * out.ld + g * 8, d);
}

// ------------------------------------------------------------------------------------------------
// Encoder output gradient assembly (encoders.py:66-80 + the out_layer ReLU): frame (b, n):
//   n == 0: dE = dref[b];  n >= 1: dE = dsrc32[b*N+n] (the warp scatter)
// times [E > 0], into dE (images b*N+n).
// ------------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void enc_grad_gate_kernel(int B, int N, int hw, int C, dbsr_tensor dref,
                                                            const float* __restrict__ dsrc32, dbsr_tensor e,
                                                            dbsr_tensor de) {
    const int groups = C / 8;
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long long)B * N * hw * groups) return;
    const int g = (int)(idx % groups);
    const long long pix = idx / groups;
    const int f = (int)(pix / hw), rr = (int)(pix - (long long)f * hw);
    const int b = f / N, n = f - b * N;
    float d[8];
    if (n == 0) {
        load8(img_ptr<T>(dref, b) + (long long)rr * dref.ld + g * 8, d);
    } else {
        const float* s = dsrc32 + ((long long)f * hw + rr) * C + g * 8;
#pragma unroll
        for (int j = 0; j < 8; ++j) d[j] = s[j];
    }
    float ev[8];
    load8(img_ptr<T>(e, f) + (long long)rr * e.ld + g * 8, ev);
#pragma unroll
    for (int j = 0; j < 8; ++j) d[j] = ev[j] > 0.f ? d[j] : 0.f;
    store8(img_ptr<T>(de, f) + (long long)rr * de.ld + g * 8, d);
}

// ------------------------------------------------------------------------------------------------
// Adam (torch.optim.Adam, weight_decay 0, amsgrad False; trainers/simple_trainer.py:81 with the
// default_synthetic.py:94 optimizer): on flat fp32 parameter / gradient / moment buffers.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void adam_kernel(long long n, float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v, float lr, float b1,
                                                   float b2, float eps, float bc1, float bc2_sqrt, float gscale) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float gi = g[i] * gscale;
    const float mi = b1 * m[i] + (1.f - b1) * gi;
    const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    // torch: p -= lr / bc1 * m / (sqrt(v) / sqrt(bc2) + eps)
    p[i] -= (lr / bc1) * mi / (sqrtf(vi) / bc2_sqrt + eps);
}

// dgrad weights: the conv of the output gradient with the transposed, spatially flipped kernel
// W'[ci][co][ky][kx] = W[co][ci][kh-1-ky][kw-1-kx] (fp32 torch layout in and out)
__global__ void dgrad_weights_kernel(const float* __restrict__ w, int cout, int cin, int kh, int kw,
                                     float* __restrict__ wt) {
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long long)cout * cin * kh * kw) return;
    const int kx = (int)(idx % kw), ky = (int)((idx / kw) % kh);
    const int co = (int)((idx / ((long long)kw * kh)) % cout), ci = (int)(idx / ((long long)kw * kh * cout));
    wt[idx] = w[(((long long)co * cin + ci) * kh + (kh - 1 - ky)) * kw + (kw - 1 - kx)];
}

}  // namespace

// ================================================================================================
static int wgrad_cb(int cin, int cout) { return (cin <= 32 && cout <= 32) ? 32 : 64; }

static int g_wgrad_dma = 1;             // dbsr_set_wgrad_algo: 0 = the register-staged kernel only (A/B, tests)

static long long wgrad_nbx(int n_frames, int h, int w, int cin, int cout) {
    const int cb = wgrad_cb(cin, cout);
    const long long units = (long long)n_frames * ((h + WG_TH - 1) / WG_TH) * ((w + WG_TW - 1) / WG_TW);
    const int nty = (cout + cb - 1) / cb, ntz = (cin + cb - 1) / cb;
    return std::max<long long>(1, std::min<long long>(units, std::max(1, wg_blocks(cb) / (nty * ntz))));
}

// the weight partial slots, then (256-B aligned) the bias partials [nbx][cout]
static size_t wgrad_slot_bytes(int n_frames, int h, int w, int cin, int cout, int k) {
    const int cb = wgrad_cb(cin, cout);
    const int nty = (cout + cb - 1) / cb, ntz = (cin + cb - 1) / cb;
    const size_t b = (size_t)wgrad_nbx(n_frames, h, w, cin, cout) * nty * ntz * (k == 3 ? 9 : 4) * cb * cb * sizeof(float);
    return (b + 255) / 256 * 256;
}

extern "C" size_t dbsr_conv_wgrad_workspace_bytes(int n_frames, int h, int w, int cin, int cout, int k) {
    if (n_frames <= 0 || h <= 0 || w <= 0 || cin <= 0 || cout <= 0 || (k != 1 && k != 3)) return 0;
    return wgrad_slot_bytes(n_frames, h, w, cin, cout, k) +
           (size_t)wgrad_nbx(n_frames, h, w, cin, cout) * cout * sizeof(float);
}

extern "C" int dbsr_conv_wgrad_bias(int n_frames, int h, int w, dbsr_tensor x, int cin, dbsr_tensor dy, int cout,
                                    int k, float* dw, float* db, int accumulate, void* workspace,
                                    size_t workspace_bytes, void* stream) {
    DBSR_CHECK_ARG(map_ok(x) && map_ok(dy) && dw && workspace, "conv_wgrad: null pointer");
    DBSR_CHECK_ARG(x.dtype == dy.dtype, "conv_wgrad: x and dy dtypes differ");
    DBSR_CHECK_ARG(k == 1 || k == 3, "conv_wgrad: k must be 1 or 3 (stride 1, pad k/2)");
    DBSR_CHECK_ARG(n_frames > 0 && h > 0 && w > 0 && cin > 0 && cout > 0, "conv_wgrad: bad sizes");
    const int esz = x.dtype == DBSR_F32 ? 4 : 2, epp = 16 / esz;
    DBSR_CHECK_ARG(vec_ok(x, epp) && vec_ok(dy, epp) && x.ld >= x.c0 + (cin + epp - 1) / epp * epp &&
                   dy.ld >= dy.c0 + (cout + epp - 1) / epp * epp,
                   "conv_wgrad: ld/c0 must be multiples of %d and cover the channels", epp);
    const size_t need = dbsr_conv_wgrad_workspace_bytes(n_frames, h, w, cin, cout, k);
    DBSR_CHECK_ARG(workspace_bytes >= need, "conv_wgrad: workspace %zu < %zu bytes", workspace_bytes, need);
    const long long units = (long long)n_frames * ((h + WG_TH - 1) / WG_TH) * ((w + WG_TW - 1) / WG_TW);
    const int cb = wgrad_cb(cin, cout);
    const int nty = (cout + cb - 1) / cb, ntz = (cin + cb - 1) / cb;
    const int nbx = (int)wgrad_nbx(n_frames, h, w, cin, cout);
    const int nw = k == 3 ? 9 : 4;
    float* part = (float*)workspace;
    float* bpart = db ? (float*)((char*)workspace + wgrad_slot_bytes(n_frames, h, w, cin, cout, k)) : nullptr;
    hipStream_t s = (hipStream_t)stream;
    // the channel slice is folded into the base pointers
    dbsr_tensor xx = x, dd = dy;
    xx.ptr = (char*)x.ptr + (long long)x.c0 * esz;
    xx.c0 = 0;
    dd.ptr = (char*)dy.ptr + (long long)dy.c0 * esz;
    dd.c0 = 0;
    const dim3 grid(nbx, nty, ntz);
    // the LDS-DMA kernel (16-bit; buffer offsets of a frame within 31 bits), else the register-staged one
    const bool dma = esz == 2 && (long long)h * w * std::max(x.ld, dy.ld) * 2 < (1LL << 31) && units < (1LL << 31) &&
                     g_wgrad_dma;
    int rc = by_dtype(x.dtype, [&](auto* tag) {
        using T = std::remove_pointer_t<decltype(tag)>;
#define DBSR_WG(KK, CBB)                                                                                     \
    do {                                                                                                     \
        if constexpr (sizeof(T) == 2)                                                                        \
            if (dma) {                                                                                       \
                hipLaunchKernelGGL((conv_wgrad_dma_kernel<T, KK, CBB>), grid, dim3(KK == 3 ? 576 : 256), 0, s, \
                                   n_frames, h, w, xx, cin, dd, cout, units, part, bpart);                   \
                break;                                                                                       \
            }                                                                                                \
        hipLaunchKernelGGL((conv_wgrad_kernel<T, KK, CBB>), grid, dim3(KK == 3 ? 576 : 256), 0, s,          \
                           n_frames, h, w, xx, cin, dd, cout, units, part, bpart);                           \
    } while (0)
        if (k == 3) {
            if (cb == 32) DBSR_WG(3, 32); else DBSR_WG(3, 64);
        } else {
            if (cb == 32) DBSR_WG(1, 32); else DBSR_WG(1, 64);
        }
#undef DBSR_WG
        DBSR_LAUNCH_CHECK();
        return 0;
    });
    if (rc) return rc;
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)(cout * k * k * ((cin + 63) / 64))), dim3(256), 0, s, nbx,
                       nty, ntz, nw, k * k, cout, cin, cb, part, dw, accumulate);
    DBSR_LAUNCH_CHECK();
    if (db) {
        hipLaunchKernelGGL(sum_rows_kernel, dim3((unsigned)((cout + 63) / 64)), dim3(256), 0, s, nbx, cout,
                           (const float*)bpart, db, accumulate, 1.0f);
        DBSR_LAUNCH_CHECK();
    }
    return 0;
}

extern "C" int dbsr_set_wgrad_algo(int algo) {
    DBSR_CHECK_ARG(algo == 0 || algo == 1, "set_wgrad_algo: 0 (register-staged) or 1 (LDS-DMA, default)");
    g_wgrad_dma = algo;
    return 0;
}

extern "C" int dbsr_conv_wgrad(int n_frames, int h, int w, dbsr_tensor x, int cin, dbsr_tensor dy, int cout, int k,
                               float* dw, int accumulate, void* workspace, size_t workspace_bytes, void* stream) {
    return dbsr_conv_wgrad_bias(n_frames, h, w, x, cin, dy, cout, k, dw, nullptr, accumulate, workspace,
                                workspace_bytes, stream);
}

// ================================================================================================
// predictor head (training step)
static int head_check(int n, int hw, const dbsr_tensor& h, int cin, int hc) {
    DBSR_CHECK_ARG(n > 0 && hw > 0 && map_ok(h), "head: bad sizes or null h");
    DBSR_CHECK_ARG(cin == HEAD_CIN, "head: cin must be %d (the decoder's 32-channel post-ResBlocks)", HEAD_CIN);
    DBSR_CHECK_ARG(hc >= 1 && hc <= 4, "head: head_cout must be 1..4");
    const int epp = h.dtype == DBSR_F32 ? 4 : 8;
    DBSR_CHECK_ARG(vec_ok(h, epp) && h.ld >= h.c0 + HEAD_CIN, "head: h ld/c0 must be multiples of 16 B and cover 32");
    return 0;
}

#define DBSR_HEAD_HC(HCV, ...) \
    switch (HCV) { case 1: { constexpr int HC = 1; __VA_ARGS__; } break; case 2: { constexpr int HC = 2; __VA_ARGS__; } break; \
                   case 3: { constexpr int HC = 3; __VA_ARGS__; } break; default: { constexpr int HC = 4; __VA_ARGS__; } }

extern "C" int dbsr_head_forward(int n, int hw, dbsr_tensor h, int cin, const float* w, const float* b, int hc,
                                 float* out, void* stream) {
    if (int rc = head_check(n, hw, h, cin, hc)) return rc;
    DBSR_CHECK_ARG(w && out, "head_forward: null pointer");
    hipStream_t s = (hipStream_t)stream;
    const int nb = head_blocks((long long)n * hw);
    return by_dtype(h.dtype, [&](auto* tag) {
        using T = std::remove_pointer_t<decltype(tag)>;
        DBSR_HEAD_HC(hc, hipLaunchKernelGGL((head_fwd_kernel<T, HC>), dim3(nb), dim3(256), 0, s, n, hw, h, w, b, out))
        DBSR_LAUNCH_CHECK();
        return 0;
    });
}

extern "C" size_t dbsr_head_backward_workspace_bytes(int n, int hw, int cin, int hc) {
    if (n <= 0 || hw <= 0 || hc < 1 || hc > 4) return 0;
    return (size_t)head_blocks((long long)n * hw) * (size_t)(hc * (cin > 0 ? cin : HEAD_CIN) + hc) * sizeof(float);
}

extern "C" int dbsr_head_backward(int n, int hw, dbsr_tensor h, int cin, dbsr_tensor dp, const float* w, int hc,
                                  dbsr_tensor dh, float* dw, float* db, int accumulate, void* workspace,
                                  size_t workspace_bytes, void* stream) {
    if (int rc = head_check(n, hw, h, cin, hc)) return rc;
    DBSR_CHECK_ARG(map_ok(dp) && map_ok(dh) && w && dw && workspace, "head_backward: null pointer");
    DBSR_CHECK_ARG(dp.dtype == h.dtype && dh.dtype == h.dtype, "head_backward: dtypes differ");
    const int epp = h.dtype == DBSR_F32 ? 4 : 8;
    DBSR_CHECK_ARG(vec_ok(dp, epp) && dp.ld >= dp.c0 + 8, "head_backward: dp needs 8 readable channels, 16-B aligned");
    DBSR_CHECK_ARG(vec_ok(dh, epp) && dh.ld >= dh.c0 + HEAD_CIN, "head_backward: dh ld/c0 must be 16-B multiples, >= 32");
    DBSR_CHECK_ARG(workspace_bytes >= dbsr_head_backward_workspace_bytes(n, hw, cin, hc), "head_backward: workspace too small");
    hipStream_t s = (hipStream_t)stream;
    const int nb = head_blocks((long long)n * hw);
    float* pw = (float*)workspace;
    float* pb = pw + (size_t)nb * hc * HEAD_CIN;
    int rc = by_dtype(h.dtype, [&](auto* tag) {
        using T = std::remove_pointer_t<decltype(tag)>;
        DBSR_HEAD_HC(hc, hipLaunchKernelGGL((head_bwd_kernel<T, HC>), dim3(nb), dim3(256), 0, s, n, hw, h, dp, w, dh, pw, pb))
        DBSR_LAUNCH_CHECK();
        return 0;
    });
    if (rc) return rc;
    hipLaunchKernelGGL(sum_rows_kernel, dim3((unsigned)((hc * HEAD_CIN + 63) / 64)), dim3(256), 0, s, nb, hc * HEAD_CIN,
                       (const float*)pw, dw, accumulate, 1.0f);
    DBSR_LAUNCH_CHECK();
    if (db) {
        hipLaunchKernelGGL(sum_rows_kernel, dim3(1), dim3(256), 0, s, nb, hc, (const float*)pb, db, accumulate, 1.0f);
        DBSR_LAUNCH_CHECK();
    }
    return 0;
}
#undef DBSR_HEAD_HC

extern "C" size_t dbsr_chan_sum_workspace_bytes(int n, int hw, int c) {
    const long long total = (long long)n * hw;
    const long long nbx = std::min<long long>(1024, std::max<long long>(1, (total + 255) / 256));
    return (size_t)nbx * c * sizeof(float);
}

extern "C" int dbsr_chan_sum(int n, int hw, int c, dbsr_tensor t, float* out, int accumulate, void* workspace,
                             size_t workspace_bytes, void* stream) {
    DBSR_CHECK_ARG(map_ok(t) && out && workspace && n > 0 && hw > 0 && c > 0, "chan_sum: bad arguments");
    DBSR_CHECK_ARG(workspace_bytes >= dbsr_chan_sum_workspace_bytes(n, hw, c), "chan_sum: workspace too small");
    const long long total = (long long)n * hw;
    const int nbx = (int)std::min<long long>(1024, std::max<long long>(1, (total + 255) / 256));
    const int ppb = (int)((total + nbx - 1) / nbx);
    hipStream_t s = (hipStream_t)stream;
    const int groups = (c + 7) / 8;
    int tpp = 1;
    while (tpp < groups) tpp *= 2;
    // 16-B loads need 8-element-aligned pixels and channel slices; channels c .. groups*8 of a pixel are read
    // and summed into LDS columns that the final reduction never reads
    const bool v16 = t.dtype != DBSR_F32 && vec_ok(t, 8) && t.ld >= t.c0 + groups * 8 && tpp <= 64;
    int rc = by_dtype(t.dtype, [&](auto* tag) {
        using T = std::remove_pointer_t<decltype(tag)>;
        if constexpr (sizeof(T) == 2) {
            if (v16) {
#define DBSR_CS16(P) if (tpp == P) hipLaunchKernelGGL((chan_sum16_kernel<T, P>), dim3(nbx), dim3(256), 0, s, n, hw, c, t, ppb, (float*)workspace);
                DBSR_CS16(1) DBSR_CS16(2) DBSR_CS16(4) DBSR_CS16(8) DBSR_CS16(16) DBSR_CS16(32) DBSR_CS16(64)
#undef DBSR_CS16
                DBSR_LAUNCH_CHECK();
                return 0;
            }
        }
        hipLaunchKernelGGL((chan_sum_kernel<T>), dim3(nbx, (c + 63) / 64), dim3(256), 0, s, n, hw, c, t, ppb,
                           (float*)workspace);
        DBSR_LAUNCH_CHECK();
        return 0;
    });
    if (rc) return rc;
    hipLaunchKernelGGL(sum_rows_kernel, dim3((unsigned)((c + 63) / 64)), dim3(256), 0, s, nbx, c,
                       (const float*)workspace, out, accumulate, 1.0f);
    DBSR_LAUNCH_CHECK();
    return 0;
}

extern "C" int dbsr_l1_loss_backward(int B, int C, int H, int W, int boundary_ignore, const float* pred,
                                     const float* gt, dbsr_tensor dpre, float* loss, void* workspace,
                                     size_t workspace_bytes, void* stream) {
    DBSR_CHECK_ARG(pred && gt && loss && workspace && map_ok(dpre), "l1_loss_backward: null pointer");
    DBSR_CHECK_ARG(B > 0 && C > 0 && H > 2 * boundary_ignore && W > 2 * boundary_ignore && boundary_ignore >= 0 &&
                   dpre.ld >= dpre.c0 + C, "l1_loss_backward: bad sizes");
    const long long total = (long long)B * H * W;
    const unsigned nb = nblocks(total, 256);
    DBSR_CHECK_ARG(workspace_bytes >= nb * sizeof(float), "l1_loss_backward: workspace < %u floats", nb);
    const float count = (float)B * C * (H - 2 * boundary_ignore) * (W - 2 * boundary_ignore);
    hipStream_t s = (hipStream_t)stream;
    const bool v8 = dpre.dtype != DBSR_F32 && dpre.ld == 8 && dpre.c0 == 0 && C <= 8;
    const unsigned nb8 = nblocks(total, 1024);            // 4 pixels per thread
    int rc = by_dtype(dpre.dtype, [&](auto* tag) {
        using T = std::remove_pointer_t<decltype(tag)>;
        if constexpr (sizeof(T) == 2) {
            if (v8) {
                hipLaunchKernelGGL((l1_loss_bwd8_kernel<T>), dim3(nb8), dim3(256), 0, s, B, C, H, W, boundary_ignore,
                                   pred, gt, 1.0f / count, dpre, (float*)workspace);
                DBSR_LAUNCH_CHECK();
                return 0;
            }
        }
        hipLaunchKernelGGL((l1_loss_bwd_kernel<T>), dim3(nb), dim3(256), 0, s, B, C, H, W, boundary_ignore, pred, gt,
                           1.0f / count, dpre, (float*)workspace);
        DBSR_LAUNCH_CHECK();
        return 0;
    });
    if (rc) return rc;
    hipLaunchKernelGGL(sum_all_kernel, dim3(1), dim3(256), 0, s, (int)(v8 ? nb8 : nb), (const float*)workspace, loss,
                       1.0f / count);
    DBSR_LAUNCH_CHECK();
    return 0;
}

extern "C" int dbsr_relu_grad(int B, int C, int H, int W, const float* pred, const float* gout, dbsr_tensor dpre,
                              void* stream) {
    DBSR_CHECK_ARG(pred && gout && map_ok(dpre), "relu_grad: null pointer");
    DBSR_CHECK_ARG(B > 0 && C > 0 && H > 0 && W > 0 && dpre.ld >= dpre.c0 + C, "relu_grad: bad sizes");
    return by_dtype(dpre.dtype, [&](auto* tag) {
        using T = std::remove_pointer_t<decltype(tag)>;
        hipLaunchKernelGGL((relu_grad_kernel<T>), dim3((unsigned)(((long long)B * H * W + 255) / 256)), dim3(256), 0,
                           (hipStream_t)stream, B, C, H, W, pred, gout, dpre);
        DBSR_LAUNCH_CHECK();
        return 0;
    });
}

extern "C" int dbsr_unshuffle_gate(int B, int H, int W, int s, int c, dbsr_tensor ds, dbsr_tensor gate, dbsr_tensor du,
                                   void* stream) {
    DBSR_CHECK_ARG(map_ok(ds) && map_ok(gate) && map_ok(du) && ds.dtype == gate.dtype && ds.dtype == du.dtype,
                   "unshuffle_gate: bad tensors");
    DBSR_CHECK_ARG(B > 0 && H > 0 && W > 0 && s > 0 && c > 0 && du.ld >= du.c0 + c * s * s, "unshuffle_gate: sizes");
    const long long total = (long long)B * H * W * c * s * s;
    const int K = c * s * s;
    const bool v16 = ds.dtype != DBSR_F32 && c % 8 == 0 && vec_ok(ds, 8) && vec_ok(gate, 8) && vec_ok(du, 8) &&
                     K % 8 == 0 && K * 2 <= 32768;
    return by_dtype(ds.dtype, [&](auto* tag) {
        using T = std::remove_pointer_t<decltype(tag)>;
        if constexpr (sizeof(T) == 2) {
            if (v16) {
                const long long npix = (long long)B * H * W;
                hipLaunchKernelGGL((unshuffle_gate16_kernel<T>), dim3((unsigned)std::min<long long>(npix, 65536)),
                                   dim3(256), K * 2, (hipStream_t)stream, B, H, W, s, c, ds, gate, du);
                DBSR_LAUNCH_CHECK();
                return 0;
            }
        }
        hipLaunchKernelGGL((unshuffle_gate_kernel<T>), dim3(nblocks(total, 256)), dim3(256), 0, (hipStream_t)stream, B,
                           H, W, s, c, ds, gate, du);
        DBSR_LAUNCH_CHECK();
        return 0;
    });
}

extern "C" int dbsr_fuse_backward(int B, int N, int hw, int c, dbsr_tensor weights, dbsr_tensor ref, dbsr_tensor oth,
                                  dbsr_tensor fused, dbsr_tensor dfused, dbsr_tensor dlogits, dbsr_tensor dref,
                                  dbsr_tensor doth, void* stream) {
    DBSR_CHECK_ARG(map_ok(weights) && map_ok(ref) && map_ok(fused) && map_ok(dfused) && map_ok(dlogits) &&
                   map_ok(dref) && (N == 1 || (map_ok(oth) && map_ok(doth))), "fuse_backward: bad tensors");
    DBSR_CHECK_ARG(B > 0 && N > 0 && hw > 0 && c % 8 == 0, "fuse_backward: c must be a multiple of 8");
    const dbsr_tensor* ts[] = {&weights, &ref, &fused, &dfused, &dlogits, &dref};
    for (auto* t : ts) DBSR_CHECK_ARG(t->dtype == ref.dtype && vec_ok(*t, 8), "fuse_backward: dtype/layout");
    const long long total = (long long)B * hw * (c / 8);
    DBSR_CHECK_ARG(total < (1LL << 31), "fuse_backward: B * hw * c / 8 must be < 2^31");
    return by_dtype(ref.dtype, [&](auto* tag) {
        using T = std::remove_pointer_t<decltype(tag)>;
        hipLaunchKernelGGL((fuse_bwd_kernel<T>), dim3(nblocks(total, 256)), dim3(256), 0, (hipStream_t)stream, B, N, hw,
                           c, weights, ref, oth, fused, dfused, dlogits, dref, doth);
        DBSR_LAUNCH_CHECK();
        return 0;
    });
}

extern "C" int dbsr_merge_prep_backward(int B, int N, int hw, int c, dbsr_tensor dwp, dbsr_tensor proj,
                                        dbsr_tensor dproj, void* stream) {
    DBSR_CHECK_ARG(map_ok(dwp) && map_ok(proj) && map_ok(dproj) && dwp.dtype == proj.dtype && dproj.dtype == proj.dtype,
                   "merge_prep_backward: bad tensors");
    DBSR_CHECK_ARG(c % 8 == 0 && vec_ok(dwp, 8) && vec_ok(proj, 8) && vec_ok(dproj, 8) && dwp.ld >= dwp.c0 + 2 * c,
                   "merge_prep_backward: layout");
    const long long total = (long long)B * N * hw * (c / 8);
    return by_dtype(proj.dtype, [&](auto* tag) {
        using T = std::remove_pointer_t<decltype(tag)>;
        hipLaunchKernelGGL((merge_prep_bwd_kernel<T>), dim3(nblocks(total, 256)), dim3(256), 0, (hipStream_t)stream, B,
                           N, hw, c, dwp, proj, dproj);
        DBSR_LAUNCH_CHECK();
        return 0;
    });
}

extern "C" int dbsr_warp_backward(int n, int h, int w, int c, dbsr_tensor dout, const float* flow,
                                  long long flow_img_stride, float* dfeat32, dbsr_frame_map fmap,
                                  long long dfeat_img_stride, void* stream) {
    DBSR_CHECK_ARG(map_ok(dout) && flow && dfeat32 && fmap.fpg > 0, "warp_backward: bad tensors");
    DBSR_CHECK_ARG(n > 0 && h > 0 && w > 0 && c % 8 == 0 && vec_ok(dout, 8), "warp_backward: layout");
    const long long total = (long long)n * h * w * (c / 8);
    return by_dtype(dout.dtype, [&](auto* tag) {
        using T = std::remove_pointer_t<decltype(tag)>;
        hipLaunchKernelGGL((warp_bwd_kernel<T>), dim3(nblocks(total, 256)), dim3(256), 0, (hipStream_t)stream, n, h, w,
                           c, dout, flow, flow_img_stride, dfeat32, fmap, dfeat_img_stride);
        DBSR_LAUNCH_CHECK();
        return 0;
    });
}

extern "C" int dbsr_enc_grad_gate(int B, int N, int hw, int c, dbsr_tensor dref, const float* dsrc32, dbsr_tensor e,
                                  dbsr_tensor de, void* stream) {
    DBSR_CHECK_ARG(map_ok(dref) && dsrc32 && map_ok(e) && map_ok(de) && dref.dtype == e.dtype && de.dtype == e.dtype,
                   "enc_grad_gate: bad tensors");
    DBSR_CHECK_ARG(c % 8 == 0 && vec_ok(dref, 8) && vec_ok(e, 8) && vec_ok(de, 8), "enc_grad_gate: layout");
    const long long total = (long long)B * N * hw * (c / 8);
    return by_dtype(e.dtype, [&](auto* tag) {
        using T = std::remove_pointer_t<decltype(tag)>;
        hipLaunchKernelGGL((enc_grad_gate_kernel<T>), dim3(nblocks(total, 256)), dim3(256), 0, (hipStream_t)stream, B,
                           N, hw, c, dref, dsrc32, e, de);
        DBSR_LAUNCH_CHECK();
        return 0;
    });
}

extern "C" size_t dbsr_warp_backward_gather_workspace_bytes(int n, int h, int w) {
    if (n <= 0 || h <= 0 || w <= 0) return 0;
    const long long px = (long long)n * h * w;
    return (size_t)(3 * px * sizeof(int) + 15) / 16 * 16 + (size_t)px * 4 * sizeof(int2);
}

extern "C" int dbsr_warp_backward_gather(int n, int h, int w, int c, dbsr_tensor dout, const float* flow,
                                         long long flow_img_stride, dbsr_tensor gate, dbsr_tensor dfeat,
                                         void* workspace, size_t workspace_bytes, void* stream) {
    DBSR_CHECK_ARG(map_ok(dout) && map_ok(dfeat) && flow && workspace && dout.dtype == dfeat.dtype,
                   "warp_backward_gather: bad tensors");
    DBSR_CHECK_ARG(!gate.ptr || (map_ok(gate) && gate.dtype == dfeat.dtype), "warp_backward_gather: bad gate");
    DBSR_CHECK_ARG(n > 0 && h > 0 && w > 0 && c > 0 && c % 8 == 0 && vec_ok(dout, 8) && vec_ok(dfeat, 8) &&
                   (!gate.ptr || vec_ok(gate, 8)) && (long long)h * w * 4 < (1LL << 31),
                   "warp_backward_gather: c, ld and c0 must be multiples of 8");
    DBSR_CHECK_ARG((long long)n * h * w < (1LL << 31), "warp_backward_gather: n * h * w must be < 2^31");
    DBSR_CHECK_ARG(workspace_bytes >= dbsr_warp_backward_gather_workspace_bytes(n, h, w),
                   "warp_backward_gather: workspace %zu < %zu bytes", workspace_bytes,
                   dbsr_warp_backward_gather_workspace_bytes(n, h, w));
    const long long px = (long long)n * h * w;
    int* counts = (int*)workspace;
    int* offsets = counts + px;
    int* cursor = offsets + px;
    int2* records = (int2*)((char*)workspace + (3 * px * sizeof(int) + 15) / 16 * 16);
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(zero_ints_kernel, dim3(nblocks(px, 256)), dim3(256), 0, s, px, counts);
    hipLaunchKernelGGL(wb_count_kernel, dim3(nblocks(px, 256)), dim3(256), 0, s, n, h, w, flow, flow_img_stride, counts);
    hipLaunchKernelGGL(wb_scan_kernel, dim3(n), dim3(1024), 0, s, h * w, counts, offsets, cursor);
    hipLaunchKernelGGL(wb_scatter_kernel, dim3(nblocks(px, 256)), dim3(256), 0, s, n, h, w, flow, flow_img_stride,
                       cursor, records);
    DBSR_LAUNCH_CHECK();
    return by_dtype(dout.dtype, [&](auto* tag) {
        using T = std::remove_pointer_t<decltype(tag)>;
        hipLaunchKernelGGL((wb_gather_kernel<T>), dim3(nblocks(px, 4)), dim3(256), 0, s, n, h, w, c, dout, counts,
                           offsets, records, gate, dfeat);
        DBSR_LAUNCH_CHECK();
        return 0;
    });
}

extern "C" int dbsr_gate_copy(int n, int hw, int c, dbsr_tensor in, dbsr_tensor gate, dbsr_tensor out, void* stream) {
    DBSR_CHECK_ARG(map_ok(in) && map_ok(gate) && map_ok(out) && in.dtype == gate.dtype && out.dtype == in.dtype,
                   "gate_copy: bad tensors");
    DBSR_CHECK_ARG(n > 0 && hw > 0 && c % 8 == 0 && vec_ok(in, 8) && vec_ok(gate, 8) && vec_ok(out, 8),
                   "gate_copy: layout");
    const long long total = (long long)n * hw * (c / 8);
    return by_dtype(in.dtype, [&](auto* tag) {
        using T = std::remove_pointer_t<decltype(tag)>;
        hipLaunchKernelGGL((gate_copy_kernel<T>), dim3(nblocks(total, 256)), dim3(256), 0, (hipStream_t)stream, n, hw,
                           c, in, gate, out);
        DBSR_LAUNCH_CHECK();
        return 0;
    });
}

extern "C" int dbsr_adam_step(long long n, float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                              float lr, float beta1, float beta2, float eps, int step, float grad_scale,
                              void* stream) {
    DBSR_CHECK_ARG(n > 0 && param && grad && exp_avg && exp_avg_sq && step >= 1, "adam_step: bad arguments");
    const float bc1 = 1.f - powf(beta1, (float)step), bc2 = 1.f - powf(beta2, (float)step);
    hipLaunchKernelGGL(adam_kernel, dim3(nblocks(n, 256)), dim3(256), 0, (hipStream_t)stream, n, param, grad, exp_avg,
                       exp_avg_sq, lr, beta1, beta2, eps, bc1, sqrtf(bc2), grad_scale);
    DBSR_LAUNCH_CHECK();
    return 0;
}

extern "C" int dbsr_dgrad_weights(const float* w, int cout, int cin, int kh, int kw, float* wt, void* stream) {
    DBSR_CHECK_ARG(w && wt && cout > 0 && cin > 0 && kh > 0 && kw > 0, "dgrad_weights: bad arguments");
    const long long total = (long long)cout * cin * kh * kw;
    hipLaunchKernelGGL(dgrad_weights_kernel, dim3(nblocks(total, 256)), dim3(256), 0, (hipStream_t)stream, w, cout, cin,
                       kh, kw, wt);
    DBSR_LAUNCH_CHECK();
    return 0;
}
