// The K-split weight-stationary 3x3 conv for 128 -> 128 channels (dbsr_conv2d picks it; the selection is in
// conv2d.hip).  Its own translation unit so the kernel builds in seconds.
#include "conv_core.hpp"

#include <algorithm>

namespace dbsr {

// ------------------------------------------------------------------------------------------------
// 128 -> 128 3x3/s1/p1 conv with both operands' reuse on chip: the weight predictor's input conv and its
// ResBlocks (merging.py:86-90, 98-101: seven 128-channel convs over every frame of the burst, ~71 GFLOP each at the
// bench shape).  The pipelined kernel streams a 64-cout tile's weights through the LDS with every 48 x 8 tile (one
// 1-KiB LDS-DMA piece per ~200 FLOP); the weight-stationary kernel's registers hold a whole cout tile only for
// Cin <= 64.  Here the eight waves of a block split the 128 x 1152 weight matrix into 4 cout quarters x 2 K halves:
// wave (kh, q) holds couts 32q .. 32q + 31 over input channels 64kh .. 64kh + 63 (2 chunks x 9 taps x 2 16-cout
// blocks of A-fragments, 144 VGPRs, loaded once), so only the tile's halo moves through the LDS (one piece per
// ~820 FLOP).  Waves kh = 0 / 1 of a quarter share a SIMD (waves w, w + 4).
//
// Per 16 x 8 output tile (8 groups of 16 pixels = the tile's rows): the 18 x 10-pixel halo of all 128 channels is
// LDS-DMA'd one tile ahead into a double buffer (halo_phys swizzle; chunk images 184 pixels apart so the swizzle
// parity is the chunk-local one; out-of-frame pixels land zeros).  Every wave runs its K half's 18 k-steps for all
// 8 groups in batches of NB, the partner's four groups first: their fp32 partial sums go to an LDS exchange area,
// its own four stay in registers.  One barrier, then wave (kh, q) adds the partner's partials to its own groups
// (rows 4kh .. 4kh + 3), applies bias / act / residual / act and stores 8 consecutive couts per lane (16 B).
// Hand-scheduled LDS reads as in the fused ResBlock kernels: each group's B-fragment for k-step s + 2 is read by
// inline asm right behind its MFMAs of step s, and each MFMA pair waits only for its own read.
// The sum of a pixel is (K half 0) + (K half 1), each an in-order chunk-major fp32 MFMA chain from zero, then the
// bias: the same value whichever wave of the pair adds it (fp32 addition commutes).
// Block -> tiles: rb_tile (a full round of 256 tiles XCD-contiguous); grid = min(CUs or cap, tiles).
// ------------------------------------------------------------------------------------------------
namespace ks128 {
constexpr int HW = TW + 2, HH = TH + 2, HPX = HW * HH;       // halo 18 x 10 = 180 pixels
constexpr int CPX = 184;                                      // pixel slots per chunk image (a multiple of 8)
constexpr int NCH = 4;                                        // 32-channel chunks
constexpr int CH_U4 = CPX * 4;                                // 16-B slots per chunk image
constexpr int PIECES = NCH * CPX / 16;                        // 46 1-KiB halo pieces per tile
constexpr int BUF_U4 = NCH * CH_U4;                           // one halo buffer (47,104 B)
constexpr int NW = 8;
constexpr int PER = (PIECES + NW - 1) / NW;                   // DMA pieces per wave per tile
#ifndef DBSR_KS_NB                                            // (experiment builds: tools/build_variant.sh)
#define DBSR_KS_NB 2
#endif
#ifndef DBSR_KS_ABL                                           // timing-only ablations: 1 no k-steps, 2 no halo DMA
#define DBSR_KS_ABL 0                                         // after the first tile, 4 no partial-sum exchange
#endif
#ifndef DBSR_KS_RING
#define DBSR_KS_RING 3
#endif
constexpr int NB = DBSR_KS_NB;                                // 16-pixel groups per MFMA batch
constexpr int RING = DBSR_KS_RING;                            // B-fragment ring depth: reads RING - 1 k-steps ahead
constexpr int HALF = TH / 2;                                  // groups a wave finishes (4)
constexpr int XCH_U4 = NW * HALF * 2 * 64;                    // exchange: [wave][group][16-cout block][lane]
constexpr int LDS_U4 = 2 * BUF_U4 + XCH_U4;
static_assert(LDS_U4 * 16 + 128 * 4 <= 160 * 1024, "ks128 LDS");
static_assert(CPX % 8 == 0 && CPX >= HPX && (NCH * CPX) % 16 == 0, "chunk images");
static_assert(HALF % NB == 0, "batches");
}  // namespace ks128

template <typename T, int EPI>
__global__ __launch_bounds__(512, 1) void conv3x3_ks128_kernel(ConvK k, int tiles_x, int tiles_y, int ntiles) {
    using namespace ks128;
    DBSR_OWN_SIMDS();
    __shared__ __attribute__((aligned(16))) u32x4_t lds[LDS_U4 + 32];
    u32x4_t* xch = lds + 2 * BUF_U4;
    float* lbias = (float*)(lds + LDS_U4);
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int kh = wave >> 2, q = wave & 3;
    const int H = k.in_h, W = k.in_w;
    // epilogues (the pipelined kernel's): 1 bias + ReLU, 2 bias + residual then ReLU, 3 bias, 0 run-time act /
    // residual / post-act, 5 as 0 then the training dgrad's ReLU-backward gate (out *= gate > 0)
    constexpr bool RT = EPI == 0 || EPI == 5, has_gate = EPI == 5;
    const bool has_res = EPI == 2 || (RT && k.r != nullptr);
    auto act1 = [&](float v) {
        if constexpr (EPI == 1) return fmaxf(v, 0.f);
        else if constexpr (RT) return apply_act(v, k.act);
        else return v;
    };
    auto act2 = [&](float v) {
        if constexpr (EPI == 2) return fmaxf(v, 0.f);
        else if constexpr (RT) return apply_act(v, k.post_act);
        else return v;
    };

    // this wave's A-fragments: piece ((16-cout block) * 4 + chunk) * 9 + tap of the chunk-major copy
    Frag<T> w[2][9][2];
    {
        const char* wsrc = (const char*)k.w_pipe;
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
            for (int tap = 0; tap < 9; ++tap)
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    w[c][tap][h].load((const T*)(wsrc + (((2 * q + h) * NCH + 2 * kh + c) * 9 + tap) * 1024 + lane * 16));
    }
    if (threadIdx.x < 128) lbias[threadIdx.x] = k.bias ? k.bias[threadIdx.x] : 0.f;   // (cout == 128) ordered by the
                                                                                      // loop's first barrier
    struct Tile { const T* xf; long long y_off, r_off, g_off; int y0, x0; };
    auto decode = [&](int i) {
        const int t = rb_tile(i, blockIdx.x, gridDim.x, ntiles);
        const int tx = t % tiles_x, r = t / tiles_x, ty = r % tiles_y, f = r / tiles_y;
        Tile tl;
        tl.y0 = ty * TH; tl.x0 = tx * TW;
        tl.xf = (const T*)k.x + map_frame(k.xm, f) * k.x_is;
        const long long pix = (long long)tl.y0 * k.out_w + tl.x0;
        tl.y_off = map_frame(k.ym, f) * k.y_is + k.y_c0 + pix * k.y_ld;
        tl.r_off = has_res ? map_frame(k.rm, f) * k.r_is + k.r_c0 + pix * k.r_ld : 0;
        tl.g_off = has_gate ? map_frame(k.gm, f) * k.g_is + k.g_c0 + pix * k.g_ld : 0;
        return tl;
    };
    const int my_tiles = ntiles / (int)gridDim.x + ((int)blockIdx.x < ntiles % (int)gridDim.x ? 1 : 0);

    // halo DMA: piece `it` of this wave is item wave + 8 it (clamped: surplus slots rewrite the last piece with
    // identical bytes); lane -> (chunk, halo pixel, physical k-group slot), tile-invariant
    const int pix_b = k.x_ld * (int)sizeof(T);
    const unsigned frame_bytes = (unsigned)((long long)H * W * pix_b);
    const unsigned lds0 = (unsigned)(unsigned long long)(__attribute__((address_space(3))) u32x4_t*)lds;
    int h_rc[PER], h_off[PER];
#pragma unroll
    for (int it = 0; it < PER; ++it) {
        const int item = min(wave + NW * it, PIECES - 1);
        const int qq = item * 16 + (lane >> 2), c = qq / CPX, p = qq - c * CPX, ph = lane & 3;
        const int gg = 2 * ((ph & 1) ^ ((p >> 2) & 1)) + (ph >> 1);
        const int r = p / HW, cc = p - r * HW;
        h_rc[it] = p < HPX ? (r << 16) | cc : 0x7fff7fff;        // pixel slots past the halo land zeros
        h_off[it] = (r * W + cc) * pix_b + c * 64 + gg * 16;
    }
    auto dma = [&](int it, const Tile& tl, int buf) {
        const int item = min(wave + NW * it, PIECES - 1);
        const int hy = tl.y0 - 1 + (h_rc[it] >> 16), hx = tl.x0 - 1 + (h_rc[it] & 0xffff);
        const bool ok = (unsigned)hy < (unsigned)H && (unsigned)hx < (unsigned)W;
        const int base = ((tl.y0 - 1) * W + (tl.x0 - 1)) * pix_b;
        lds_dma16(tl.xf, frame_bytes, ok ? base + h_off[it] : BUF_OOB, 0,
                  lds0 + (unsigned)((buf * BUF_U4 + item * 64) * 16));
    };

    // the 18 k-steps of this wave's K half for groups J0 .. J0 + NB - 1 (tile rows) of halo buffer `buf`; `hook(st)`
    // runs after k-step st's MFMAs (the DMA pieces of the next tile)
    auto taps = [&](int buf, auto j0_, f32x4_t (&acc)[NB][2], auto&& hook) {
        constexpr int J0 = decltype(j0_)::value, NS = 18;
        if constexpr ((DBSR_KS_ABL & 1) != 0) {
            for (int j = 0; j < NB; ++j) acc[j][0] = acc[j][1] = f32x4_t{(float)(J0 + j + buf), 0.f, 0.f, 0.f};
            StaticFor<0, NS>::run([&](auto s_) { hook(decltype(s_)::value); });
            return;
        }
        const int g = lane >> 4, col = lane & 15;
        const unsigned base = lds0 + (unsigned)((buf * BUF_U4 + kh * 2 * CH_U4) * 16);
        unsigned ba[8];                 // byte address of pixel col + rho, k-group g (halo_phys), rho = imm & 7
#pragma unroll
        for (int rho = 0; rho < 8; ++rho) ba[rho] = base + 16u * (4 * col + halo_phys(col + rho, g));
        Frag<T> bq[NB][RING];
        constexpr int AH = RING - 1;
        auto rd = [&](auto j_, auto st_) {
            constexpr int j = decltype(j_)::value, st = decltype(st_)::value;
            constexpr int c = st / 9, tap = st % 9, imm = (J0 + j + tap / 3) * HW + tap % 3;
            // (asm operands name this lambda's own locals: clang does not capture for asm operands)
            const unsigned a = ba[imm & 7];
            bf16x8_t v;
            asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(a), "i"(16 * (c * CH_U4 + 4 * imm)));
            bq[j][st % RING].v = v;
        };
        StaticFor<0, AH>::run([&](auto s0_) {
            StaticFor<0, NB>::run([&](auto j_) { rd(j_, s0_); });
        });
        StaticFor<0, NS>::run([&](auto s_) {
            constexpr int st = decltype(s_)::value, c = st / 9, tap = st % 9;
            const f32x4_t z = {0.f, 0.f, 0.f, 0.f};
            StaticFor<0, NB>::run([&](auto j_) {
                constexpr int j = decltype(j_)::value;
                // reads issued after R(st, j): R(st, j' > j), R(st + 1 .. st + AH - 1, all), R(st + AH, j' < j)
                constexpr int mid = (AH - 1 < NS - 1 - st) ? AH - 1 : NS - 1 - st;
                constexpr int newer = (NB - 1 - j) + NB * mid + (st + AH < NS ? j : 0);
                bf16x8_t v = bq[j][st % RING].v;
                asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(v) : "i"(newer));
                bq[j][st % RING].v = v;
                acc[j][0] = mma(w[c][tap][0], bq[j][st % RING], st == 0 ? z : acc[j][0]);
                acc[j][1] = mma(w[c][tap][1], bq[j][st % RING], st == 0 ? z : acc[j][1]);
                if constexpr (st + AH < NS) rd(j_, std::integral_constant<int, st + AH>{});
            });
            hook(st);
        });
    };

    Tile cur = decode(0);
    if (my_tiles > 0) {
#pragma unroll
        for (int it = 0; it < PER; ++it) dma(it, cur, 0);
    }
    const int own0 = HALF * kh;         // first row of this wave's groups (the partner's: HALF - own0)
    for (int ti = 0; ti < my_tiles; ++ti) {
        // this wave's DMA pieces of tile ti landed (the youngest vector-memory ops, the HALF output stores of tile
        // ti - 1, may stay in flight), then everyone's
        if (ti == 0) vm_drain();
        else DBSR_VM_WAIT(HALF);
        __syncthreads();
        const bool more = ti + 1 < my_tiles;
        const Tile nxt = more ? decode(ti + 1) : cur;
        const int buf = ti & 1;
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const int g = ln >> 4, col = ln & 15;
        // ---- the partner's groups: k-steps, the next tile's halo DMA spread over the first batch, partials out ----
        StaticFor<0, HALF / NB>::run([&](auto b_) {
            constexpr int b = decltype(b_)::value;
            f32x4_t acc[NB][2];
            auto hook = [&](int st) {
                if constexpr (b == 0 && (DBSR_KS_ABL & 2) == 0) {     // (ablation 2: stale halos after tile 0)
                    if (more) {
#pragma unroll
                        for (int it = 0; it < PER; ++it)
                            if (st == 2 * it + 1) dma(it, nxt, buf ^ 1);
                    }
                }
            };
            if (kh == 0) taps(buf, std::integral_constant<int, HALF + NB * b>{}, acc, hook);
            else taps(buf, std::integral_constant<int, NB * b>{}, acc, hook);
#pragma unroll
            for (int j = 0; j < NB; ++j)
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    if constexpr ((DBSR_KS_ABL & 4) == 0)
                        xch[((wave * HALF + NB * b + j) * 2 + h) * 64 + ln] = __builtin_bit_cast(u32x4_t, acc[j][h]);
                    else if (acc[j][h][0] == 12345.f) xch[ln] = u32x4_t{0u, 0u, 0u, 0u};
        });
        // ---- this wave's own groups: residual loads, k-steps ----
        // (run-time epilogues: loaded in the epilogue beside the gate, which leaves the k-steps their registers)
        u32x4_t resv[HALF];
        auto load_res = [&]() {
#pragma unroll
            for (int j = 0; j < HALF; ++j)
                resv[j] = *(const u32x4_t*)((const T*)k.r + cur.r_off + ((long long)(own0 + j) * k.out_w + col) * k.r_ld +
                                            32 * q + 8 * g);
        };
        if (!RT && has_res) load_res();
        f32x4_t mine[HALF][2];
        StaticFor<0, HALF / NB>::run([&](auto b_) {
            constexpr int b = decltype(b_)::value;
            f32x4_t acc[NB][2];
            auto hook = [&](int) {};
            if (kh == 0) taps(buf, std::integral_constant<int, NB * b>{}, acc, hook);
            else taps(buf, std::integral_constant<int, HALF + NB * b>{}, acc, hook);
#pragma unroll
            for (int j = 0; j < NB; ++j) {
                mine[NB * b + j][0] = acc[j][0];
                mine[NB * b + j][1] = acc[j][1];
            }
        });
        // the partials of every wave are in the exchange area; the next tile's halo pieces and this tile's residual
        // loads (issued a batch or more earlier) are drained first, so no LDS-DMA is in flight at any barrier
        if constexpr ((DBSR_KS_ABL & 4) == 0) dma_barrier();
        // ---- epilogue of rows own0 .. own0 + HALF - 1: + partner partials, bias, act, residual, act, 16-B stores ----
        const int partner = wave ^ 4;
        const float4 b0 = *(const float4*)(lbias + 32 * q + 8 * g), b1 = *(const float4*)(lbias + 32 * q + 8 * g + 4);
        const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
        if (RT && has_res) load_res();
        u32x4_t gatev[has_gate ? HALF : 1];     // EPI 5: the gate, all pieces in flight at once
        if constexpr (has_gate) {
#pragma unroll
            for (int j = 0; j < HALF; ++j)
                gatev[j] = *(const u32x4_t*)((const T*)k.gt + cur.g_off + ((long long)(own0 + j) * k.out_w + col) * k.g_ld +
                                             32 * q + 8 * g);
        }
#pragma unroll
        for (int j = 0; j < HALF; ++j) {
            f32x4_t o0 = {0.f, 0.f, 0.f, 0.f}, o1 = o0;
            if constexpr ((DBSR_KS_ABL & 4) == 0) {
                o0 = __builtin_bit_cast(f32x4_t, xch[((partner * HALF + j) * 2 + 0) * 64 + ln]);
                o1 = __builtin_bit_cast(f32x4_t, xch[((partner * HALF + j) * 2 + 1) * 64 + ln]);
            }
            float v[8];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                v[r] = act1((mine[j][0][r] + o0[r]) + bv[r]);
                v[4 + r] = act1((mine[j][1][r] + o1[r]) + bv[4 + r]);
            }
            if (has_res) {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    v[2 * e] = act2(v[2 * e] + H16<T>::lo(resv[j][e]));
                    v[2 * e + 1] = act2(v[2 * e + 1] + H16<T>::hi(resv[j][e]));
                }
            }
            if constexpr (has_gate) {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    v[2 * e] = H16<T>::lo(gatev[j][e]) > 0.f ? v[2 * e] : 0.f;
                    v[2 * e + 1] = H16<T>::hi(gatev[j][e]) > 0.f ? v[2 * e + 1] : 0.f;
                }
            }
            u32x4_t o;
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = H16<T>::pack(v[2 * e], v[2 * e + 1]);
            *(u32x4_t*)((T*)k.y + cur.y_off + ((long long)(own0 + j) * k.out_w + col) * k.y_ld + 32 * q + 8 * g) = o;
        }
        cur = nxt;
    }
    vm_drain();                         // (no LDS-DMA outstanding at s_endpgm: tools/isa_audit.py)
}

// a 128 -> 128 conv of n_frames frames (multiples of 16 x 8) on grid = min(cap or CUs, tiles) persistent blocks
int ks128_launch(const ConvK& k, int n_frames, bool f16, int epi, int max_blocks, int cus, hipStream_t s) {
    const int tiles_x = k.out_w / ks128::TW, tiles_y = k.out_h / ks128::TH;
    const long long nt = (long long)n_frames * tiles_x * tiles_y;
    DBSR_CHECK_ARG(nt > 0 && nt < (1LL << 31), "conv2d: bad tile count for the K-split 128-channel kernel");
    const int ntiles = (int)nt;
    int grid = max_blocks > 0 ? std::min(max_blocks, cus) : cus;
    grid = std::min(grid, ntiles);
    DBSR_CHECK_ARG(rb_mapping_ok(grid, ntiles), "conv2d: tile mapping out of range (grid %d, %d tiles)", grid, ntiles);
#define DBSR_KS_LAUNCH(TT, E) \
    hipLaunchKernelGGL((conv3x3_ks128_kernel<TT, E>), dim3(grid), dim3(512), 0, s, k, tiles_x, tiles_y, ntiles)
#define DBSR_KS_EPI(TT)                          \
    switch (epi) {                               \
        case 1: DBSR_KS_LAUNCH(TT, 1); break;    \
        case 2: DBSR_KS_LAUNCH(TT, 2); break;    \
        case 3: DBSR_KS_LAUNCH(TT, 3); break;    \
        case 5: DBSR_KS_LAUNCH(TT, 5); break;    \
        default: DBSR_KS_LAUNCH(TT, 0); break;   \
    }
    if (f16) {
        DBSR_KS_EPI(f16_t)
    } else {
        DBSR_KS_EPI(bf16_t)
    }
#undef DBSR_KS_EPI
#undef DBSR_KS_LAUNCH
    DBSR_LAUNCH_CHECK();
    return 0;
}

}  // namespace dbsr
