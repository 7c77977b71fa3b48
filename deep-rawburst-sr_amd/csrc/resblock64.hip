// The fused 64-channel ResBlock kernel (dbsr_resblock for C = 64; the entry point and its checks are in
// conv2d.hip).  Its own translation unit so the kernel builds in seconds.
#include "conv_core.hpp"

#include <algorithm>

namespace dbsr {

// ------------------------------------------------------------------------------------------------
// Fused 64-channel ResBlock (blocks.py:81-96: y = relu(x + conv2(relu(conv1(x))))): the frame encoder's ResBlocks
// (encoders.py:36-46, 66-72), the offset-feature extractor's (merging.py:85-87) and the decoder's pre-ResBlocks
// (decoders.py:41-44) -- 15 of the forward's 16 weight-stationary conv pairs.  Per block of the
// two-launch path (conv3x3_ws_kernel x 2) the intermediate makes one HBM round trip and each launch pays its own
// 7.5k-cycle weight prologue and per-tile barrier skew; here the intermediate stays in the LDS.
//
// Two wave roles, pipelined over the block's tiles (16 x 8 output pixels each): waves 0-3 (one per SIMD) run conv1
// of tile i, waves 4-7 (the other wave of each SIMD) run conv2 of tile i - 1 and stream the halos.  A wave holds
// only its own conv's A-fragments for its 32 couts (144 VGPRs, the weight-stationary kernel's budget: both convs'
// 288 in one wave did not leave the allocator room for the B-fragment ring, and every MFMA pair then waited on its
// own LDS read), and each SIMD's two waves hide each other's LDS latency.  Wave (role, wc, wp): couts 32 wc .. 32 wc
// + 31 x the pixel groups of parity wp.  LDS: a 3-deep ring of input halos (20 x 12 pixels x 64 channels, the
// halo_phys swizzle of the weight-stationary kernel, LDS-DMA'd one tile ahead by the conv2 waves, out-of-frame
// pixels land zeros) and a 2-deep ring of intermediates (the 18 x 10 conv1 region, 12 flattened 16-pixel groups:
// 1.5x the output's 8).  One barrier per tile: after it, conv1 reads halo i % 3 and writes relu(conv1 + b1) rounded
// to T -- zeros outside the frame, conv2's padding -- into intermediate i & 1, while conv2 reads intermediate
// (i - 1) & 1, adds b2 and the residual (the centre of halo (i - 1) % 3) and stores relu(...).  Groups run in
// batches of 2 (4 MFMAs per k-step), their LDS reads two k-steps ahead.  Each output is the arithmetic of
// conv3x3_ws_kernel's epilogues 1 and 2 (k-steps chunk-major from zero, the bias after, the residual after the
// bias), so the result is bitwise that of the two dbsr_conv2d launches.
// ------------------------------------------------------------------------------------------------
namespace rb64 {
constexpr int MW = TW + 2, MH = TH + 2, MPX = MW * MH;        // conv1 region 18 x 10
constexpr int IW = TW + 4, IH = TH + 4, IPX = IW * IH;        // input halo 20 x 12
constexpr int NCH = 2;                                        // 32-channel chunks
constexpr int IN_PIECES = (IPX + 15) / 16;                    // 15 1-KiB pieces per chunk
constexpr int IN_CH_U4 = IN_PIECES * 64;                      // one chunk's halo image, 16-B slots
constexpr int IN_U4 = NCH * IN_CH_U4;
constexpr int G1 = (MPX + 15) / 16;                           // 12 conv1 groups
constexpr int MID_CH_U4 = G1 * 16 * 4;
constexpr int MID_U4 = NCH * MID_CH_U4;
constexpr int NHALO = 3, NMID = 2;                            // ring depths
constexpr int NW = 8;                                         // 4 conv1 + 4 conv2 waves
constexpr int Q1 = G1 / 2;                                    // conv1 groups per wave (6)
constexpr int Q2 = TH / 2;                                    // conv2 groups (= tile rows) per wave (4)
#ifndef DBSR_RB64_RB1                                         // (experiment builds: tools/build_variant.sh)
#define DBSR_RB64_RB1 3
#define DBSR_RB64_RB2 4
#endif
#ifndef DBSR_RB64_DMA_ALL
#define DBSR_RB64_DMA_ALL 0
#endif
#ifndef DBSR_RB64_ABL                                         // timing-only ablations (tools/gpu_rb64_ab.sh):
#define DBSR_RB64_ABL 0                                       // 1 no conv1 taps, 2 no conv2 taps, 4 no halo DMA
#endif
constexpr int RB1 = DBSR_RB64_RB1, RB2 = DBSR_RB64_RB2;       // groups per MFMA batch (conv1, conv2)
constexpr bool DMA_ALL = DBSR_RB64_DMA_ALL;                   // halo DMA by all 8 waves (else by the conv2 waves)
constexpr int NDW = DMA_ALL ? 8 : 4;                          // DMA waves
constexpr int PER = (NCH * IN_PIECES + NDW - 1) / NDW;        // halo DMA pieces per DMA wave per tile
constexpr int LDS_U4 = NHALO * IN_U4 + NMID * MID_U4;
static_assert(LDS_U4 * 16 + 128 * 4 <= 160 * 1024, "resblock64 LDS");
static_assert(Q1 % RB1 == 0 && Q2 % RB2 == 0 && TW == 16, "batches");
}  // namespace rb64

template <typename T>
__global__ __launch_bounds__(512, 1) void resblock64_kernel(ConvK k1, ConvK k2, int tiles_x, int tiles_y, int ntiles) {
    using namespace rb64;
    DBSR_OWN_SIMDS();
    __shared__ __attribute__((aligned(16))) u32x4_t lds[LDS_U4 + 32];
    u32x4_t* lmid = lds + NHALO * IN_U4;
    float* lbias = (float*)(lds + LDS_U4);                        // [b1 (64)][b2 (64)]
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int role = wave >> 2, wc = wave & 1, wp = (wave >> 1) & 1;
    const int H = k1.in_h, W = k1.in_w;

    // this wave's conv's A-fragments: piece ((2 wc + h) * 2 + c) * 9 + tap of the chunk-major copy (16-cout block
    // 2 wc + h of the 64-cout tile, chunk c), lane-major 1 KiB
    Frag<T> w[NCH][9][2];
    {
        const char* wsrc = (const char*)(role ? k2.w_pipe : k1.w_pipe);
#pragma unroll
        for (int c = 0; c < NCH; ++c)
#pragma unroll
            for (int tap = 0; tap < 9; ++tap)
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    w[c][tap][h].load((const T*)(wsrc + (((2 * wc + h) * NCH + c) * 9 + tap) * 1024 + lane * 16));
    }
    if (threadIdx.x < 128) {            // ordered before its first read (an epilogue) by the loop's first barrier
        const ConvK& kb = threadIdx.x < 64 ? k1 : k2;
        lbias[threadIdx.x] = kb.bias ? kb.bias[threadIdx.x & 63] : 0.f;
    }

    struct Tile { const T* xf; long long y_off; int y0, x0; };
    auto decode = [&](int i) {
        const int t = rb_tile(i, blockIdx.x, gridDim.x, ntiles);
        Tile tl;
        const int tx = t % tiles_x, r = t / tiles_x, ty = r % tiles_y, f = r / tiles_y;
        tl.y0 = ty * TH; tl.x0 = tx * TW;
        tl.xf = (const T*)k1.x + map_frame(k1.xm, f) * k1.x_is;
        tl.y_off = map_frame(k2.ym, f) * k2.y_is + k2.y_c0 + ((long long)tl.y0 * W + tl.x0) * k2.y_ld;
        return tl;
    };
    const int my_tiles = ntiles / (int)gridDim.x + ((int)blockIdx.x < ntiles % (int)gridDim.x ? 1 : 0);
    const int pix_b = k1.x_ld * (int)sizeof(T);
    const unsigned frame_bytes = (unsigned)((long long)H * W * pix_b);
    const unsigned lds0 = (unsigned)(unsigned long long)(__attribute__((address_space(3))) u32x4_t*)lds;
    // a tile's halo (both chunks) into ring slot buf, by the conv2 waves: inline-asm LDS-DMA (lds_dma16), drained
    // before the next barrier
    auto dma = [&](const Tile& tl, int buf) {
        if constexpr ((DBSR_RB64_ABL & 4) != 0) return;
        int ln = lane;
        asm volatile("" : "+v"(ln));
#pragma unroll
        for (int it = 0; it < PER; ++it) {
            const int item = min((DMA_ALL ? wave : wave - 4) + NDW * it, NCH * IN_PIECES - 1);
            const int cch = item / IN_PIECES, piece = item - cch * IN_PIECES;
            const int p = piece * 16 + (ln >> 2), ph = ln & 3;
            const int gg = 2 * ((ph & 1) ^ ((p >> 2) & 1)) + (ph >> 1);
            const int r = p / IW, c = p - r * IW;
            const int hy = tl.y0 - 2 + r, hx = tl.x0 - 2 + c;
            const bool ok = (unsigned)hy < (unsigned)H && (unsigned)hx < (unsigned)W;     // (p < IPX: 240 = 15 x 16)
            lds_dma16(tl.xf, frame_bytes, ok ? (hy * W + hx) * pix_b + cch * 64 + gg * 16 : BUF_OOB, 0,
                      lds0 + (buf * IN_U4 + cch * IN_CH_U4 + piece * 64) * 16);
        }
    };

    // the 18 k-steps (chunk-major, taps 0..8) of NB 16-pixel groups of an image iw pixels wide (chunk images ch_u4
    // slots apart; group j's tap-(0,0) pixel P0[j]).  Hand-scheduled: each group's B-fragment for k-step s + 2 is read
    // (inline-asm ds_read_b128) right behind its two MFMAs of step s, and each MFMA pair waits (s_waitcnt lgkmcnt,
    // tied to its fragment) only for its own read -- the reads that follow it in issue order may stay in flight.  With
    // compiler-visible reads the scheduler sank every read to its MFMAs and each pair waited out a full LDS latency.
    auto taps = [&](const u32x4_t* img, auto ch_, auto iw_, int g, const auto& P0, auto& acc) {
        constexpr int NB = std::extent<std::remove_reference_t<decltype(P0)>>::value;
        constexpr int NS = NCH * 9, ch_u4 = decltype(ch_)::value, iw = decltype(iw_)::value;
        const unsigned base = (unsigned)(unsigned long long)(__attribute__((address_space(3))) const u32x4_t*)img;
        unsigned ba[NB][8];             // byte address of group j's pixel P0[j] + rho, k-group g (halo_phys)
#pragma unroll
        for (int j = 0; j < NB; ++j)
#pragma unroll
            for (int rho = 0; rho < 8; ++rho) ba[j][rho] = base + 16u * (4 * P0[j] + halo_phys(P0[j] + rho, g));
        Frag<T> bq[NB][3];
        auto rd = [&](auto j_, auto st_) {
            constexpr int j = decltype(j_)::value, st = decltype(st_)::value;
            constexpr int c = st / 9, tap = st % 9, imm = (tap / 3) * iw + tap % 3;
            // (asm operands name this lambda's own locals: clang does not capture for asm operands)
            const unsigned a = ba[j][imm & 7];
            bf16x8_t v;
            asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(a), "i"(16 * (c * ch_u4 + 4 * imm)));
            bq[j][st % 3].v = v;
        };
        StaticFor<0, NB>::run([&](auto j_) {
            rd(j_, std::integral_constant<int, 0>{});
        });
        StaticFor<0, NB>::run([&](auto j_) {
            rd(j_, std::integral_constant<int, 1>{});
        });
        StaticFor<0, NS>::run([&](auto s_) {
            constexpr int st = decltype(s_)::value, c = st / 9, tap = st % 9;
            const f32x4_t z = {0.f, 0.f, 0.f, 0.f};
            StaticFor<0, NB>::run([&](auto j_) {
                constexpr int j = decltype(j_)::value;
                // reads issued after R(st, j): R(st, j' > j), R(st + 1, all), R(st + 2, j' < j)
                constexpr int newer = (NB - 1 - j) + (st + 1 < NS ? NB : 0) + (st + 2 < NS ? j : 0);
                bf16x8_t v = bq[j][st % 3].v;
                asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(v) : "i"(newer));
                bq[j][st % 3].v = v;
                acc[j][0] = mma(w[c][tap][0], bq[j][st % 3], st == 0 ? z : acc[j][0]);
                acc[j][1] = mma(w[c][tap][1], bq[j][st % 3], st == 0 ? z : acc[j][1]);
                if constexpr (st + 2 < NS) rd(j_, std::integral_constant<int, st + 2>{});
            });
        });
    };

    if ((DMA_ALL || role == 1) && my_tiles > 0) dma(decode(0), 0);
    for (int it = 0; it <= my_tiles; ++it) {
        // this wave's vector-memory work since the last barrier: its DMA pieces of tile it's halo, then (conv2 waves,
        // from it == 2) their Q2 output stores of tile it - 2 -- vmcnt is in order, so vmcnt(Q2) leaves only the stores
        if (role == 1 && it >= 2) DBSR_VM_WAIT(Q2);
        else vm_drain();
        __syncthreads();
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const int g = ln >> 4, col = ln & 15;
        if (role == 0) {
            if (DMA_ALL && it + 1 < my_tiles) dma(decode(it + 1), (it + 1) % NHALO);
            if (it >= my_tiles) continue;
            // ---- conv1 of tile it on its 18 x 10 region: groups wp + 2 i (i < 6), batches of 2 ----
            const Tile cur = decode(it);
            const u32x4_t* lin = lds + (it % NHALO) * IN_U4;
            u32x4_t* mid = lmid + (it & 1) * MID_U4;
            const float4 b0 = *(const float4*)(lbias + 32 * wc + 8 * g), b1 = *(const float4*)(lbias + 32 * wc + 8 * g + 4);
            const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
            StaticFor<0, Q1 / RB1>::run([&](auto bt_) {
                constexpr int I0 = RB1 * decltype(bt_)::value;
                int pa[RB1], P0[RB1];
#pragma unroll
                for (int j = 0; j < RB1; ++j) {
                    pa[j] = min(16 * (wp + 2 * (I0 + j)) + col, MPX - 1);
                    const int r = pa[j] / MW, c = pa[j] - r * MW;
                    P0[j] = r * IW + c;
                }
                f32x4_t acc[RB1][2];
                if constexpr ((DBSR_RB64_ABL & 1) == 0)
                    taps(lin, std::integral_constant<int, IN_CH_U4>{}, std::integral_constant<int, IW>{}, g, P0, acc);
                else
                    for (int j = 0; j < RB1; ++j) acc[j][0] = acc[j][1] = f32x4_t{(float)P0[j], 0.f, 0.f, 0.f};
#pragma unroll
                for (int j = 0; j < RB1; ++j) {
                    const int p = 16 * (wp + 2 * (I0 + j)) + col;
                    const int r = pa[j] / MW, c = pa[j] - r * MW;
                    const int fy = cur.y0 - 1 + r, fx = cur.x0 - 1 + c;
                    const bool inside = (unsigned)fy < (unsigned)H && (unsigned)fx < (unsigned)W;
                    u32x4_t o;
#pragma unroll
                    for (int e = 0; e < 2; ++e) {
                        o[e] = relu16x2(H16<T>::pack(acc[j][0][2 * e] + bv[2 * e], acc[j][0][2 * e + 1] + bv[2 * e + 1]));
                        o[2 + e] = relu16x2(H16<T>::pack(acc[j][1][2 * e] + bv[4 + 2 * e],
                                                         acc[j][1][2 * e + 1] + bv[4 + 2 * e + 1]));
                    }
                    if (!inside) o = u32x4_t{0u, 0u, 0u, 0u};
                    if (p < MPX) mid[wc * MID_CH_U4 + 4 * p + halo_phys(p, g)] = o;
                }
            });
        } else {
            // ---- the next tile's halo, then conv2 of tile it - 1: rows wp + 2 i (i < 4), batches of 2 ----
            if (it + 1 < my_tiles) dma(decode(it + 1), (it + 1) % NHALO);
            if (it == 0) continue;
            const Tile cur = decode(it - 1);
            const u32x4_t* lin = lds + ((it - 1) % NHALO) * IN_U4;
            const u32x4_t* mid = lmid + ((it - 1) & 1) * MID_U4;
            const float4 b0 = *(const float4*)(lbias + 64 + 32 * wc + 8 * g);
            const float4 b1 = *(const float4*)(lbias + 64 + 32 * wc + 8 * g + 4);
            const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
            StaticFor<0, Q2 / RB2>::run([&](auto bt_) {
                constexpr int I0 = RB2 * decltype(bt_)::value;
                int row[RB2], P0[RB2];
#pragma unroll
                for (int j = 0; j < RB2; ++j) {
                    row[j] = wp + 2 * (I0 + j);
                    P0[j] = row[j] * MW + col;
                }
                f32x4_t acc[RB2][2];
                if constexpr ((DBSR_RB64_ABL & 2) == 0)
                    taps(mid, std::integral_constant<int, MID_CH_U4>{}, std::integral_constant<int, MW>{}, g, P0, acc);
                else
                    for (int j = 0; j < RB2; ++j) acc[j][0] = acc[j][1] = f32x4_t{(float)P0[j], 0.f, 0.f, 0.f};
#pragma unroll
                for (int j = 0; j < RB2; ++j) {
                    const int PR = (row[j] + 2) * IW + col + 2;
                    const u32x4_t rq = lin[wc * IN_CH_U4 + 4 * PR + halo_phys(PR, g)];
                    float v[8];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        v[r] = acc[j][0][r] + bv[r];
                        v[4 + r] = acc[j][1][r] + bv[4 + r];
                    }
                    u32x4_t o;
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        o[e] = relu16x2(H16<T>::pack(v[2 * e] + H16<T>::lo(rq[e]), v[2 * e + 1] + H16<T>::hi(rq[e])));
                    *(u32x4_t*)((T*)k2.y + cur.y_off + ((long long)row[j] * W + col) * k2.y_ld + 32 * wc + 8 * g) = o;
                }
            });
        }
    }
    vm_drain();                         // (no LDS-DMA outstanding at s_endpgm: tools/isa_audit.py)
}

int resblock64_launch(const ConvK& k1, const ConvK& k2, int n_frames, bool f16, int max_blocks, int cus,
                      hipStream_t s) {
    const int tiles_x = k1.in_w / rb64::TW, tiles_y = k1.in_h / rb64::TH;
    const int ntiles = n_frames * tiles_x * tiles_y;
    int grid = max_blocks > 0 ? std::min(max_blocks, cus) : cus;
    grid = std::min(grid, ntiles);
    DBSR_CHECK_ARG(rb_mapping_ok(grid, ntiles), "resblock: tile mapping out of range (grid %d, %d tiles)", grid, ntiles);
    if (f16)
        hipLaunchKernelGGL((resblock64_kernel<f16_t>), dim3(grid), dim3(512), 0, s, k1, k2, tiles_x, tiles_y, ntiles);
    else
        hipLaunchKernelGGL((resblock64_kernel<bf16_t>), dim3(grid), dim3(512), 0, s, k1, k2, tiles_x, tiles_y, ntiles);
    DBSR_LAUNCH_CHECK();
    return 0;
}

}  // namespace dbsr
