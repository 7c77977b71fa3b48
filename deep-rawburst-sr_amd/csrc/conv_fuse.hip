// Fused weight-predictor output conv + softmax over the burst + weighted fusion.
//
// Reference (models/dbsr/merging.py:55-57, 113-124):
//   logits  = conv3x3(h) + bias  (last weight_predictor layer, 2*proj -> C, no activation)
//   weights = softmax(logits.view(B, N, C, H, W), dim=1)          -> aux 'fusion_weights'
//             (softmax=False, :119-121: relu(logits) / (sum_n relu(logits) + 1e-12); dbsr_conv_fuse_relu_norm,
//              template flag RELU -- only the epilogue's normalisation differs)
//   fused   = (all_feat * weights).sum(dim=1),  all_feat = [ref_feat, warped oth_feat]
//
// The two-kernel path (dbsr_conv2d to a logits buffer + dbsr_fuse_softmax) writes the logits [B*N, H, W, C]
// to HBM rounded to 16 bits and reads them back: 2 x 264 MB per cfg2 step.  Here the logits never leave
// the CU and are never rounded: a block owns one "super-tile" -- (burst, 16x2 pixels, 128 output
// channels) -- and computes the conv for ALL N frames of the burst at once, every frame's fp32 logits
// in the accumulators of the wave that owns the super-tile's (pixel, channel) element.  The softmax over
// N is per (pixel, channel), so it runs lane-locally on those accumulators after the last K stage.
//
// Block = 8 waves (two per SIMD), persistent over super-tiles.  Wave (wc, wr) owns couts
// 32wc..32wc+31 of the super-tile's 128 (two 16-cout MFMA blocks; the packer's pipe_cout_perm gives each
// lane 8 consecutive couts of its pixel) x tile row wr (16 pixels) x all N frames: 2N accumulator tiles
// (112 registers at N = 14).  The conv's K = 9 taps x Cin runs in stages of (32-channel chunk, kernel
// row ky): per stage the block stages, by buffer-resource LDS-DMA into one of two LDS buffers,
//   - the 3 taps' weights of the 128 couts (24 1-KiB pieces of the chunk-major packed copy), read by
//     every wave for all N frames (the weights' reuse over the burst is what the two-kernel path lacks),
//   - for each of the N frames the 2 input rows x 18 pixels the kernel row needs (3 pieces per frame;
//     out-of-frame pixels land zeros),
// and every wave runs 3 taps x N frames x 2 MFMAs 16x16x32 on them.  The next stage's pieces are issued
// between the taps' MFMAs; one barrier per stage (84 MFMAs per wave at N = 14).
//
// Epilogue of a finished super-tile (after the next super-tile's first barrier; it needs no LDS but the
// bias): the N frames' feature loads are issued first (16 B per lane and frame), then bias + max +
// exp + sum over the frames run on the accumulators while they arrive; then weight = e / sum (the aux
// output, 16-B stores per frame) and fused = sum_n weight * feature (fp32, one 16-B store).
#include "common.hpp"

#include <algorithm>
#include <cmath>
#include <type_traits>

using namespace dbsr;

// Ablation switches for same-box A/B builds only (tools/build_variant.sh; the product build compiles none of
// them): bit 1 replaces the epilogue's softmax by a plain sum of the accumulators, 2 skips the halo DMA, 4 the
// weight DMA, 8 the feature loads, 16 the stage barriers
#ifndef DBSR_FUSE_ABL
#define DBSR_FUSE_ABL 0
#endif

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bfv8_t;
typedef __attribute__((ext_vector_type(8))) _Float16 hv8_t;

template <typename T>
__device__ __forceinline__ f32x4_t mfma16(const bf16x8_t& a, const bf16x8_t& b, f32x4_t c) {
    if constexpr (std::is_same<T, bf16_t>::value)
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bfv8_t, a), __builtin_bit_cast(bfv8_t, b), c,
                                                       0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(hv8_t, a), __builtin_bit_cast(hv8_t, b), c,
                                                      0, 0, 0);
}


// pixel-major halo image of one 32-channel chunk: halo pixel p's 4 k-groups at slots 4p..4p+3, k-group g
// at 4p + phys(p, g) (the pipelined conv kernel's swizzle: conflict-free ds_read_b128 for every tap shift)
__device__ __forceinline__ int halo_phys(int p, int g) { return 2 * (g & 1) + ((g >> 1) ^ ((p >> 2) & 1)); }

// Every tensor is addressed by element offsets that are affine in (burst b, frame n) -- checked on the host
// over every (b, n) the launch touches -- so the kernel does no frame-map divisions.
struct FuseK {
    const void* x; long long x_b; int x_nb, x_ld;         // h: frame (b, n) at byte x + 2*b*x_b + n*x_nb
    unsigned x_span;                                        // bytes of a burst's N frames from frame 0
    int H, W, nchunks, cout;
    const void* w_pipe; const float* bias;                  // chunk-major packed weights, fp32 bias (or null)
    const void* ref; long long ref_b; int ref_ld;          // feature of frame 0 of burst b
    const void* oth; long long oth_b, oth_n; int oth_ld;   // frame n >= 1: oth + b*oth_b + (n-1)*oth_n
    void* fused; long long fus_b; int fus_ld;
    void* wts; long long wts_b, wts_n; int wts_ld;         // aux fusion weights (nullptr: not written)
    // the epilogue's loads / stores go through a buffer resource per (tensor, burst): byte spans of a burst's
    // frames (< 2^31, checked on the host) and per-frame byte strides (wave-uniform soffset)
    unsigned ref_span, oth_span, wts_span;
    int oth_nb, wts_nb;
};

template <int NF>
struct FuseCfg {
    static constexpr int WM = 128, TW = 16, TH = 2, NWAVES = 8;
    static constexpr int HWD = TW + 2;                        // input row width of a tile: 18
    static constexpr int ROW_PX = NF * HWD;                   // one input row of the burst's N frames: 252
    static constexpr int RP = (ROW_PX + 15) / 16;             // its 1-KiB pieces (16 pixels x 4 k-groups): 16
    static constexpr int NROW = 5;                            // row ring slots
    static constexpr int W_ITEMS = 3 * (WM / 16);             // weight pieces per stage: (tap, 16-cout block)
    static constexpr int NWB = 3;                             // weight ring buffers
    static constexpr int W_U4 = W_ITEMS * 64, ROW_U4 = RP * 64;
    static constexpr int ROWS_OFF = NWB * W_U4;               // row ring after the weight ring
    static constexpr int BIAS_OFF = ROWS_OFF + NROW * ROW_U4;
    static constexpr int LDS_U4 = BIAS_OFF + 512 / 4;         // + cout <= 512 fp32 biases
    static constexpr int PER1 = (W_ITEMS + RP) / NWAVES;      // DMA pieces per wave for a stage with one new row
    static constexpr int PER2 = (W_ITEMS + 2 * RP) / NWAVES;  // ... with two (kernel row 0 of a chunk)
    static_assert((W_ITEMS + RP) % NWAVES == 0 && (W_ITEMS + 2 * RP) % NWAVES == 0, "whole pieces per wave");
    static_assert(LDS_U4 * 16 <= 160 * 1024, "weight ring + row ring + bias must fit the LDS");
};

template <typename T, int NF, bool RELU>
__global__ __launch_bounds__(512, 1) void conv_fuse_kernel(FuseK k, int tiles_x, int tiles_y, int nct, int ntiles) {
    using C = FuseCfg<NF>;
    DBSR_OWN_SIMDS();
    __shared__ __attribute__((aligned(16))) u32x4_t lds[C::LDS_U4];
    float* lbias = (float*)(lds + C::BIAS_OFF);

    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g = lane >> 4, col = lane & 15;
    const int wc = wave & 3, wr = wave >> 2;
    // bias into LDS once; ordered before its first read (the first epilogue) by the loop's barriers
    for (int c = threadIdx.x; c < k.cout; c += 512) lbias[c] = k.bias ? k.bias[c] : 0.f;

    // persistent super-tile walk, XCD-grouped: the blocks of one XCD (equal blockIdx % 8) take a contiguous
    // range of super-tile ids per round -- the cout tiles of a spatial tile and neighbouring tiles' shared
    // input rows meet in one L2 (grid is a multiple of 8)
    const int grid = gridDim.x, blk = blockIdx.x;
    const int pb = (blk & 7) * (grid >> 3) + (blk >> 3);
    const int my_tiles = pb < ntiles ? (ntiles - pb + grid - 1) / grid : 0;
    if (my_tiles == 0) return;

    struct Tile { int bb, y0, x0, cb; };          // wave-uniform: scalar registers
    auto decode = [&](int i) {
        int L = i * grid + pb;
        Tile t;
        t.cb = (L % nct) * C::WM; L /= nct;
        t.x0 = (L % tiles_x) * C::TW; L /= tiles_x;
        t.y0 = (L % tiles_y) * C::TH;
        t.bb = L / tiles_y;
        return t;
    };

    // The LDS holds a 3-buffer ring of stage weights and a 5-slot ring of input rows, and the pieces of stage
    // s + 2 are issued during stage s (two stages in flight: the LDS-DMA latency, not the MFMAs, bounded the
    // double-buffered version).  Stage (chunk c, kernel row ky) reads input rows ky, ky + 1 of the chunk's 4
    // (tile rows y0 - 1 .. y0 + 2); each row, with all N frames' 18 pixels, is loaded once per chunk: 2 new rows
    // for ky = 0, one for ky = 1, 2.  Row r of global chunk number gc lives in slot (4 gc + r) % 5, which no
    // stage in flight still reads.
    // One 1-KiB DMA piece of stage (super-tile t, chunk c, kernel row ky, global chunk gc) into weight buffer wb:
    // piece `it` of this wave is item wave + 8*it; items [0, W_ITEMS): weights of tap 3ky + kx, 16-cout block b
    // (contiguous 1 KiB of the packed copy); then the new rows' pieces of 16 row pixels x 4 k-groups (lane ->
    // frame n = p / 18, column p % 18, physical slot).
    const int pix_b = k.x_ld * (int)sizeof(T);
    const unsigned lds0 = (unsigned)(unsigned long long)(__attribute__((address_space(3))) u32x4_t*)lds;
    // one buffer resource over the burst's N input frames (x_span bytes < 2^31, checked on the host): an
    // out-of-frame pixel gets voffset BUF_OOB, past num_records, and lands zeros
    auto dma = [&](int it, const Tile& t, int c, int ky, int gc, int wb) {
        const int item = wave + C::NWAVES * it;
        if ((DBSR_FUSE_ABL & 4) && item < C::W_ITEMS) return;   // (timing only)
        if ((DBSR_FUSE_ABL & 2) && item >= C::W_ITEMS) return;
        if (item < C::W_ITEMS) {
            const int kx = item / (C::WM / 16), b16 = item % (C::WM / 16);
            const int piece = (((t.cb >> 4) + b16) * k.nchunks + c) * 9 + 3 * ky + kx;
            lds_dma16(k.w_pipe, 0xffffffffu, lane * 16, piece * 1024, lds0 + (wb * C::W_U4 + item * 64) * 16);
        } else {
            const int ri = item - C::W_ITEMS;
            const int r = (ky == 0 ? 0 : ky + 1) + ri / C::RP, j = ri % C::RP;
            const int slot = (4 * gc + r) % C::NROW;
            int ln = lane;
            asm volatile("" : "+v"(ln));        // keep the lane math here (not hoisted into spilled registers)
            const int p = 16 * j + (ln >> 2), ph = ln & 3;
            const int gg = 2 * ((ph & 1) ^ ((p >> 2) & 1)) + (ph >> 1);
            const int n = p / C::HWD, cc = p - n * C::HWD;
            const int hy = t.y0 - 1 + r, hx = t.x0 - 1 + cc;
            const bool ok = p < C::ROW_PX && (unsigned)hy < (unsigned)k.H && (unsigned)hx < (unsigned)k.W;
            lds_dma16((const T*)k.x + t.bb * k.x_b, k.x_span,
                   ok ? n * k.x_nb + (hy * k.W + hx) * pix_b + c * 64 + gg * 16 : BUF_OOB, 0,
                   lds0 + (C::ROWS_OFF + slot * C::ROW_U4 + j * 64) * 16);
        }
    };

    // lane-dependent LDS bases: the B-fragment of frame n at tap kx reads row pixel m = 18n + kx + col of the
    // row slot, k-group g: slot 4(m + col) + halo_phys(m + col, g), where halo_phys depends on m only through
    // m & 7 (8 per-lane bases + an immediate 4m); the A-fragment of 16-cout block (2wc + i) at tap kx is weight
    // item kx*8 + 2wc + i, row col, k-group g
    int base8[8];
#pragma unroll
    for (int rho = 0; rho < 8; ++rho) base8[rho] = 4 * col + halo_phys(col + rho, g);
    const int a_base = 2 * wc * 64 + g * 16 + col;

    f32x4_t acc[NF][2];
#pragma unroll
    for (int n = 0; n < NF; ++n) acc[n][0] = acc[n][1] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    // lane (g, col) of wave (wc, wr) holds, for every frame n, couts ch..ch+7 (ch = cb + 32wc + 8g) of pixel
    // (y0 + wr, x0 + col): acc[n][0] = couts ch..ch+3, acc[n][1] = ch+4..ch+7
    auto lane_pix = [&](const Tile& t) { return (t.y0 + wr) * k.W + t.x0 + col; };
    auto lane_ch = [&](const Tile& t) { return t.cb + 32 * wc + 8 * g; };
    // (buffer loads / stores: a per-(tensor, burst) resource, the lane's 32-bit byte offset -- the same for every
    // frame -- and the frame's uniform byte offset as soffset; no per-frame 64-bit lane addresses in registers)
    auto feat_load = [&](const Tile& t, int n, u32x4_t& dst) {
        const unsigned pix = lane_pix(t), ch = lane_ch(t);
        if (n == 0) {
            const auto r = buf_rsrc((const T*)k.ref + t.bb * k.ref_b, k.ref_span);
            dst = __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(
                r, (int)((pix * (unsigned)k.ref_ld + ch) * (unsigned)sizeof(T)), 0, 2));
        } else {
            const auto r = buf_rsrc((const T*)k.oth + t.bb * k.oth_b, k.oth_span);
            dst = __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(
                r, (int)((pix * (unsigned)k.oth_ld + ch) * (unsigned)sizeof(T)), (n - 1) * k.oth_nb, 2));
        }
    };
    // The weights go out as global stores: ROCm 7.2 pads a VALU write of a global store's data registers right
    // after the store with the wait states gfx950 needs, but not after the buffer-store builtin, where the store
    // then wrote the overwritten values for part of the wave.  The lane offset passes an empty asm
    // inside the epilogue, so the per-frame 64-bit addresses are formed there and not hoisted out of the stage loop.
    auto store_w = [&](const Tile& t, int n, const u32x4_t& v) {
        if (k.wts) {
            unsigned off = ((unsigned)lane_pix(t) * (unsigned)k.wts_ld + (unsigned)lane_ch(t)) * (unsigned)sizeof(T);
            asm volatile("" : "+v"(off));
            char* fb = (char*)((T*)k.wts + t.bb * k.wts_b) + n * k.wts_nb;
            __builtin_nontemporal_store(v, (u32x4_t*)(fb + off));
        }
    };
    // xb: a ring of NH frames' features (16-B loads; the first NH issued first, so their latency overlaps the
    // softmax, each later one as its slot's frame is consumed); each frame's weights are stored as computed.  (Spreading these loads and stores over the MFMA stages measured slower: a
    // wave's vector-memory operations complete in issue order, so an HBM load ahead of the next stage's LDS-DMA
    // pieces delays the barrier that waits for them.)
    constexpr int NH = (NF + 1) / 2;     // feature registers: a ring of half the frames
    auto epilogue = [&](const Tile& t) {
        u32x4_t xb[NH];
        StaticFor<0, NH>::run([&](auto n_) {
            if constexpr ((DBSR_FUSE_ABL & 8) != 0)         // (timing only: no feature loads)
                xb[decltype(n_)::value] = __builtin_bit_cast(u32x4_t, acc[decltype(n_)::value][0]);
            else
                feat_load(t, decltype(n_)::value, xb[decltype(n_)::value]);
        });
        const int ch = lane_ch(t);
        const float4 b0 = *(const float4*)(lbias + ch), b1 = *(const float4*)(lbias + ch + 4);
        const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
        float m[8], sum[8], inv[8], fz[8];
        if constexpr ((DBSR_FUSE_ABL & 1) != 0) {         // (timing only: every accumulator consumed, cheaply)
#pragma unroll
            for (int e = 0; e < 8; ++e) fz[e] = bv[e];
            StaticFor<0, NF>::run([&](auto n_) {
                constexpr int n = decltype(n_)::value;
#pragma unroll
                for (int e = 0; e < 8; ++e) fz[e] += acc[n][e >> 2][e & 3] + H16<T>::lo(xb[n % NH][e >> 1]);
                if constexpr (n + NH < NF && (DBSR_FUSE_ABL & 8) == 0) feat_load(t, n + NH, xb[n % NH]);
                acc[n][0] = acc[n][1] = f32x4_t{0.f, 0.f, 0.f, 0.f};
            });
        } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) sum[e] = 0.f;
            if constexpr (RELU) {
                // softmax=False (merging.py:119-121): relu(logit) / (sum over the burst + 1e-12)
#pragma unroll
                for (int n = 0; n < NF; ++n)
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        const float x = fmaxf(acc[n][e >> 2][e & 3] + bv[e], 0.f);   // fp32 logit, never rounded
                        acc[n][e >> 2][e & 3] = x;
                        sum[e] += x;
                    }
#pragma unroll
                for (int e = 0; e < 8; ++e) sum[e] += 1e-12f;
            } else {
#pragma unroll
                for (int e = 0; e < 8; ++e) m[e] = -INFINITY;
#pragma unroll
                for (int n = 0; n < NF; ++n)
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        const float l = acc[n][e >> 2][e & 3] + bv[e];      // the logit, fp32 (never rounded)
                        acc[n][e >> 2][e & 3] = l;
                        m[e] = fmaxf(m[e], l);
                    }
#pragma unroll
                for (int n = 0; n < NF; ++n)
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        const float x = __expf(acc[n][e >> 2][e & 3] - m[e]);
                        acc[n][e >> 2][e & 3] = x;
                        sum[e] += x;
                    }
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                inv[e] = 1.0f / sum[e];
                fz[e] = 0.f;
            }
            // frame by frame: weights, their store, the weighted features; frame n's feature register then takes
            // frame n + NH's load
            StaticFor<0, NF>::run([&](auto n_) {
                constexpr int n = decltype(n_)::value;
                float w[8];
                u32x4_t o;
#pragma unroll
                for (int e = 0; e < 8; ++e) w[e] = acc[n][e >> 2][e & 3] * inv[e];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    fz[2 * j] = fmaf(H16<T>::lo(xb[n % NH][j]), w[2 * j], fz[2 * j]);
                    fz[2 * j + 1] = fmaf(H16<T>::hi(xb[n % NH][j]), w[2 * j + 1], fz[2 * j + 1]);
                    o[j] = H16<T>::pack(w[2 * j], w[2 * j + 1]);
                }
                if constexpr (n + NH < NF) feat_load(t, n + NH, xb[n % NH]);
                store_w(t, n, o);
                acc[n][0] = acc[n][1] = f32x4_t{0.f, 0.f, 0.f, 0.f};
            });
        }
        u32x4_t o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = H16<T>::pack(fz[2 * j], fz[2 * j + 1]);
        *(u32x4_t*)((T*)k.fused + t.bb * k.fus_b + lane_pix(t) * k.fus_ld + ch) = o;
    };

    int s3 = 0;                         // stage index mod 3 (weight ring buffer)
    int gc = 0;                         // global chunk number (row ring slots)
    Tile cur = decode(0), prev = cur;
    // prologue: stages 0 and 1 of the first super-tile
#pragma unroll
    for (int it = 0; it < C::PER2; ++it) dma(it, cur, 0, 0, 0, 0);
#pragma unroll
    for (int it = 0; it < C::PER1; ++it) dma(it, cur, 0, 1, 0, 1);
    int pending = C::PER1;              // this wave's pieces of the stage after the current one (in flight)

    for (int ti = 0; ti < my_tiles; ++ti) {
        const bool has_next = ti + 1 < my_tiles;
        const Tile nxt = has_next ? decode(ti + 1) : cur;
        int c = 0, ky = 0;
        for (int st = 0; st < 3 * k.nchunks; ++st) {
            // stage (c, ky) landed: every wave waits for its own pieces of it (the next stage's may still be in
            // flight), then the barrier makes every wave's visible
            switch (pending) {
                case C::PER1: DBSR_VM_WAIT(C::PER1); break;
                case C::PER2: DBSR_VM_WAIT(C::PER2); break;
                default: vm_drain(); break;
            }
            if constexpr ((DBSR_FUSE_ABL & 16) == 0) __syncthreads();   // (timing only: no barrier)
            if (st == 0 && ti > 0) epilogue(prev);
            // the stage two ahead: (c, 2) from ky 0, else kernel row ky - 1 of the next chunk, which may be the next
            // super-tile's first
            const int ky2 = ky == 0 ? 2 : ky - 1;
            int c2 = ky == 0 ? c : c + 1;
            Tile t2 = cur;
            bool issue = true;
            if (c2 == k.nchunks) {
                c2 = 0;
                t2 = nxt;
                issue = has_next;
            }
            const int gc2 = ky == 0 ? gc : gc + 1, wb2 = s3 == 0 ? 2 : s3 - 1;
            const u32x4_t* lw = lds + s3 * C::W_U4;
            // this wave's B row: kernel row ky + wr of the chunk
            const u32x4_t* lr = lds + C::ROWS_OFF + ((4 * gc + ky + wr) % C::NROW) * C::ROW_U4;
            // the stage's 3 taps x N frames as one flat sequence of steps q = kx*N + n; each step's B-fragment is
            // read PD steps ahead (a ring of PD registers) and the next tap's A-fragments one tap ahead, so the LDS
            // latency hides behind the MFMAs instead of a wait before every MFMA pair
            auto read_a = [&](int kx, int i) {
                return __builtin_bit_cast(bf16x8_t, lw[a_base + (kx * (C::WM / 16) + i) * 64]);
            };
            auto read_b = [&](int q) {
                const int m = (q % NF) * C::HWD + q / NF;
                return __builtin_bit_cast(bf16x8_t, lr[base8[m & 7] + 4 * m]);
            };
            constexpr int PD = 6, NQ = 3 * NF;
            bf16x8_t bq[PD], a[2][2];
            a[0][0] = read_a(0, 0);
            a[0][1] = read_a(0, 1);
#pragma unroll
            for (int q = 0; q < PD; ++q) bq[q] = read_b(q);
            StaticFor<0, NQ>::run([&](auto q_) {
                constexpr int q = decltype(q_)::value, kx = q / NF, n = q % NF;
                if constexpr (n == 0) {
                    if constexpr (kx + 1 < 3) {
                        a[(kx + 1) & 1][0] = read_a(kx + 1, 0);
                        a[(kx + 1) & 1][1] = read_a(kx + 1, 1);
                    }
                    // the pieces of the stage two ahead, a third of them per tap between this stage's MFMAs
                    if (issue) {
                        if (ky2 == 0) {
#pragma unroll
                            for (int it = 0; it < C::PER2; ++it)
                                if ((it * 3) / C::PER2 == kx) dma(it, t2, c2, ky2, gc2, wb2);
                        } else {
#pragma unroll
                            for (int it = 0; it < C::PER1; ++it)
                                if ((it * 3) / C::PER1 == kx) dma(it, t2, c2, ky2, gc2, wb2);
                        }
                    }
                }
                const bf16x8_t b = bq[q % PD];
                if constexpr (q + PD < NQ) bq[q % PD] = read_b(q + PD);
                acc[n][0] = mfma16<T>(a[kx & 1][0], b, acc[n][0]);
                acc[n][1] = mfma16<T>(a[kx & 1][1], b, acc[n][1]);
                __builtin_amdgcn_sched_barrier(0);      // keep the ring's order (the scheduler re-serialises it)
            });
            pending = !issue ? 0 : ky2 == 0 ? C::PER2 : C::PER1;
            s3 = s3 == 2 ? 0 : s3 + 1;
            if (ky == 2) {
                ky = 0;
                ++c;
                ++gc;
            } else {
                ++ky;
            }
        }
        prev = cur;
        cur = nxt;
    }
    vm_drain();                         // (the epilogue reads no LDS but the bias; keeps the DMA queue drained)
    __syncthreads();
    epilogue(prev);
}

int g_fuse_cus = 0;
int fuse_cus() {
    if (g_fuse_cus == 0) {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
            g_fuse_cus = n;
        else
            g_fuse_cus = 256;
    }
    return g_fuse_cus;
}

inline int cin_pad32(int cin) { return (cin + 31) / 32 * 32; }
constexpr int FUSE_NF = 14;             // burst size the kernel is built for (the SyntheticBurst / BurstSR bursts)
constexpr int FUSE_WM = 128;            // couts per super-tile

// element offset of logical frame f of t (host copy of map_frame)
long long frame_off(const dbsr_tensor& t, long long f) {
    const dbsr_frame_map& m = t.map;
    return ((f / m.fpg) * m.group_stride + m.group_offset + (f % m.fpg) * m.inner_stride) * t.img_stride;
}
// t's frame fb*b + fn*n + f0 sits at element base + b*sb + n*sn for every b < B, n < N
bool affine_frames(const dbsr_tensor& t, int B, int N, int fb, int fn, int f0, long long& base, long long& sb,
                   long long& sn) {
    if (t.map.fpg <= 0) return false;
    base = frame_off(t, f0);
    sb = B > 1 ? frame_off(t, fb + f0) - base : 0;
    sn = N > 1 ? frame_off(t, fn + f0) - base : 0;
    for (int b = 0; b < B; ++b)
        for (int n = 0; n < N; ++n)
            if (frame_off(t, (long long)fb * b + (long long)fn * n + f0) != base + b * sb + n * sn) return false;
    return true;
}

// the conv side of the fused kernel's contract (the features / outputs are checked at launch)
bool fuse_conv_ok(const dbsr_conv_desc* d, int B, int N) {
    if (!d || (d->x.dtype != DBSR_BF16 && d->x.dtype != DBSR_F16) || d->kh != 3 || d->kw != 3 || d->stride != 1 ||
        d->pad != 1 || d->dil != 1 || d->precise || d->cin <= 16)
        return false;
    if (N != FUSE_NF || B <= 0 || d->n_frames != B * N) return false;
    if (d->cout % FUSE_WM || d->cout > 512 || d->in_h != d->out_h || d->in_w != d->out_w) return false;
    if (d->in_w % 16 || d->in_h % 2 || d->in_h <= 0 || d->in_w <= 0) return false;
    if (d->x.ld % 8 || d->x.c0 % 8 || d->x.c0 + cin_pad32(d->cin) > d->x.ld) return false;
    if ((long long)d->in_h * d->in_w * d->x.ld * 2 >= (1LL << 31)) return false;   // 32-bit offsets per frame
    long long base, sb, sn;
    return affine_frames(d->x, B, N, N, 1, 0, base, sb, sn);
}

// a feature / output tensor of the fused kernel: 16-bit NHWC of the conv's dtype, 16-B channel runs inside
// its pixel (c0 + cout <= ld, 8-aligned), 32-bit pixel offsets
bool fuse_tensor_ok(const dbsr_tensor& t, int dt, int cout, int hw) {
    return t.ptr && t.dtype == dt && t.ld % 8 == 0 && t.c0 % 8 == 0 && t.c0 >= 0 && t.c0 + cout <= t.ld &&
           (long long)hw * t.ld < (1LL << 31);
}

}  // namespace

extern "C" int dbsr_conv_fuse_ok(const dbsr_conv_desc* d, int B, int N) { return fuse_conv_ok(d, B, N) ? 1 : 0; }

namespace {

int conv_fuse(const dbsr_conv_desc* d, int B, int N, dbsr_tensor ref, dbsr_tensor oth, dbsr_tensor fused,
              dbsr_tensor weights, bool relu, void* stream) {
    DBSR_CHECK_ARG(fuse_conv_ok(d, B, N), "conv_fuse_softmax: unsupported conv / burst (needs dbsr_conv_fuse_ok)");
    DBSR_CHECK_ARG(d->x.ptr && d->w, "conv_fuse_softmax: null pointer");
    const int C = d->cout, dt = d->x.dtype, hw = d->in_h * d->in_w;
    DBSR_CHECK_ARG(fuse_tensor_ok(ref, dt, C, hw) && fuse_tensor_ok(oth, dt, C, hw) && fuse_tensor_ok(fused, dt, C, hw),
                   "conv_fuse_softmax: ref / oth / fused must be NHWC tensors of the conv's dtype with "
                   "ld, c0 multiples of 8 and c0 + cout <= ld");
    if (weights.ptr)
        DBSR_CHECK_ARG(fuse_tensor_ok(weights, dt, C, hw), "conv_fuse_softmax: bad weights tensor");
    FuseK k;
    long long base, sb, sn;
    const int esz = 2;
    // h: frame b*N + n
    affine_frames(d->x, B, N, N, 1, 0, base, sb, sn);
    k.x = (const char*)d->x.ptr + (base + d->x.c0) * esz; k.x_b = sb; k.x_ld = d->x.ld;
    const long long span = ((N - 1) * sn + (long long)d->in_h * d->in_w * d->x.ld) * esz;
    DBSR_CHECK_ARG(sn >= 0 && span < (1LL << 31), "conv_fuse_softmax: a burst's input frames span >= 2 GiB");
    k.x_nb = (int)(sn * esz); k.x_span = (unsigned)span;
    k.H = d->in_h; k.W = d->in_w;
    const int cp = cin_pad32(d->cin);
    k.nchunks = cp / 32;
    k.cout = C;
    const int Kp = (9 * cp / 8 + 3) / 4 * 4 * 8;                 // dbsr_hip.h packed layout
    k.w_pipe = (const char*)d->w + (size_t)((C + 63) / 64 * 64) * Kp * esz;
    k.bias = d->bias;
    DBSR_CHECK_ARG(affine_frames(ref, B, 1, 1, 0, 0, base, sb, sn), "conv_fuse_softmax: ref frame map not affine");
    k.ref = (const char*)ref.ptr + (base + ref.c0) * esz; k.ref_b = sb; k.ref_ld = ref.ld;
    DBSR_CHECK_ARG(affine_frames(oth, B, N - 1, N - 1, 1, 0, base, sb, sn), "conv_fuse_softmax: oth frame map not affine");
    k.oth = (const char*)oth.ptr + (base + oth.c0) * esz; k.oth_b = sb; k.oth_n = sn; k.oth_ld = oth.ld;
    {
        const long long span = ((N - 2) * sn + C + (long long)(hw - 1) * oth.ld) * esz;
        DBSR_CHECK_ARG(sn >= 0 && span < (1LL << 31), "conv_fuse_softmax: a burst's other frames span >= 2 GiB");
        k.oth_span = (unsigned)span;
        k.oth_nb = (int)(sn * esz);
    }
    {
        const long long span = ((long long)C + (long long)(hw - 1) * ref.ld) * esz;
        DBSR_CHECK_ARG(span < (1LL << 31), "conv_fuse_softmax: ref frame >= 2 GiB");
        k.ref_span = (unsigned)span;
    }
    DBSR_CHECK_ARG(affine_frames(fused, B, 1, 1, 0, 0, base, sb, sn), "conv_fuse_softmax: fused frame map not affine");
    k.fused = (char*)fused.ptr + (base + fused.c0) * esz; k.fus_b = sb; k.fus_ld = fused.ld;
    if (weights.ptr) {
        DBSR_CHECK_ARG(affine_frames(weights, B, N, N, 1, 0, base, sb, sn),
                       "conv_fuse_softmax: weights frame map not affine");
        k.wts = (char*)weights.ptr + (base + weights.c0) * esz; k.wts_b = sb; k.wts_n = sn; k.wts_ld = weights.ld;
        const long long span = ((N - 1) * sn + C + (long long)(hw - 1) * weights.ld) * esz;
        DBSR_CHECK_ARG(sn >= 0 && span < (1LL << 31), "conv_fuse_softmax: a burst's fusion weights span >= 2 GiB");
        k.wts_span = (unsigned)span;
        k.wts_nb = (int)(sn * esz);
    } else {
        k.wts = nullptr; k.wts_b = k.wts_n = 0; k.wts_ld = 0; k.wts_span = 0; k.wts_nb = 0;
    }
    const int tiles_x = k.W / 16, tiles_y = k.H / 2, nct = C / FUSE_WM;
    const long long nt = (long long)B * tiles_x * tiles_y * nct;
    DBSR_CHECK_ARG(nt < (1LL << 31), "conv_fuse_softmax: grid too large");
    const int cap = d->max_blocks > 0 ? std::min(d->max_blocks, fuse_cus()) : fuse_cus();
    int grid = (int)std::min<long long>(nt, cap);
    // a multiple of 8 (the XCD-grouped walk), rounded DOWN so a max_blocks cap is not exceeded (each
    // block takes ~160 KB of LDS and its SIMDs, CUs meant for a concurrent lane); at least 8 (surplus blocks exit)
    grid = grid >= 8 ? grid / 8 * 8 : 8;
    hipStream_t s = (hipStream_t)stream;
    auto launch = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(grid), dim3(512), 0, s, k, tiles_x, tiles_y, nct, (int)nt);
    };
    if (dt == DBSR_F16)
        relu ? launch(conv_fuse_kernel<f16_t, FUSE_NF, true>) : launch(conv_fuse_kernel<f16_t, FUSE_NF, false>);
    else
        relu ? launch(conv_fuse_kernel<bf16_t, FUSE_NF, true>) : launch(conv_fuse_kernel<bf16_t, FUSE_NF, false>);
    DBSR_LAUNCH_CHECK();
    return 0;
}

}  // namespace

extern "C" int dbsr_conv_fuse_softmax(const dbsr_conv_desc* d, int B, int N, dbsr_tensor ref, dbsr_tensor oth,
                                      dbsr_tensor fused, dbsr_tensor weights, void* stream) {
    return conv_fuse(d, B, N, ref, oth, fused, weights, false, stream);
}

extern "C" int dbsr_conv_fuse_relu_norm(const dbsr_conv_desc* d, int B, int N, dbsr_tensor ref, dbsr_tensor oth,
                                        dbsr_tensor fused, dbsr_tensor weights, void* stream) {
    return conv_fuse(d, B, N, ref, oth, fused, weights, true, stream);
}
