// Fused weight-predictor output conv + softmax over the burst + weighted fusion.
//
// Reference (models/dbsr/merging.py:55-57, 113-124):
//   logits  = conv3x3(h)  (last weight_predictor layer, 2*proj -> C, no activation)
//   weights = softmax(logits.view(B, N, C, H, W), dim=1)          -> aux 'fusion_weights'
//   fused   = (all_feat * weights).sum(dim=1),  all_feat = [ref_feat, warped oth_feat]
//
// The two-kernel path writes the logits [B*N, H, W, C] to HBM and reads them back in the fusion kernel
// (2 x 66 MB per burst at C = 512, bf16).  Here the logits never leave the CU: a block owns one
// (burst, 16x4-pixel tile, 64-channel slice) "super-tile" and computes the conv for ALL N frames of the
// burst in turn, keeping every frame's logits (bf16-rounded, as the two-kernel path stores them) in
// registers.  Softmax over N is per (pixel, channel), so it is local to the lane that owns the value:
// no cross-lane or cross-block communication.
//
// Block = 4 waves, one per SIMD (the whole VGPR+AGPR file).  Wave w owns couts 16w..16w+15 of the
// block's 64-channel slice for the tile's 4 rows x 16 pixels (4 MFMA 16x16 tiles) and holds its
// weights for the whole K = 9 taps x Cin in VGPRs (144 registers at Cin 128), loaded once: blocks are
// persistent with a fixed channel slice, so only the input halo moves through the LDS (LDS-DMA,
// double-buffered per frame, out-of-frame pixels land zeros).  Per k-step a wave reads 4 B-fragments
// for 4 MFMAs.
//
// Per lane and frame: 16 logits (4 rows x 4 consecutive channels), an online max / sum-of-exp, and a
// 14-deep register bank of the bf16 logits that rotates by one frame per frame.  The fusion of a
// finished super-tile runs during the N frames of the next one: in frame n the lane turns the oldest
// bank entry (the previous super-tile's frame n) into softmax weights, stores them (aux output) and
// accumulates weight x feature (the feature loads are issued one frame ahead), so the HBM traffic of
// the fusion overlaps the MFMAs.  After the last super-tile a drain pass finishes its fusion.
#include "common.hpp"

#include <algorithm>
#include <type_traits>

// Measured slower than dbsr_conv2d + dbsr_fuse_softmax and therefore not in the product
// library: built only with -DDBSR_EXPERIMENTAL=1 (`make exp EXP_FLAGS=-DDBSR_EXPERIMENTAL=1 EXP_NAME=fuse`, then
// DBSR_HIP_LIB=.../libdbsr_hip_fuse.so).  Without it the two entry points report the shape as unserved.
#if DBSR_EXPERIMENTAL

using namespace dbsr;

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

constexpr int BUF_OOB = (int)0x80000000u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, unsigned bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ void blds16(__amdgpu_buffer_rsrc_t r, int voff, u32x4_t* lds_piece) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_piece, 16, voff, 0, 0, 0);
}
// pixel-major halo image of one 32-channel chunk: halo pixel p's 4 k-groups at slots 4p..4p+3, k-group g
// at 4p + phys(p, g) (the pipelined conv kernel's swizzle: conflict-free ds_read_b128 for every tap shift)
__device__ __forceinline__ int halo_phys(int p, int g) { return 2 * (g & 1) + ((g >> 1) ^ ((p >> 2) & 1)); }

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

struct FuseK {
    const void* x; long long x_is; int x_ld; dbsr_frame_map xm;   // h: [B*N frames][H][W][x_ld]
    int H, W;
    const void* w; int Kp; const float* bias;                       // packed rows [cout_pad][Kp], fp32 bias
    dbsr_tensor ref, oth, fused, weights;                           // weights.ptr may be null (no aux output)
    int B, N, C;
};

template <int NCH>
struct FuseCfg {
    static constexpr int TW = 16, TH = 4, HWD = TW + 2, HHT = TH + 2, NQ = HWD * HHT;   // 18 x 6 halo
    static constexpr int IN_ITEMS = (NQ + 15) / 16;            // 1-KiB DMA pieces per 32-channel chunk
    static constexpr int ITEMS = NCH * IN_ITEMS;               // pieces per frame
    static constexpr int PER = (ITEMS + 3) / 4;                // pieces per wave per frame
    static constexpr int STAGE_U4 = ITEMS * 64;                // 16-B slots per frame buffer
    static constexpr int STEPS_W = NCH / 2 * 9;                // (chunk, tap) k-steps per wave and frame (K half)
    static constexpr int XCH_U4 = 2 * 2 * 2 * 4 * 64;          // exchange: [parity][ch][src kc][4 tiles][64 lanes]
    static constexpr int ST_U4 = 4 * 12 * 64;                  // fusion state: [wave][mp 4 | ip 4 | fz 4][64 lanes]
    static constexpr int LDS_U4 = 2 * STAGE_U4 + XCH_U4 + ST_U4 + 64 / 4;   // + the slice's 64 biases
    static_assert(NCH % 2 == 0, "K split in halves");
    static_assert(LDS_U4 * 16 <= 160 * 1024, "two frame buffers + exchange + fusion state must fit the LDS");
};

template <typename T, int NCH, int NF>
__global__ __launch_bounds__(256, 1) void conv_fuse_kernel(FuseK k, int tiles_x, int tiles_y, int nct, int nsp,
                                                           int px) {
    using C = FuseCfg<NCH>;
    // one wave per SIMD with the register file to itself (the LDS-DMA kernels own their SIMDs, common.hpp)
    asm volatile("" ::: "v255", "a255");
    __shared__ __attribute__((aligned(16))) u32x4_t lds[C::LDS_U4];

    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g = lane >> 4, col = lane & 15;

    // block -> (channel slice, spatial stream), XCD-grouped: the nct slices of a tile share its halo in one L2
    const int b = blockIdx.x, slot = b >> 3, spx = px / nct;
    const int ct = slot % nct, S = 8 * spx, sid = (b & 7) * spx + slot / nct;
    const int my_st = sid < nsp ? (nsp - sid + S - 1) / S : 0;
    if (my_st == 0) return;

    // wave (kc, ch): K half kc (chunks kc*NCW .. +NCW-1) x couts 32ch..32ch+31 of the slice, all 4 tile rows.
    // MFMA row m of the wave's 16-cout block i is cout 32ch + 8(m>>2) + 4i + (m&3) (rows permuted at load):
    // lane (g, col) then holds 8 consecutive couts cl..cl+7 of its pixel in blocks 0 and 1 -> 16-B accesses
    constexpr int NCW = NCH / 2;                        // 32-channel chunks per wave
    const int kc = wave & 1, ch = wave >> 1;
    const int cs = ct * 64 + 32 * ch;                   // first cout of the wave
    constexpr int CG = NCH * 4;                         // k-groups per tap
    bf16x8_t wr[NCW][9][2];
#pragma unroll
    for (int c = 0; c < NCW; ++c)
#pragma unroll
        for (int tap = 0; tap < 9; ++tap)
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int co = cs + 8 * (col >> 2) + 4 * i + (col & 3);
                wr[c][tap][i] = *(const bf16x8_t*)((const T*)k.w + (long long)co * k.Kp +
                                                   (tap * CG + (kc * NCW + c) * 4 + g) * 8);
            }
    const int cl = cs + 8 * g;                          // the lane's 8 output channels cl..cl+7
    // per-lane state that is touched once per frame lives in the LDS (registers hold the weights and the
    // logit bank): the previous super-tile's max / 1/sum / fused accumulator, and the slice's bias
    float4* st = (float4*)(lds + 2 * C::STAGE_U4 + C::XCH_U4) + wave * 12 * 64 + lane;   // st[q * 64], q < 12
    float* lbias = (float*)(lds + 2 * C::STAGE_U4 + C::XCH_U4 + C::ST_U4);
    if (threadIdx.x < 64) lbias[threadIdx.x] = k.bias ? k.bias[ct * 64 + threadIdx.x] : 0.f;   // before the first barrier
    const float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int q = 0; q < 12; ++q) st[q * 64] = zero4;

    struct Tile { int bb, y0, x0; };
    auto decode = [&](int i) {
        int L = sid + i * S;
        Tile t;
        t.x0 = (L % tiles_x) * C::TW; L /= tiles_x;
        t.y0 = (L % tiles_y) * C::TH;
        t.bb = L / tiles_y;
        return t;
    };

    // halo DMA (all NCH chunks of a frame): piece `it` of this wave = item wave + 4 it (clamped: surplus slots
    // rewrite the last piece with identical bytes); lane -> (halo pixel, physical k-group slot)
    const int pix_b = k.x_ld * (int)sizeof(T);
    const unsigned frame_bytes = (unsigned)((long long)k.H * k.W * pix_b);
    // (offsets recomputed per piece: a dozen VALU ops between MFMAs instead of 2 * PER registers, whose
    // spill reloads would wait on vmcnt behind the in-flight feature loads)
    auto dma = [&](int it, const T* xf, int ty0, int tx0, int buf) {
        const int item = min(wave + 4 * it, C::ITEMS - 1);
        const int cch = item / C::IN_ITEMS, ii = item - cch * C::IN_ITEMS;
        int ln = lane;
        asm volatile("" : "+v"(ln));        // keep the lane math here (not hoisted into spilled registers)
        const int p = ii * 16 + (ln >> 2), ph = ln & 3;
        const int gg = 2 * ((ph & 1) ^ ((p >> 2) & 1)) + (ph >> 1);
        const int r = p / C::HWD, cc = p - r * C::HWD;
        const int hy = ty0 - 1 + r, hx = tx0 - 1 + cc;
        const bool ok = p < C::NQ && (unsigned)hy < (unsigned)k.H && (unsigned)hx < (unsigned)k.W;
        const int off = (hy * k.W + hx) * pix_b + cch * 64 + gg * 16;
        blds16(buf_rsrc(xf, frame_bytes), ok ? off : BUF_OOB, lds + buf * C::STAGE_U4 + item * 64);
    };
    auto frame_ptr = [&](const Tile& t, int n) { return (const T*)k.x + map_frame(k.xm, t.bb * NF + n) * k.x_is; };
    // B-fragment of row j at k-step (own chunk c, tap): halo pixel col + (j + ky) * HWD + kx, k-group g
    int in_base[8];
#pragma unroll
    for (int rho = 0; rho < 8; ++rho) in_base[rho] = (kc * NCW) * C::IN_ITEMS * 64 + 4 * col + halo_phys(col + rho, g);
    auto read_b = [&](const u32x4_t* lb, int step, int j) {
        const int c = step / 9, tap = step % 9, ky = tap / 3, kx = tap % 3;
        const int imm = (j + ky) * C::HWD + kx;
        return __builtin_bit_cast(bf16x8_t, lb[c * C::IN_ITEMS * 64 + in_base[imm & 7] + 4 * imm]);
    };
    // K-half exchange: the partial sums of the rows the partner owns (rows 2(1-kc), 2(1-kc)+1), 4 tiles
    // x 16 B per lane, double-buffered by frame parity
    float4* xr = (float4*)(lds + 2 * C::STAGE_U4);
    auto xslot = [&](int pb, int src_kc, int q) { return xr + ((pb * 2 + ch) * 2 + src_kc) * 256 + q * 64 + lane; };

    // fusion operands of super-tile t, frame n, own row r (tile row 2kc + r): 8 channels of one pixel
    auto pix_of = [&](const Tile& t, int r) { return (long long)(t.y0 + 2 * kc + r) * k.W + t.x0 + col; };
    auto feat_ptr = [&](const Tile& t, int n, int r) {
        const T* p = n == 0 ? img_ptr<T>(k.ref, t.bb) + pix_of(t, r) * k.ref.ld
                            : img_ptr<T>(k.oth, t.bb * (NF - 1) + n - 1) + pix_of(t, r) * k.oth.ld;
        return (const u32x4_t*)(p + cl);
    };

    u32x4_t bank[NF][2];                  // 16-bit logits of the own rows, oldest first: [frame][row] x 8 channels
    float m[16], s[16];                   // online max / sum of exp of the current super-tile
    u32x4_t fv[2];                        // prefetched features (next fusion step)
#pragma unroll
    for (int e = 0; e < 16; ++e) { m[e] = -3.0e38f; s[e] = 0.f; }
#pragma unroll
    for (int n = 0; n < NF; ++n) bank[n][0] = bank[n][1] = u32x4_t{0u, 0u, 0u, 0u};
    fv[0] = fv[1] = u32x4_t{0u, 0u, 0u, 0u};

    // fusion step n of super-tile pt (logits bank[slot]); stores the fused result at n = NF-1
    auto fuse_step = [&](const Tile& pt, int n, int slot) {
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            float mp[8], ip[8], fz[8], wv[8];
            *(float4*)mp = st[(2 * r) * 64]; *(float4*)(mp + 4) = st[(2 * r + 1) * 64];
            *(float4*)ip = st[(4 + 2 * r) * 64]; *(float4*)(ip + 4) = st[(5 + 2 * r) * 64];
            *(float4*)fz = st[(8 + 2 * r) * 64]; *(float4*)(fz + 4) = st[(9 + 2 * r) * 64];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const unsigned u = bank[slot][r][e >> 1];
                const float l = (e & 1) ? H16<T>::hi(u) : H16<T>::lo(u);
                wv[e] = __expf(l - mp[e]) * ip[e];
                const float f = (e & 1) ? H16<T>::hi(fv[r][e >> 1]) : H16<T>::lo(fv[r][e >> 1]);
                fz[e] = fmaf(f, wv[e], fz[e]);
            }
            if (k.weights.ptr) {
                T* wp = img_ptr<T>(k.weights, pt.bb * NF + n) + pix_of(pt, r) * k.weights.ld + cl;
                *(u32x4_t*)wp = u32x4_t{H16<T>::pack(wv[0], wv[1]), H16<T>::pack(wv[2], wv[3]),
                                        H16<T>::pack(wv[4], wv[5]), H16<T>::pack(wv[6], wv[7])};
            }
            if (n == NF - 1) {
                T* fp = img_ptr<T>(k.fused, pt.bb) + pix_of(pt, r) * k.fused.ld + cl;
                *(u32x4_t*)fp = u32x4_t{H16<T>::pack(fz[0], fz[1]), H16<T>::pack(fz[2], fz[3]),
                                        H16<T>::pack(fz[4], fz[5]), H16<T>::pack(fz[6], fz[7])};
                st[(8 + 2 * r) * 64] = zero4;
                st[(9 + 2 * r) * 64] = zero4;
            } else {
                st[(8 + 2 * r) * 64] = *(const float4*)fz;
                st[(9 + 2 * r) * 64] = *(const float4*)(fz + 4);
            }
        }
    };
    auto prefetch = [&](const Tile& t, int n) {
        fv[0] = *feat_ptr(t, n, 0);
        fv[1] = *feat_ptr(t, n, 1);
    };
    // the frame's MFMAs over the own K half, with the next frame's halo DMA spread over the first k-steps;
    // then the partner's rows go out to the exchange slots
    f32x4_t acc[2][4];
    auto conv_frame = [&](int buf, int pb, bool more, const T* nxf, int ny0, int nx0) {
        const u32x4_t* lb = lds + buf * C::STAGE_U4;
        bf16x8_t bq[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) bq[j] = read_b(lb, 0, j);
#pragma unroll
        for (int step = 0; step < C::STEPS_W; ++step) {
            // the next frame's halo: one piece per k-step from the first, so the last has ~2/3 of the frame
            // to land (issued in a burst at the frame start they stall the wave instead)
            if (more && step < C::PER) dma(step, nxf, ny0, nx0, buf ^ 1);
            const int c = step / 9, tap = step % 9;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const f32x4_t z = {0.f, 0.f, 0.f, 0.f};
                acc[0][j] = mfma16<T>(wr[c][tap][0], bq[j], step == 0 ? z : acc[0][j]);
                acc[1][j] = mfma16<T>(wr[c][tap][1], bq[j], step == 0 ? z : acc[1][j]);
                if (step + 1 < C::STEPS_W) bq[j] = read_b(lb, step + 1, j);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);     // 2 MFMA
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);     // 1 DS read
            }
        }
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const f32x4_t v = acc[i][2 * (1 - kc) + r];
                *xslot(pb, kc, 2 * r + i) = make_float4(v[0], v[1], v[2], v[3]);
            }
    };
    // after the barrier: own partial + partner's partial (P0 + P1 in either wave: commutative, bitwise equal),
    // bias, rounding to the storage dtype (as the two-kernel path stores the logits), online softmax
    // statistics from the rounded values, into bank[n]
    auto finish_frame = [&](int pb) {
#pragma unroll
        for (int q = 0; q + 1 < NF; ++q) {      // oldest entry out (the fusion step consumed it)
            bank[q][0] = bank[q + 1][0];
            bank[q][1] = bank[q + 1][1];
        }
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            float v[8];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const float4 o = *xslot(pb, 1 - kc, 2 * r + i);
                const f32x4_t a = acc[i][2 * kc + r];
                v[4 * i + 0] = a[0] + o.x; v[4 * i + 1] = a[1] + o.y;
                v[4 * i + 2] = a[2] + o.z; v[4 * i + 3] = a[3] + o.w;
            }
            u32x4_t q;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float2 bv = *(const float2*)(lbias + 32 * ch + 8 * g + 2 * e);
                q[e] = H16<T>::pack(v[2 * e] + bv.x, v[2 * e + 1] + bv.y);
            }
            bank[NF - 1][r] = q;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float l = (e & 1) ? H16<T>::hi(q[e >> 1]) : H16<T>::lo(q[e >> 1]);
                const int x = 8 * r + e;       // (m, s) start a super-tile at (-3e38, 0): no branch on n
                const float mn = fmaxf(m[x], l);
                s[x] = s[x] * __expf(m[x] - mn) + __expf(l - mn);
                m[x] = mn;
            }
        }
    };
    auto close_stats = [&]() {
        float ip[16];
#pragma unroll
        for (int e = 0; e < 16; ++e) ip[e] = 1.f / s[e];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            st[q * 64] = *(const float4*)(m + 4 * q);
            st[(4 + q) * 64] = *(const float4*)(ip + 4 * q);
        }
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            m[e] = -3.0e38f;
            s[e] = 0.f;
        }
    };

    Tile cur = decode(0), prev = cur;
    {
        const T* xf = frame_ptr(cur, 0);
#pragma unroll
        for (int it = 0; it < C::PER; ++it) dma(it, xf, cur.y0, cur.x0, 0);
    }
    // frame (t, n) runs on halo buffer n & 1 and exchange parity n & 1 (NF even)
    static_assert(NF % 2 == 0, "buffer parity per frame index");
    for (int t = 0; t < my_st; ++t) {
        const Tile nxt_st = t + 1 < my_st ? decode(t + 1) : cur;
        for (int n = 0; n < NF; ++n) {
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            __syncthreads();            // halo (t, n) landed; the previous frame's exchange slots are written
            // the previous frame: (t, n-1), or (t-1, NF-1) which also closes super-tile t-1's statistics; the
            // bank then holds (t-1, n .. NF-1), (t, 0 .. n-1): its oldest entry is the fusion step due now
            if (n > 0) {
                finish_frame((n - 1) & 1);
            } else if (t > 0) {
                finish_frame((NF - 1) & 1);
                close_stats();
            }
            // fusion step n of super-tile t-1 (its features arrived with the barrier's vmcnt(0)), then the
            // features of the next step: (t-1, n+1), or step 0 of super-tile t after its last frame
            if (t > 0) fuse_step(prev, n, 0);
            if (n + 1 < NF) {
                if (t > 0) prefetch(prev, n + 1);
            } else {
                prefetch(cur, 0);
            }
            const bool more = n + 1 < NF || t + 1 < my_st;
            const bool same = n + 1 < NF;
            const int nb = __builtin_amdgcn_readfirstlane(same ? cur.bb : nxt_st.bb);
            const int ny0 = __builtin_amdgcn_readfirstlane(same ? cur.y0 : nxt_st.y0);
            const int nx0 = __builtin_amdgcn_readfirstlane(same ? cur.x0 : nxt_st.x0);
            const T* nxf = (const T*)k.x + map_frame(k.xm, nb * NF + (same ? n + 1 : 0)) * k.x_is;
            conv_frame(n & 1, n & 1, more, nxf, ny0, nx0);
        }
        prev = cur;
        cur = nxt_st;
    }
    // the last frame, then the last super-tile's fusion (its step-0 features were prefetched in its last frame)
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
    finish_frame((NF - 1) & 1);
    close_stats();
    StaticFor<0, NF>::run([&](auto n_) {
        constexpr int n = decltype(n_)::value;
        fuse_step(prev, n, n);
        if (n + 1 < NF) prefetch(prev, n + 1);
    });
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

// blocks per XCD for `d` (0: shape not served): 16-bit 3x3/s1/p1 conv, Cin 128 (after padding),
// cout == C a multiple of 64 (<= 1024), frames a multiple of 16 wide and 4 high, burst size 14
int fuse_px(const dbsr_conv_desc* d, int B, int N) {
    if (!d || (d->x.dtype != DBSR_BF16 && d->x.dtype != DBSR_F16) || d->kh != 3 || d->kw != 3 || d->stride != 1 ||
        d->pad != 1 || d->dil != 1 || d->precise)
        return 0;
    if (cin_pad32(d->cin) != 128) return 0;
    if (N != 14 || B <= 0 || d->n_frames != B * N) return 0;
    if (d->cout % 64 || d->cout > 1024 || d->in_h % 4 || d->in_w % 16) return 0;
    if (d->x.ld % 8 || d->x.c0 % 8 || d->x.c0 + 128 > d->x.ld) return 0;
    if ((long long)d->in_h * d->in_w * d->x.ld * 2 >= (1LL << 31)) return 0;
    const int nct = d->cout / 64;
    const long long nsp = (long long)B * (d->in_w / 16) * (d->in_h / 4);
    const long long spx = std::min<long long>(fuse_cus() / 8 / nct, (nsp + 7) / 8);
    if (spx < 1) return 0;
    return (int)(spx * nct);
}

}  // namespace

extern "C" int dbsr_conv_fuse_ok(const dbsr_conv_desc* d, int B, int N) { return fuse_px(d, B, N) > 0; }

extern "C" int dbsr_conv_fuse_softmax(const dbsr_conv_desc* d, int B, int N, dbsr_tensor ref, dbsr_tensor oth,
                                      dbsr_tensor fused, dbsr_tensor weights, void* stream) {
    const int px = fuse_px(d, B, N);
    DBSR_CHECK_ARG(px > 0, "conv_fuse_softmax: unsupported conv / burst (needs dbsr_conv_fuse_ok)");
    DBSR_CHECK_ARG(d->x.ptr && d->w, "conv_fuse_softmax: null pointer");
    const int C = d->cout, dt = d->x.dtype;
    DBSR_CHECK_ARG(ref.ptr && oth.ptr && fused.ptr && ref.dtype == dt && oth.dtype == dt && fused.dtype == dt &&
                   ref.map.fpg > 0 && oth.map.fpg > 0 && fused.map.fpg > 0,
                   "conv_fuse_softmax: ref / oth / fused must be tensors of the conv's dtype");
    DBSR_CHECK_ARG(ref.ld % 4 == 0 && ref.c0 % 4 == 0 && oth.ld % 4 == 0 && oth.c0 % 4 == 0 && fused.ld % 4 == 0 &&
                   fused.c0 % 4 == 0, "conv_fuse_softmax: ld/c0 must be multiples of 4");
    if (weights.ptr)
        DBSR_CHECK_ARG(weights.dtype == dt && weights.map.fpg > 0 && weights.ld % 4 == 0 && weights.c0 % 4 == 0,
                       "conv_fuse_softmax: bad weights tensor");
    FuseK k;
    const int esz = 2;
    k.x = (const char*)d->x.ptr + (long long)d->x.c0 * esz;
    k.x_is = d->x.img_stride; k.x_ld = d->x.ld; k.xm = d->x.map;
    k.H = d->in_h; k.W = d->in_w;
    const int cp = cin_pad32(d->cin);
    k.w = d->w; k.Kp = (9 * cp / 8 + 3) / 4 * 4 * 8; k.bias = d->bias;
    k.ref = ref; k.oth = oth; k.fused = fused; k.weights = weights;
    k.B = B; k.N = N; k.C = C;
    const int tiles_x = k.W / 16, tiles_y = k.H / 4, nct = C / 64;
    const int nsp = B * tiles_x * tiles_y;
    hipStream_t s = (hipStream_t)stream;
#define DBSR_FUSE_LAUNCH(TT, NCH)                                                                              \
    hipLaunchKernelGGL((conv_fuse_kernel<TT, NCH, 14>), dim3(8 * px), dim3(256), 0, s, k, tiles_x, tiles_y, nct, \
                       nsp, px)
    if (dt == DBSR_F16)
        DBSR_FUSE_LAUNCH(f16_t, 4);
    else
        DBSR_FUSE_LAUNCH(bf16_t, 4);
#undef DBSR_FUSE_LAUNCH
    DBSR_LAUNCH_CHECK();
    return 0;
}

#else
extern "C" int dbsr_conv_fuse_ok(const dbsr_conv_desc*, int, int) { return 0; }

extern "C" int dbsr_conv_fuse_softmax(const dbsr_conv_desc*, int, int, dbsr_tensor, dbsr_tensor, dbsr_tensor,
                                      dbsr_tensor, void*) {
    DBSR_CHECK_ARG(false, "conv_fuse_softmax: experimental kernel not built (-DDBSR_EXPERIMENTAL=1)");
    return 0;
}
#endif
