// torch.ops.dbsr.* -- the reference's functional sub-seams as PyTorch operators (one
// shared object loaded with torch.ops.load_library, TORCH_LIBRARY(dbsr, m) schemas with a HIP-device
// implementation).  Each op validates its inputs like the reference (TORCH_CHECK on device, dtype,
// contiguity: correlation.py:286-287), lays the NCHW tensors out channels-last for the C ABI of
// libdbsr_hip.so (include/dbsr_hip.h), launches on the current HIP stream and returns NCHW tensors.
//
//   dbsr::correlation(first, second, leaky)        external/pwcnet/correlation/correlation.py:278-330,385
//   dbsr::correlation_backward(...)                correlation.py:332-383 (K3/K4)
//   dbsr::backwarp(input, flow)                    models/alignment/pwcnet.py:16-38
//   dbsr::warp_bilinear(feat, flow)                models/layers/warp.py:19-46
//   dbsr::warp_bilinear_backward(grad, flow)       (grid_sample backward w.r.t. the features)
//   dbsr::fuse_softmax(logits, feats, want_weights) models/dbsr/merging.py:116-126
//   dbsr::fuse_backward(weights, feats, fused, dfused)
//   dbsr::conv2d_fused(x, w, b, stride, padding, dilation, act, residual, post_act)
//                                                  nn.Conv2d + models/layers/blocks.py:46-96 epilogues
// Autograd formulas for correlation / warp / fusion are registered from Python (dbsr_amd/torch_ops.py)
// with torch.library.register_autograd on top of the *_backward ops.
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <torch/library.h>

#include <map>
#include <mutex>
#include <optional>
#include <tuple>
#include <vector>

#include "../../../include/dbsr_hip.h"

namespace {

int dcode(at::ScalarType t) {
    switch (t) {
        case at::kFloat: return DBSR_F32;
        case at::kBFloat16: return DBSR_BF16;
        case at::kHalf: return DBSR_F16;
        default: TORCH_CHECK(false, "dbsr: unsupported dtype ", t, " (float32, bfloat16, float16)");
    }
    return -1;
}

void check(int rc, const char* what) {
    TORCH_CHECK(rc == 0, what, " failed (rc=", rc, "): ", dbsr_last_error());
}

void* cur_stream() { return (void*)at::hip::getCurrentHIPStream().stream(); }

int64_t r8(int64_t c) { return (c + 7) / 8 * 8; }
int64_t conv_ld(int64_t c) { return c <= 16 ? r8(c) : (c + 31) / 32 * 32; }   // dbsr_conv2d channel padding

// [N,C,H,W] -> zero-padded channels-last [N,H,W,ld]
at::Tensor nhwc(const at::Tensor& x, int64_t ld, at::ScalarType dt) {
    auto t = x.permute({0, 2, 3, 1}).to(dt);
    auto out = at::zeros({x.size(0), x.size(2), x.size(3), ld}, x.options().dtype(dt));
    out.narrow(3, 0, x.size(1)).copy_(t);
    return out;
}
at::Tensor nchw(const at::Tensor& y, int64_t c) { return y.narrow(3, 0, c).permute({0, 3, 1, 2}).contiguous(); }

dbsr_tensor desc(const at::Tensor& t, int64_t ld, int64_t c0 = 0, int64_t img_stride = -1, dbsr_frame_map m = {1, 1, 0, 1}) {
    dbsr_tensor d;
    d.ptr = t.data_ptr();
    d.dtype = dcode(t.scalar_type());
    d.img_stride = img_stride >= 0 ? img_stride : (t.dim() > 1 ? t[0].numel() : t.numel());
    d.ld = (int)ld;
    d.c0 = (int)c0;
    d.map = m;
    return d;
}
dbsr_tensor null_desc() {
    dbsr_tensor d{};
    d.map = {1, 1, 0, 1};
    return d;
}

void need_hip(const at::Tensor& t, const char* name) {
    TORCH_CHECK(t.is_cuda(), "dbsr::", name, ": inputs must be on the HIP device (correlation.py:324-325 has no "
                "CPU path either)");
}

// ------------------------------------------------------------------------------------------------
at::Tensor correlation(const at::Tensor& first, const at::Tensor& second, bool leaky) {
    need_hip(first, "correlation");
    TORCH_CHECK(first.is_contiguous() && second.is_contiguous(), "dbsr::correlation: inputs must be contiguous "
                "(correlation.py:286-287)");
    TORCH_CHECK(first.sizes() == second.sizes() && first.dim() == 4, "dbsr::correlation: [N,C,H,W] inputs of equal shape");
    const int64_t N = first.size(0), C = first.size(1), H = first.size(2), W = first.size(3);
    const auto dt = first.scalar_type();
    auto a = nhwc(first, r8(C), dt), b = nhwc(second, r8(C), dt);
    auto out = at::zeros({N, H, W, 88}, first.options());
    check(dbsr_correlation(N, H, W, C, desc(a, r8(C)), desc(b, r8(C)), desc(out, 88), leaky ? 1 : 0, cur_stream()),
          "dbsr_correlation");
    return nchw(out, 81);
}

std::tuple<at::Tensor, at::Tensor> correlation_backward(const at::Tensor& grad, const at::Tensor& first,
                                                        const at::Tensor& second, const at::Tensor& out, bool leaky) {
    need_hip(grad, "correlation_backward");
    const int64_t N = first.size(0), C = first.size(1), H = first.size(2), W = first.size(3);
    const auto dt = first.scalar_type();
    auto a = nhwc(first, r8(C), dt), b = nhwc(second, r8(C), dt);
    auto g = nhwc(grad, 88, dt), o = nhwc(out, 88, dt);
    auto da = at::zeros_like(a), db = at::zeros_like(b);
    check(dbsr_correlation_backward(N, H, W, C, desc(a, r8(C)), desc(b, r8(C)), desc(o, 88), desc(g, 88),
                                    leaky ? 1 : 0, desc(da, r8(C)), desc(db, r8(C)), cur_stream()),
          "dbsr_correlation_backward");
    return {nchw(da, C), nchw(db, C)};
}

at::Tensor backwarp(const at::Tensor& input, const at::Tensor& flow) {
    need_hip(input, "backwarp");
    TORCH_CHECK(input.dim() == 4 && flow.dim() == 4 && flow.size(1) == 2, "dbsr::backwarp: [N,C,H,W] x [N,2,H,W]");
    const int64_t N = input.size(0), C = input.size(1), H = input.size(2), W = input.size(3);
    const auto dt = input.scalar_type();
    auto x = nhwc(input, r8(C), dt);
    auto fl = flow.permute({0, 2, 3, 1}).to(at::kFloat).contiguous();
    auto out = at::zeros_like(x);
    check(dbsr_backwarp(N, H, W, C, desc(x, r8(C)), desc(fl, 2), 1.0f, desc(out, r8(C)), cur_stream()),
          "dbsr_backwarp");
    return nchw(out, C);
}

at::Tensor warp_bilinear(const at::Tensor& feat, const at::Tensor& flow) {
    need_hip(feat, "warp_bilinear");
    TORCH_CHECK(feat.dim() == 4 && flow.dim() == 4 && flow.size(1) == 2, "dbsr::warp_bilinear: [N,C,H,W] x [N,2,H,W]");
    const int64_t N = feat.size(0), C = feat.size(1), H = feat.size(2), W = feat.size(3);
    const auto dt = feat.scalar_type();
    auto x = nhwc(feat, r8(C), dt);
    auto fl = flow.to(at::kFloat).contiguous();
    auto out = at::zeros_like(x);
    check(dbsr_warp_bilinear(N, H, W, r8(C), desc(x, r8(C)), fl.data_ptr<float>(), 2 * H * W, desc(out, r8(C)),
                             cur_stream()),
          "dbsr_warp_bilinear");
    return nchw(out, C);
}

at::Tensor warp_bilinear_backward(const at::Tensor& grad, const at::Tensor& flow) {
    need_hip(grad, "warp_bilinear_backward");
    const int64_t N = grad.size(0), C = grad.size(1), H = grad.size(2), W = grad.size(3);
    auto g = nhwc(grad, r8(C), grad.scalar_type());
    auto fl = flow.to(at::kFloat).contiguous();
    auto out = at::zeros({N, H, W, r8(C)}, grad.options().dtype(at::kFloat));
    check(dbsr_warp_backward(N, H, W, r8(C), desc(g, r8(C)), fl.data_ptr<float>(), 2 * H * W, out.data_ptr<float>(),
                             dbsr_frame_map{1, 1, 0, 1}, H * W * r8(C), cur_stream()),
          "dbsr_warp_backward");
    return nchw(out, C).to(grad.scalar_type());
}

// feats [B,N,C,H,W] (frame 0 = the reference), logits [B,N,C,H,W] -> (fused [B,C,H,W], weights [B,N,C,H,W])
std::tuple<at::Tensor, at::Tensor> fuse_softmax(const at::Tensor& logits, const at::Tensor& feats, bool want_weights) {
    need_hip(logits, "fuse_softmax");
    TORCH_CHECK(logits.dim() == 5 && logits.sizes() == feats.sizes(), "dbsr::fuse_softmax: [B,N,C,H,W] inputs");
    const int64_t B = feats.size(0), N = feats.size(1), C = feats.size(2), H = feats.size(3), W = feats.size(4);
    TORCH_CHECK(C % 4 == 0, "dbsr::fuse_softmax: C % 4 == 0");
    const auto dt = feats.scalar_type();
    auto cl = [&](const at::Tensor& t) { return t.to(dt).reshape({B * N, C, H, W}).permute({0, 2, 3, 1}).contiguous(); };
    auto l = cl(logits), f = cl(feats);
    auto fused = at::empty({B, H, W, C}, feats.options());
    auto w = want_weights ? at::empty({B * N, H, W, C}, feats.options()) : at::Tensor();
    const int64_t img = H * W * C;
    check(dbsr_fuse_softmax(B, N, H * W, C, desc(l, C, 0, img), desc(f, C, 0, img, {1, (int)N, 0, 1}),
                            desc(f, C, 0, img, {(int)(N - 1), (int)N, 1, 1}), desc(fused, C, 0, img),
                            want_weights ? desc(w, C, 0, img) : null_desc(), cur_stream()),
          "dbsr_fuse_softmax");
    auto wout = want_weights ? w.view({B, N, H, W, C}).permute({0, 1, 4, 2, 3}).contiguous()
                             : at::empty({0}, feats.options());
    return {fused.permute({0, 3, 1, 2}).contiguous(), wout};
}

std::tuple<at::Tensor, at::Tensor> fuse_backward(const at::Tensor& weights, const at::Tensor& feats,
                                                 const at::Tensor& fused, const at::Tensor& dfused) {
    need_hip(weights, "fuse_backward");
    const int64_t B = feats.size(0), N = feats.size(1), C = feats.size(2), H = feats.size(3), W = feats.size(4);
    TORCH_CHECK(C % 8 == 0, "dbsr::fuse_backward: C % 8 == 0");
    const auto dt = feats.scalar_type();
    auto cl5 = [&](const at::Tensor& t) { return t.to(dt).reshape({-1, C, H, W}).permute({0, 2, 3, 1}).contiguous(); };
    auto w = cl5(weights), f = cl5(feats), fu = cl5(fused), dfu = cl5(dfused);
    auto dl = at::empty_like(w), df = at::empty_like(f);
    const int64_t img = H * W * C;
    check(dbsr_fuse_backward(B, N, H * W, C, desc(w, C, 0, img), desc(f, C, 0, img, {1, (int)N, 0, 1}),
                             desc(f, C, 0, img, {(int)(N - 1), (int)N, 1, 1}), desc(fu, C, 0, img),
                             desc(dfu, C, 0, img), desc(dl, C, 0, img), desc(df, C, 0, img, {1, (int)N, 0, 1}),
                             desc(df, C, 0, img, {(int)(N - 1), (int)N, 1, 1}), cur_stream()),
          "dbsr_fuse_backward");
    auto back = [&](const at::Tensor& t) { return t.view({B, N, H, W, C}).permute({0, 1, 4, 2, 3}).contiguous(); };
    return {back(dl), back(df)};
}

// Packed weights, one cache entry per weight tensor (repacking on every call is what made the op-level conv
// slow).  An entry is valid only while it describes the same live tensors: weak
// references to the weight's and the bias's TensorImpl (a freed tensor whose address a new one reuses never
// matches), their versions (an optimizer step bumps them and repacks once), data pointers, shapes and the
// compute dtype.  A stale entry is replaced, and entries of freed weights are evicted on every insert, so the
// cache holds at most one packed copy per live weight.  In-place writes that bypass version counting
// (`p.data.copy_(...)`, raw pointers) are invisible to it: call torch.ops.dbsr.clear_pack_cache() after them.
using WeakImpl = c10::weak_intrusive_ptr<c10::TensorImpl, c10::UndefinedTensorImpl>;
struct PackEntry {
    std::optional<WeakImpl> w, b;  // b empty when the conv has no bias
    int64_t w_version = -1, b_version = -1;
    const void* w_ptr = nullptr;
    const void* b_ptr = nullptr;
    std::vector<int64_t> w_shape;
    int dtype = -1;
    at::Tensor wp, bp;
};
std::mutex g_pack_mu;
std::map<const c10::TensorImpl*, PackEntry> g_pack_cache;

bool same_live(const std::optional<WeakImpl>& weak, const at::Tensor& t) {
    if (!weak) return false;
    auto strong = weak->lock();
    return strong.defined() && strong.get() == t.unsafeGetTensorImpl();
}

bool entry_valid(const PackEntry& e, const at::Tensor& w, const c10::optional<at::Tensor>& bias, int dc) {
    if (!same_live(e.w, w) || e.w_version != (int64_t)w._version() || e.w_ptr != w.data_ptr() ||
        e.w_shape != w.sizes().vec() || e.dtype != dc)
        return false;
    const bool has_b = bias.has_value() && bias->defined();
    if (has_b != e.bp.defined()) return false;
    if (has_b && (!same_live(e.b, *bias) || e.b_version != (int64_t)bias->_version() || e.b_ptr != bias->data_ptr()))
        return false;
    return true;
}

void clear_pack_cache() {
    std::lock_guard<std::mutex> lk(g_pack_mu);
    g_pack_cache.clear();
}

int64_t pack_cache_size() {
    std::lock_guard<std::mutex> lk(g_pack_mu);
    return (int64_t)g_pack_cache.size();
}

at::Tensor conv2d_fused(const at::Tensor& x, const at::Tensor& weight, const c10::optional<at::Tensor>& bias,
                        int64_t stride, int64_t padding, int64_t dilation, int64_t act,
                        const c10::optional<at::Tensor>& residual, int64_t post_act) {
    need_hip(x, "conv2d_fused");
    TORCH_CHECK(x.dim() == 4 && weight.dim() == 4 && weight.size(1) == x.size(1), "dbsr::conv2d_fused: shapes");
    const auto dt = x.scalar_type();
    const int dc = dcode(dt);
    const int64_t N = x.size(0), Cin = x.size(1), H = x.size(2), W = x.size(3);
    const int64_t Cout = weight.size(0), kh = weight.size(2), kw = weight.size(3);
    const int64_t oh = (H + 2 * padding - dilation * (kh - 1) - 1) / stride + 1;
    const int64_t ow = (W + 2 * padding - dilation * (kw - 1) - 1) / stride + 1;
    void* s = cur_stream();
    at::Tensor wp, bp;
    const bool has_b = bias.has_value() && bias->defined();
    if (has_b) TORCH_CHECK(bias->dim() == 1 && bias->size(0) == Cout, "dbsr::conv2d_fused: bias must be [Cout]");
    {
        std::lock_guard<std::mutex> lk(g_pack_mu);
        auto it = g_pack_cache.find(weight.unsafeGetTensorImpl());
        if (it != g_pack_cache.end() && entry_valid(it->second, weight, bias, dc)) {
            wp = it->second.wp;
            bp = it->second.bp;
        } else {
            auto w32 = weight.to(at::kFloat).contiguous();
            auto b32 = has_b ? bias->to(at::kFloat).contiguous() : at::Tensor();
            wp = at::empty({(int64_t)dbsr_conv_packed_elems(Cout, Cin, kh, kw)}, x.options());
            bp = has_b ? at::empty({Cout}, x.options().dtype(at::kFloat)) : at::Tensor();
            check(dbsr_conv_pack_weights(w32.data_ptr<float>(), has_b ? b32.data_ptr<float>() : nullptr,
                                         Cout, Cin, kh, kw, dc, 1, wp.data_ptr(),
                                         has_b ? bp.data_ptr<float>() : nullptr, s),
                  "dbsr_conv_pack_weights");
            // evict entries whose weight is gone, then (re)place this weight's entry
            for (auto e = g_pack_cache.begin(); e != g_pack_cache.end();)
                e = (!e->second.w || e->second.w->expired()) ? g_pack_cache.erase(e) : std::next(e);
            PackEntry ent;
            ent.w.emplace(weight.getIntrusivePtr());
            ent.w_version = weight._version();
            ent.w_ptr = weight.data_ptr();
            ent.w_shape = weight.sizes().vec();
            ent.dtype = dc;
            if (has_b) {
                ent.b.emplace(bias->getIntrusivePtr());
                ent.b_version = bias->_version();
                ent.b_ptr = bias->data_ptr();
            }
            ent.wp = wp;
            ent.bp = bp;
            g_pack_cache.insert_or_assign(weight.unsafeGetTensorImpl(), std::move(ent));
        }
    }
    auto xs = nhwc(x, conv_ld(Cin), dt);
    const int64_t ldy = r8(Cout);
    auto y = at::zeros({N, oh, ow, ldy}, x.options());
    at::Tensor rr;
    dbsr_conv_desc d{};
    d.n_frames = N;
    d.x = desc(xs, conv_ld(Cin));
    d.in_h = H; d.in_w = W; d.cin = Cin;
    d.w = wp.data_ptr();
    d.bias = has_b ? bp.data_ptr<float>() : nullptr;
    d.cout = Cout; d.kh = kh; d.kw = kw; d.stride = stride; d.pad = padding; d.dil = dilation;
    d.y = desc(y, ldy);
    d.out_h = oh; d.out_w = ow;
    d.act = act;
    if (residual.has_value()) {
        rr = nhwc(*residual, ldy, dt);
        d.res = desc(rr, ldy);
    } else {
        d.res = null_desc();
    }
    d.gate = null_desc();
    d.post_act = post_act;
    d.out_mode = DBSR_OUT_NHWC;
    d.shuffle = 0;
    const size_t need = dbsr_conv_workspace_bytes(&d);
    auto ws = at::zeros({(int64_t)std::max<size_t>(need / 4, 1)}, x.options().dtype(at::kFloat));
    d.workspace = ws.data_ptr();
    d.workspace_bytes = need;
    d.precise = 0;
    d.max_blocks = 0;
    check(dbsr_conv2d(&d, s), "dbsr_conv2d");
    return nchw(y, Cout);
}

}  // namespace

TORCH_LIBRARY(dbsr, m) {
    m.def("correlation(Tensor first, Tensor second, bool leaky=False) -> Tensor");
    m.def("correlation_backward(Tensor grad, Tensor first, Tensor second, Tensor out, bool leaky) -> (Tensor, Tensor)");
    m.def("backwarp(Tensor input, Tensor flow) -> Tensor");
    m.def("warp_bilinear(Tensor feat, Tensor flow) -> Tensor");
    m.def("warp_bilinear_backward(Tensor grad, Tensor flow) -> Tensor");
    m.def("fuse_softmax(Tensor logits, Tensor feats, bool want_weights=True) -> (Tensor, Tensor)");
    m.def("fuse_backward(Tensor weights, Tensor feats, Tensor fused, Tensor dfused) -> (Tensor, Tensor)");
    m.def("conv2d_fused(Tensor x, Tensor weight, Tensor? bias=None, int stride=1, int padding=0, int dilation=1, "
          "int act=0, Tensor? residual=None, int post_act=0) -> Tensor");
    m.def("clear_pack_cache() -> ()");
    m.impl("clear_pack_cache", &clear_pack_cache);
    m.def("pack_cache_size() -> int");
    m.impl("pack_cache_size", &pack_cache_size);
}

// the ROCm build of PyTorch dispatches HIP tensors under the CUDA key
TORCH_LIBRARY_IMPL(dbsr, CUDA, m) {
    m.impl("correlation", &correlation);
    m.impl("correlation_backward", &correlation_backward);
    m.impl("backwarp", &backwarp);
    m.impl("warp_bilinear", &warp_bilinear);
    m.impl("warp_bilinear_backward", &warp_bilinear_backward);
    m.impl("fuse_softmax", &fuse_softmax);
    m.impl("fuse_backward", &fuse_backward);
    m.impl("conv2d_fused", &conv2d_fused);
}
