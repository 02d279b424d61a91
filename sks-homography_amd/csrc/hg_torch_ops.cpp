// hg_torch_ops.cpp -- the PyTorch-ROCm operators of SURVEY.md 8(b).3, native.
//
// torch.ops.sks_amd.{aca, sks, tensor_aca_rect, tensor_aca_offsets} (+ .out overloads and
// the backward ops) are registered here with the dispatcher: CUDA (= HIP on ROCm) kernels
// that call the C ABI (include/sks_homography.h) on torch's current stream, Meta kernels
// for shape propagation, and C++ autograd for the two TensorACA forms.  Compared with a
// Python custom op this keeps the per-call host cost to one dispatcher hop plus the
// launch, which is what bounds the reference's B = 64 K case (Modules_Runtime_Test.py:
// 286-309 is launch-bound).  There is no CPU kernel: CPU tensors raise.
#include <ATen/ATen.h>
#include <ATen/Parallel.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <c10/core/DeviceGuard.h>
#include <torch/autograd.h>
#include <torch/library.h>

#include <vector>

#include "sks_homography.h"

namespace {

using torch::autograd::AutogradContext;
using torch::autograd::variable_list;

void* stream_of(const at::Tensor& t) {
    return at::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.device().index()).stream();
}

void hip_ok(int rc, const char* fn) {
    TORCH_CHECK(rc == 0, fn, " failed with hipError_t ", rc);
}

// on `dev`; float32 unless `any_float` (the general-quad ops take float64 too and check
// that their tensors agree)
void on_gpu(const at::Tensor& t, const char* name, const at::Device& dev, bool any_float = false) {
    TORCH_CHECK(t.is_cuda(), "sks_amd: ", name, " must be a GPU tensor (no CPU path), got ",
                t.device());
    TORCH_CHECK(t.device() == dev, "sks_amd: ", name, " is on ", t.device(), ", expected ", dev);
    TORCH_CHECK(t.scalar_type() == at::kFloat || (any_float && t.scalar_type() == at::kDouble),
                "sks_amd: ", name, any_float ? " must be float32 or float64, got " : " must be float32, got ",
                t.scalar_type());
}

void check_rect(const at::Tensor& src, const at::Tensor& tar) {
    for (const auto* p : {&src, &tar}) {
        TORCH_CHECK(p->dim() == 3 && p->size(1) == 3 && p->size(2) == 4,
                    "sks_amd::tensor_aca_rect: src/tar must be (B,3,4), got ", p->sizes());
    }
    TORCH_CHECK(src.size(0) == tar.size(0), "sks_amd::tensor_aca_rect: batch sizes differ");
}

void check_out(const at::Tensor& out, at::IntArrayRef shape, const at::Device& dev,
               bool any_float = false) {
    on_gpu(out, "out", dev, any_float);
    TORCH_CHECK(out.sizes() == shape && out.is_contiguous(), "sks_amd: out must be a contiguous ",
                shape, " tensor, got ", out.sizes());
}

// ------------------------------------------------------------------ TensorACA rect
// scale / div as the reference composition takes them (.py:301-302): torch.mul(div, X) and
// scale * h_temp broadcast against the (B,3,1) columns X, h_temp and are assigned into the
// (B,3,1) column of H, so any shape whose broadcast with (B,3,1) is (B,3,1) -- after the
// leading size-1 dimensions beyond three, which the assignment drops -- is accepted: one
// value, (B,1,1) per problem, (3,1) per row, (B,3,1) per (problem, row).  Anything else
// raises, as the reference's assignment would.
struct Bcast {
    int64_t sb = 0, sr = 0;  // element strides along b and r; 0 where broadcast
    bool over_b = false, over_r = false;
};

Bcast bcast_of(const at::Tensor& t, int64_t B, const char* name) {
    std::vector<int64_t> sz(t.sizes().begin(), t.sizes().end());
    std::vector<int64_t> st(t.strides().begin(), t.strides().end());
    while (sz.size() > 3 && sz.front() == 1) {
        sz.erase(sz.begin());
        st.erase(st.begin());
    }
    TORCH_CHECK(sz.size() <= 3, "sks_amd::tensor_aca_rect: ", name, " of shape ", t.sizes(),
                " does not broadcast to the (B,3,1) column it scales (.py:301-302)");
    const int64_t target[3] = {B, 3, 1};
    int64_t s3[3] = {1, 1, 1}, t3[3] = {0, 0, 0};
    const size_t off = 3 - sz.size();
    for (size_t i = 0; i < sz.size(); ++i) {
        s3[off + i] = sz[i];
        t3[off + i] = st[i];
    }
    for (int j = 0; j < 3; ++j)
        TORCH_CHECK(s3[j] == 1 || s3[j] == target[j], "sks_amd::tensor_aca_rect: ", name,
                    " of shape ", t.sizes(), " does not broadcast to (", B, ",3,1) (.py:301-302)");
    Bcast b;
    b.over_b = s3[0] != 1;
    b.over_r = s3[1] != 1;
    b.sb = b.over_b ? t3[0] : 0;
    b.sr = b.over_r ? t3[1] : 0;
    return b;
}

bool one_value(const at::Tensor& t) { return t.numel() == 1; }

// Whose evaluation of the statements to reproduce (HG_ORDER_*, include/sks_homography.h):
// 0 ATen-CPU (the fixtures' order), 1 torch-ROCm (the reference's device='cuda' run).
int order_of(int64_t order) {
    TORCH_CHECK(order == HG_ORDER_ATEN_CPU || order == HG_ORDER_ATEN_ROCM,
                "sks_amd::tensor_aca_rect: order must be 0 (ATen-CPU) or 1 (torch-ROCm), got ",
                order);
    return (int)order;
}

at::Tensor& rect_out(const at::Tensor& src_, const at::Tensor& tar_, const at::Tensor& scale_,
                     const at::Tensor& div_, int64_t order_, at::Tensor& out) {
    const at::Device dev = tar_.device();
    on_gpu(src_, "src", dev);
    on_gpu(tar_, "tar", dev);
    on_gpu(scale_, "scale", dev);
    on_gpu(div_, "div", dev);
    check_rect(src_, tar_);
    const int64_t B = tar_.size(0);
    const Bcast sb = bcast_of(scale_, B, "scale"), db = bcast_of(div_, B, "div");
    check_out(out, {B, 3, 3}, dev);
    const int order = order_of(order_);
    const at::Tensor src = src_.contiguous(), tar = tar_.contiguous();
    const c10::DeviceGuard guard(dev);
    if (order == HG_ORDER_ATEN_ROCM) {
        hip_ok(hg_tensor_aca_rect_order_f32(src.data_ptr<float>(), tar.data_ptr<float>(),
                                            out.data_ptr<float>(), B, scale_.data_ptr<float>(),
                                            sb.sb, sb.sr, div_.data_ptr<float>(), db.sb, db.sr,
                                            order, stream_of(tar)),
               "hg_tensor_aca_rect_order_f32");
        return out;
    }
    if (one_value(scale_) && one_value(div_)) {  // the reference's own (1,) tensors (.py:33-35)
        hip_ok(hg_tensor_aca_rect_f32(src.data_ptr<float>(), tar.data_ptr<float>(),
                                      out.data_ptr<float>(), B, scale_.data_ptr<float>(),
                                      div_.data_ptr<float>(), stream_of(tar)),
               "hg_tensor_aca_rect_f32");
        return out;
    }
    hip_ok(hg_tensor_aca_rect_bcast_f32(src.data_ptr<float>(), tar.data_ptr<float>(),
                                        out.data_ptr<float>(), B, scale_.data_ptr<float>(), sb.sb,
                                        sb.sr, div_.data_ptr<float>(), db.sb, db.sr,
                                        stream_of(tar)),
           "hg_tensor_aca_rect_bcast_f32");
    return out;
}

at::Tensor rect(const at::Tensor& src, const at::Tensor& tar, const at::Tensor& scale,
                const at::Tensor& div, int64_t order) {
    at::Tensor out = at::empty({tar.size(0), 3, 3}, tar.options());
    rect_out(src, tar, scale, div, order, out);
    return out;
}

at::Tensor& rect_scalar_out(const at::Tensor& src_, const at::Tensor& tar_, double scale,
                            double div, at::Tensor& out) {
    const at::Device dev = tar_.device();
    on_gpu(src_, "src", dev);
    on_gpu(tar_, "tar", dev);
    check_rect(src_, tar_);
    const int64_t B = tar_.size(0);
    check_out(out, {B, 3, 3}, dev);
    const at::Tensor src = src_.contiguous(), tar = tar_.contiguous();
    const c10::DeviceGuard guard(dev);
    hip_ok(hg_tensor_aca_rect_f32_hostscalar(src.data_ptr<float>(), tar.data_ptr<float>(),
                                             out.data_ptr<float>(), B, (float)scale, (float)div,
                                             stream_of(tar)),
           "hg_tensor_aca_rect_f32_hostscalar");
    return out;
}

at::Tensor rect_scalar(const at::Tensor& src, const at::Tensor& tar, double scale, double div) {
    at::Tensor out = at::empty({tar.size(0), 3, 3}, tar.options());
    rect_scalar_out(src, tar, scale, div, out);
    return out;
}

// ATen autograd reduces a broadcast parameter's (B,3,1) gradient terms with ATen-CPU's sum
// (the reference runs its statements under .backward(), Modules_Runtime_Test.py:301-302):
// its order depends on the vector width of the sum kernel -- 8 lanes on every x86 capability
// (its AVX-512 build is not used for sums; measured, tests/test_aten_sum_order.py) -- and,
// for a batch-uniform parameter of >= 32768 terms, on at::get_num_threads().  The op takes
// the caller's thread count, so its gradient equals the one ATen-CPU autograd gives in the
// calling process; aten_threads > 0 names another (a fixture made elsewhere).
constexpr int kAtenLanes = 8;

int aten_threads_of(int64_t requested) {
    const int64_t t = requested > 0 ? requested : at::get_num_threads();
    return (int)(t < 1 ? 1 : (t > 1024 ? 1024 : t));
}

// How the kernel writes a parameter's terms (hg_tensor_aca_rect_bcast_backward_f32's modes):
// per problem (final for (B,1,1)), (3,B) rows, or (B,3) in ATen's full-reduction order.
int terms_mode(const Bcast& b) {
    if (b.over_b) return b.over_r ? 1 : 0;
    return b.over_r ? 1 : 2;
}

// In torch-ROCm's order a batch-reduced parameter's terms are always laid out as the (B,3,1)
// tensor autograd reduces (mode 2), since ROCm's reduction tree depends on that layout.
int terms_mode_for(const Bcast& b, int order) {
    return order == HG_ORDER_ATEN_ROCM && !b.over_b ? 2 : terms_mode(b);
}

// A batch-wide sum of (B,3) terms in torch-ROCm's GPU order (hg_sum_rocm_f32): at::sum_to of
// the (B,3,1) tensor to a (1,) parameter (cols = false) or a (3,1) one (cols = true).
at::Tensor rocm_batch_sum(const at::Tensor& terms, int64_t B, bool cols, void* stream) {
    at::Tensor g = at::empty({cols ? 3 : 1}, terms.options());
    at::Tensor ws = at::empty({HG_SUM_ROCM_WORKSPACE}, terms.options());  // never the output
    hip_ok(hg_sum_rocm_f32(terms.data_ptr<float>(), B, cols ? HG_SUM_ROCM_COLS : HG_SUM_ROCM_FULL,
                           g.data_ptr<float>(), ws.data_ptr<float>(), stream),
           "hg_sum_rocm_f32");
    return g;
}

// A parameter's gradient from the kernel's terms: summed over the dimensions it was
// broadcast along in the evaluation order asked for, and shaped like the parameter.
at::Tensor reduce_param_grad(at::Tensor part, const Bcast& b, const at::Tensor& param, int64_t B,
                             int threads, int order, void* stream) {
    if (b.over_b && b.over_r)  // (3,B) -> (B,3)
        return part.view({3, B}).t().contiguous().reshape(param.sizes());
    if (b.over_b) return part.reshape(param.sizes());  // (B): the per-problem three-row sums
    if (order == HG_ORDER_ATEN_ROCM)  // (B,3) terms
        return rocm_batch_sum(part, B, b.over_r, stream).reshape(param.sizes());
    at::Tensor g = at::empty({b.over_r ? 3 : 1}, part.options());
    // (3,1): each (3,B) row as ATen sums a strided column (one lane, no threads); one value:
    // the (B,3) terms as one run
    const int rc = b.over_r ? hg_sum_aten_f32(part.data_ptr<float>(), 3, B, B, 1, 1, 1,
                                              g.data_ptr<float>(), stream)
                            : hg_sum_aten_f32(part.data_ptr<float>(), 1, 3 * B, 0, 1, kAtenLanes,
                                              threads, g.data_ptr<float>(), stream);
    hip_ok(rc, "hg_sum_aten_f32");
    return g.reshape(param.sizes());
}

// (grad_src (B,3,4) or (0,), grad_tar (B,3,4), grad_scale, grad_div shaped like scale / div,
// or (0,) when not needed)
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> rect_backward(
    const at::Tensor& src_, const at::Tensor& tar_, const at::Tensor& grad_,
    const at::Tensor& scale_, const at::Tensor& div_, bool need_src, bool need_scale_div,
    int64_t aten_threads, int64_t order_) {
    const at::Device dev = tar_.device();
    on_gpu(src_, "src", dev);
    on_gpu(tar_, "tar", dev);
    on_gpu(grad_, "grad", dev);
    on_gpu(scale_, "scale", dev);
    on_gpu(div_, "div", dev);
    check_rect(src_, tar_);
    const int64_t B = tar_.size(0);
    const Bcast sb = bcast_of(scale_, B, "scale"), db = bcast_of(div_, B, "div");
    TORCH_CHECK(grad_.dim() == 3 && grad_.size(0) == B && grad_.size(1) == 3 && grad_.size(2) == 3,
                "sks_amd::tensor_aca_rect_backward: grad must be (B,3,3)");
    const at::Tensor src = src_.contiguous(), tar = tar_.contiguous(), grad = grad_.contiguous();
    at::Tensor g_tar = at::empty({B, 3, 4}, tar.options());
    at::Tensor g_src = need_src ? at::empty({B, 3, 4}, tar.options()) : at::empty({0}, tar.options());
    at::Tensor none = at::empty({0}, tar.options());
    const c10::DeviceGuard guard(dev);
    void* st = stream_of(tar);
    const int threads = aten_threads_of(aten_threads);
    const int order = order_of(order_);
    if (one_value(scale_) && one_value(div_)) {
        at::Tensor part = need_scale_div ? at::empty({2, 3 * B}, tar.options()) : none;
        float* gs = need_src && B ? g_src.data_ptr<float>() : nullptr;
        float* pp = need_scale_div && B ? part.data_ptr<float>() : nullptr;
        if (order == HG_ORDER_ATEN_CPU && need_scale_div) {
            // the backward and ATen's batch sum in one pass over the terms (the bits of the
            // terms kernel + hg_sum_aten_f32 below)
            at::Tensor g_sd = at::empty({2}, tar.options());
            hip_ok(hg_tensor_aca_rect_backward_sum_f32(
                       src.data_ptr<float>(), tar.data_ptr<float>(), grad.data_ptr<float>(), B,
                       scale_.data_ptr<float>(), div_.data_ptr<float>(), gs,
                       g_tar.data_ptr<float>(), pp, kAtenLanes, threads, g_sd.data_ptr<float>(), st),
                   "hg_tensor_aca_rect_backward_sum_f32");
            return {g_src, g_tar, g_sd.slice(0, 0, 1).reshape(scale_.sizes()),
                    g_sd.slice(0, 1, 2).reshape(div_.sizes())};
        }
        if (order == HG_ORDER_ATEN_CPU)
            hip_ok(hg_tensor_aca_rect_backward_terms_f32(
                       src.data_ptr<float>(), tar.data_ptr<float>(), grad.data_ptr<float>(), B,
                       scale_.data_ptr<float>(), div_.data_ptr<float>(), gs,
                       g_tar.data_ptr<float>(), pp, st),
                   "hg_tensor_aca_rect_backward_terms_f32");
        else  // the same (2,B,3) terms, the (B,3) halves named apart
            hip_ok(hg_tensor_aca_rect_backward_order_f32(
                       src.data_ptr<float>(), tar.data_ptr<float>(), grad.data_ptr<float>(), B,
                       scale_.data_ptr<float>(), 0, 0, div_.data_ptr<float>(), 0, 0, gs,
                       g_tar.data_ptr<float>(), pp, 2, pp ? pp + 3 * B : nullptr, 2, order, st),
                   "hg_tensor_aca_rect_backward_order_f32");
        if (!need_scale_div) return {g_src, g_tar, none, none};
        if (order == HG_ORDER_ATEN_ROCM)  // each half as torch-ROCm's autograd sums it
            return {g_src, g_tar,
                    rocm_batch_sum(part[0], B, false, st).reshape(scale_.sizes()),
                    rocm_batch_sum(part[1], B, false, st).reshape(div_.sizes())};
        // each half's (B,3) terms summed in ATen-CPU's order (two rows of one call)
        at::Tensor g_sd = at::empty({2}, tar.options());
        hip_ok(hg_sum_aten_f32(part.data_ptr<float>(), 2, 3 * B, 3 * B, 1, kAtenLanes, threads,
                               g_sd.data_ptr<float>(), st),
               "hg_sum_aten_f32");
        return {g_src, g_tar, g_sd.slice(0, 0, 1).reshape(scale_.sizes()),
                g_sd.slice(0, 1, 2).reshape(div_.sizes())};
    }
    // each parameter's terms in the layout its reduction reads (terms_mode_for); in ROCm order
    // the per-problem three-row sums follow the GPU's ((0 + t0) + t2) + t1 and the batch sums
    // its reduction tree (hg_sum_rocm_f32)
    const int ms = terms_mode_for(sb, order), md = terms_mode_for(db, order);
    at::Tensor ps = need_scale_div ? at::empty({ms ? 3 * B : B}, tar.options()) : none;
    at::Tensor pd = need_scale_div ? at::empty({md ? 3 * B : B}, tar.options()) : none;
    hip_ok(hg_tensor_aca_rect_backward_order_f32(
               src.data_ptr<float>(), tar.data_ptr<float>(), grad.data_ptr<float>(), B,
               scale_.data_ptr<float>(), sb.sb, sb.sr, div_.data_ptr<float>(), db.sb, db.sr,
               need_src && B ? g_src.data_ptr<float>() : nullptr, g_tar.data_ptr<float>(),
               need_scale_div && B ? ps.data_ptr<float>() : nullptr, ms,
               need_scale_div && B ? pd.data_ptr<float>() : nullptr, md, order, st),
           "hg_tensor_aca_rect_backward_order_f32");
    if (!need_scale_div) return {g_src, g_tar, none, none};
    return {g_src, g_tar, reduce_param_grad(ps, sb, scale_, B, threads, order, st),
            reduce_param_grad(pd, db, div_, B, threads, order, st)};
}

// ------------------------------------------------------------------ compact offsets form
void check_offsets(const at::Tensor& corner, const at::Tensor& offsets) {
    TORCH_CHECK((offsets.dim() == 3 && offsets.size(1) == 4 && offsets.size(2) == 2) ||
                    (offsets.dim() == 2 && offsets.size(1) == 8),
                "sks_amd::tensor_aca_offsets: offsets must be (B,4,2) or (B,8), got ",
                offsets.sizes());
    TORCH_CHECK(corner.dim() == 2 && corner.size(0) == offsets.size(0) && corner.size(1) == 2,
                "sks_amd::tensor_aca_offsets: corner must be (B,2), got ", corner.sizes());
}

at::Tensor& offsets_out(const at::Tensor& corner_, const at::Tensor& offsets_, double width,
                        double height, at::Tensor& out) {
    const at::Device dev = offsets_.device();
    on_gpu(corner_, "corner", dev);
    on_gpu(offsets_, "offsets", dev);
    check_offsets(corner_, offsets_);
    const int64_t B = offsets_.size(0);
    check_out(out, {B, 3, 3}, dev);
    const at::Tensor corner = corner_.contiguous(), offsets = offsets_.contiguous();
    const c10::DeviceGuard guard(dev);
    hip_ok(hg_tensor_aca_offsets_f32(corner.data_ptr<float>(), offsets.data_ptr<float>(),
                                     out.data_ptr<float>(), B, (float)width, (float)height,
                                     stream_of(offsets)),
           "hg_tensor_aca_offsets_f32");
    return out;
}

at::Tensor offsets_fwd(const at::Tensor& corner, const at::Tensor& offsets, double width,
                       double height) {
    at::Tensor out = at::empty({offsets.size(0), 3, 3}, offsets.options());
    offsets_out(corner, offsets, width, height, out);
    return out;
}

std::tuple<at::Tensor, at::Tensor> offsets_backward(const at::Tensor& corner_,
                                                    const at::Tensor& offsets_,
                                                    const at::Tensor& grad_, double width,
                                                    double height, bool need_corner) {
    const at::Device dev = offsets_.device();
    on_gpu(corner_, "corner", dev);
    on_gpu(offsets_, "offsets", dev);
    on_gpu(grad_, "grad", dev);
    check_offsets(corner_, offsets_);
    const int64_t B = offsets_.size(0);
    TORCH_CHECK(grad_.numel() == B * 9, "sks_amd::tensor_aca_offsets_backward: grad must be (B,3,3)");
    const at::Tensor corner = corner_.contiguous(), offsets = offsets_.contiguous();
    const at::Tensor grad = grad_.contiguous();
    at::Tensor g_off = at::empty(offsets.sizes(), offsets.options());
    at::Tensor g_cor = need_corner ? at::empty({B, 2}, offsets.options())
                                   : at::empty({0}, offsets.options());
    const c10::DeviceGuard guard(dev);
    hip_ok(hg_tensor_aca_offsets_backward_f32(
               corner.data_ptr<float>(), offsets.data_ptr<float>(), grad.data_ptr<float>(), B,
               (float)width, (float)height, g_off.data_ptr<float>(),
               need_corner && B ? g_cor.data_ptr<float>() : nullptr, stream_of(offsets)),
           "hg_tensor_aca_offsets_backward_f32");
    return {g_off, g_cor};
}

// ------------------------------------------------------------------ general-quad ACA / SKS
// ACA_vanilla's layout (Modules_Runtime_Test.py:312): (B,4,2) or (B,8) -> (B,3,3).
template <int ALGO>
at::Tensor& quad_out(const at::Tensor& src_, const at::Tensor& tar_, bool normalize,
                     at::Tensor& out) {
    const at::Device dev = tar_.device();
    on_gpu(src_, "src", dev, true);
    on_gpu(tar_, "tar", dev, true);
    for (const auto* p : {&src_, &tar_}) {
        TORCH_CHECK((p->dim() == 3 && p->size(1) == 4 && p->size(2) == 2) ||
                        (p->dim() == 2 && p->size(1) == 8),
                    "sks_amd::aca/sks: src/tar must be (B,4,2) or (B,8), got ", p->sizes());
    }
    TORCH_CHECK(src_.size(0) == tar_.size(0), "sks_amd::aca/sks: batch sizes differ");
    const int64_t B = tar_.size(0);
    check_out(out, {B, 3, 3}, dev, true);
    const auto dt = tar_.scalar_type();
    TORCH_CHECK((dt == at::kFloat || dt == at::kDouble) && src_.scalar_type() == dt &&
                    out.scalar_type() == dt,
                "sks_amd::aca/sks: src/tar/out must all be float32 or all float64");
    const at::Tensor src = src_.contiguous(), tar = tar_.contiguous();
    const c10::DeviceGuard guard(dev);
    const int flags = normalize ? HG_FLAG_NORMALIZE : 0;
    if (dt == at::kDouble) {
        auto fn = ALGO == 0 ? hg_aca_f64 : hg_sks_f64;
        hip_ok(fn(src.data_ptr<double>(), tar.data_ptr<double>(), out.data_ptr<double>(), B,
                  HG_LAYOUT_AOS, flags, stream_of(tar)),
               ALGO == 0 ? "hg_aca_f64" : "hg_sks_f64");
        return out;
    }
    auto fn = ALGO == 0 ? hg_aca_f32 : hg_sks_f32;
    hip_ok(fn(src.data_ptr<float>(), tar.data_ptr<float>(), out.data_ptr<float>(), B,
              HG_LAYOUT_AOS, flags, stream_of(tar)),
           ALGO == 0 ? "hg_aca_f32" : "hg_sks_f32");
    return out;
}

// ACA_vanilla's gradients (.py:312-388 under ATen autograd): dL/dsrc, dL/dtar shaped like
// src / tar, or (0,) where not needed.
std::tuple<at::Tensor, at::Tensor> aca_backward(const at::Tensor& src_, const at::Tensor& tar_,
                                                const at::Tensor& grad_, bool need_src,
                                                bool need_tar) {
    const at::Device dev = tar_.device();
    on_gpu(src_, "src", dev, true);
    on_gpu(tar_, "tar", dev, true);
    on_gpu(grad_, "grad", dev, true);
    for (const auto* p : {&src_, &tar_}) {
        TORCH_CHECK((p->dim() == 3 && p->size(1) == 4 && p->size(2) == 2) ||
                        (p->dim() == 2 && p->size(1) == 8),
                    "sks_amd::aca_backward: src/tar must be (B,4,2) or (B,8), got ", p->sizes());
    }
    const int64_t B = tar_.size(0);
    TORCH_CHECK(src_.size(0) == B, "sks_amd::aca_backward: batch sizes differ");
    TORCH_CHECK(grad_.numel() == B * 9, "sks_amd::aca_backward: grad must be (B,3,3)");
    const auto dt = tar_.scalar_type();
    TORCH_CHECK((dt == at::kFloat || dt == at::kDouble) && src_.scalar_type() == dt &&
                    grad_.scalar_type() == dt,
                "sks_amd::aca_backward: src/tar/grad must all be float32 or all float64");
    const at::Tensor src = src_.contiguous(), tar = tar_.contiguous(), grad = grad_.contiguous();
    // (0,) placeholders only where a gradient is not wanted (one allocation less per step)
    at::Tensor g_src = at::empty(need_src ? src_.sizes() : at::IntArrayRef{0}, src.options());
    at::Tensor g_tar = at::empty(need_tar ? tar_.sizes() : at::IntArrayRef{0}, tar.options());
    if (B == 0 || (!need_src && !need_tar)) return {g_src, g_tar};
    const c10::DeviceGuard guard(dev);
    if (dt == at::kDouble) {
        hip_ok(hg_aca_backward_f64(src.data_ptr<double>(), tar.data_ptr<double>(),
                                   grad.data_ptr<double>(), B,
                                   need_src ? g_src.data_ptr<double>() : nullptr,
                                   need_tar ? g_tar.data_ptr<double>() : nullptr, stream_of(tar)),
               "hg_aca_backward_f64");
    } else {
        hip_ok(hg_aca_backward_f32(src.data_ptr<float>(), tar.data_ptr<float>(),
                                   grad.data_ptr<float>(), B,
                                   need_src ? g_src.data_ptr<float>() : nullptr,
                                   need_tar ? g_tar.data_ptr<float>() : nullptr, stream_of(tar)),
               "hg_aca_backward_f32");
    }
    return {g_src, g_tar};
}

template <int ALGO>
at::Tensor quad(const at::Tensor& src, const at::Tensor& tar, bool normalize) {
    at::Tensor out = at::empty({tar.size(0), 3, 3}, tar.options());
    quad_out<ALGO>(src, tar, normalize, out);
    return out;
}

// ------------------------------------------------------------------ the general batch solve
// algo 0 ACA, 1 SKS, 2 RHO-GE, 3 GPT-LU (f64 only); layout 0 AoS (n,8)|(n,4,2) -> (n,9),
// 1 SoA (8,n) -> (9,n).  What ops.solve() calls.
using SolveF32 = int (*)(const float*, const float*, float*, int64_t, int, int, void*);
using SolveF64 = int (*)(const double*, const double*, double*, int64_t, int, int, void*);
constexpr SolveF32 kSolveF32[4] = {hg_aca_f32, hg_sks_f32, hg_ge_f32, nullptr};
constexpr SolveF64 kSolveF64[4] = {hg_aca_f64, hg_sks_f64, hg_ge_f64, hg_gpt_f64};

std::vector<int64_t> solve_shape(const at::Tensor& src, const at::Tensor& tar, int64_t layout) {
    TORCH_CHECK(layout == 0 || layout == 1, "sks_amd::solve: layout must be 0 (AoS) or 1 (SoA)");
    if (layout == 0) {
        for (const auto* p : {&src, &tar})
            TORCH_CHECK((p->dim() == 2 && p->size(1) == 8) ||
                            (p->dim() == 3 && p->size(1) == 4 && p->size(2) == 2),
                        "sks_amd::solve: AoS problems must be (n,8) or (n,4,2), got ", p->sizes());
        TORCH_CHECK(src.size(0) == tar.size(0), "sks_amd::solve: src/tar batch sizes differ");
        return {src.size(0), 9};
    }
    for (const auto* p : {&src, &tar})
        TORCH_CHECK(p->dim() == 2 && p->size(0) == 8, "sks_amd::solve: SoA problems must be (8,n), got ",
                    p->sizes());
    TORCH_CHECK(src.size(1) == tar.size(1), "sks_amd::solve: src/tar batch sizes differ");
    return {9, src.size(1)};
}

at::Tensor& solve_out(const at::Tensor& src_, const at::Tensor& tar_, int64_t algo,
                      bool normalize, int64_t layout, at::Tensor& out) {
    const at::Device dev = tar_.device();
    TORCH_CHECK(src_.is_cuda() && tar_.is_cuda() && out.is_cuda(),
                "sks_amd::solve: GPU tensors only (no CPU path)");
    TORCH_CHECK(src_.device() == dev && out.device() == dev, "sks_amd::solve: devices differ");
    const auto dt = tar_.scalar_type();
    TORCH_CHECK((dt == at::kFloat || dt == at::kDouble) && src_.scalar_type() == dt &&
                    out.scalar_type() == dt,
                "sks_amd::solve: src/tar/out must all be float32 or all float64");
    TORCH_CHECK(algo >= 0 && algo <= 3, "sks_amd::solve: algo must be 0..3");
    TORCH_CHECK(!(algo == 3 && dt == at::kFloat), "sks_amd::solve: GPT-LU is float64 only");
    const auto shape = solve_shape(src_, tar_, layout);
    TORCH_CHECK(out.sizes() == at::IntArrayRef(shape) && out.is_contiguous(),
                "sks_amd::solve: out must be a contiguous ", at::IntArrayRef(shape), " tensor");
    const at::Tensor src = src_.contiguous(), tar = tar_.contiguous();
    const int64_t n = layout == 0 ? shape[0] : shape[1];
    const int flags = normalize ? HG_FLAG_NORMALIZE : 0;
    const int lay = layout == 0 ? HG_LAYOUT_AOS : HG_LAYOUT_SOA;
    const c10::DeviceGuard guard(dev);
    const int rc = dt == at::kFloat
                       ? kSolveF32[algo](src.data_ptr<float>(), tar.data_ptr<float>(),
                                         out.data_ptr<float>(), n, lay, flags, stream_of(tar))
                       : kSolveF64[algo](src.data_ptr<double>(), tar.data_ptr<double>(),
                                         out.data_ptr<double>(), n, lay, flags, stream_of(tar));
    hip_ok(rc, "sks_amd::solve");
    return out;
}

at::Tensor solve(const at::Tensor& src, const at::Tensor& tar, int64_t algo, bool normalize,
                 int64_t layout) {
    at::Tensor out = at::empty(solve_shape(src, tar, layout), tar.options());
    solve_out(src, tar, algo, normalize, layout, out);
    return out;
}

// ------------------------------------------------------------------ Meta (shapes only)
at::Tensor meta_b33(const at::Tensor& t) { return at::empty({t.size(0), 3, 3}, t.options()); }

// ------------------------------------------------------------------ autograd
at::Tensor call_rect(const at::Tensor& src, const at::Tensor& tar, const at::Tensor& scale,
                     const at::Tensor& div, int64_t order) {
    static auto op = c10::Dispatcher::singleton()
                         .findSchemaOrThrow("sks_amd::tensor_aca_rect", "")
                         .typed<at::Tensor(const at::Tensor&, const at::Tensor&,
                                           const at::Tensor&, const at::Tensor&, int64_t)>();
    return op.call(src, tar, scale, div, order);
}

// The backward ops are reached through the dispatcher too, so tracing (fake tensors,
// AOT autograd) sees their Meta kernels instead of a raw launch.
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> call_rect_backward(
    const at::Tensor& src, const at::Tensor& tar, const at::Tensor& grad, const at::Tensor& scale,
    const at::Tensor& div, bool need_src, bool need_sd, int64_t threads, int64_t order) {
    static auto op = c10::Dispatcher::singleton()
                         .findSchemaOrThrow("sks_amd::tensor_aca_rect_backward", "")
                         .typed<std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor>(
                             const at::Tensor&, const at::Tensor&, const at::Tensor&,
                             const at::Tensor&, const at::Tensor&, bool, bool, int64_t,
                             int64_t)>();
    return op.call(src, tar, grad, scale, div, need_src, need_sd, threads, order);
}

std::tuple<at::Tensor, at::Tensor> call_offsets_backward(const at::Tensor& corner,
                                                         const at::Tensor& offsets,
                                                         const at::Tensor& grad, double w,
                                                         double h, bool need_corner) {
    static auto op = c10::Dispatcher::singleton()
                         .findSchemaOrThrow("sks_amd::tensor_aca_offsets_backward", "")
                         .typed<std::tuple<at::Tensor, at::Tensor>(
                             const at::Tensor&, const at::Tensor&, const at::Tensor&, double,
                             double, bool)>();
    return op.call(corner, offsets, grad, w, h, need_corner);
}

class RectFunction : public torch::autograd::Function<RectFunction> {
   public:
    static at::Tensor forward(AutogradContext* ctx, const at::Tensor& src, const at::Tensor& tar,
                              const at::Tensor& scale, const at::Tensor& div, int64_t order) {
        at::AutoDispatchBelowADInplaceOrView below;
        ctx->save_for_backward({src, tar, scale, div});
        // the caller's ATen thread count: the backward may run on an autograd device thread
        ctx->saved_data["threads"] = (int64_t)at::get_num_threads();
        ctx->saved_data["order"] = order;
        return call_rect(src, tar, scale, div, order);
    }

    static variable_list backward(AutogradContext* ctx, variable_list grads) {
        const auto saved = ctx->get_saved_variables();
        const at::Tensor &src = saved[0], &tar = saved[1], &scale = saved[2], &div = saved[3];
        const bool need_src = ctx->needs_input_grad(0);
        const bool need_sd = ctx->needs_input_grad(2) || ctx->needs_input_grad(3);
        auto [g_src, g_tar, g_scale, g_div] =
            call_rect_backward(src, tar, grads[0].contiguous(), scale, div, need_src, need_sd,
                               ctx->saved_data["threads"].toInt(), ctx->saved_data["order"].toInt());
        at::Tensor none;
        return {need_src ? g_src : none, ctx->needs_input_grad(1) ? g_tar : none,
                ctx->needs_input_grad(2) ? g_scale : none, ctx->needs_input_grad(3) ? g_div : none,
                none};
    }
};

bool any_requires_grad(std::initializer_list<const at::Tensor*> ts) {
    if (!at::GradMode::is_enabled()) return false;
    for (const at::Tensor* t : ts)
        if (t->requires_grad()) return true;
    return false;
}

at::Tensor rect_autograd(const at::Tensor& src, const at::Tensor& tar, const at::Tensor& scale,
                         const at::Tensor& div, int64_t order) {
    if (!any_requires_grad({&src, &tar, &scale, &div})) {  // inference: no graph node
        at::AutoDispatchBelowADInplaceOrView below;
        return call_rect(src, tar, scale, div, order);
    }
    return RectFunction::apply(src, tar, scale, div, order);
}

at::Tensor call_rect_scalar(const at::Tensor& src, const at::Tensor& tar, double scale, double div) {
    static auto op = c10::Dispatcher::singleton()
                         .findSchemaOrThrow("sks_amd::tensor_aca_rect", "scalar")
                         .typed<at::Tensor(const at::Tensor&, const at::Tensor&, double, double)>();
    return op.call(src, tar, scale, div);
}

// tensor_aca_rect.scalar: scale / div are constants, so src and tar are the only inputs with a
// gradient -- the tensor overload's backward with the two values as (1,) device tensors
// (the same float32 values the forward's host-scalar kernel uses).
class RectScalarFunction : public torch::autograd::Function<RectScalarFunction> {
   public:
    static at::Tensor forward(AutogradContext* ctx, const at::Tensor& src, const at::Tensor& tar,
                              double scale, double div) {
        at::AutoDispatchBelowADInplaceOrView below;
        ctx->save_for_backward({src, tar});
        ctx->saved_data["scale"] = scale;
        ctx->saved_data["div"] = div;
        return call_rect_scalar(src, tar, scale, div);
    }

    static variable_list backward(AutogradContext* ctx, variable_list grads) {
        const auto saved = ctx->get_saved_variables();
        const auto opts = saved[1].options();
        const at::Tensor sc = at::full({1}, (float)ctx->saved_data["scale"].toDouble(), opts);
        const at::Tensor dv = at::full({1}, (float)ctx->saved_data["div"].toDouble(), opts);
        const bool need_src = ctx->needs_input_grad(0);
        auto [g_src, g_tar, g_sc, g_dv] =
            call_rect_backward(saved[0], saved[1], grads[0].contiguous(), sc, dv, need_src, false, 0,
                               HG_ORDER_ATEN_CPU);
        at::Tensor none;
        return {need_src ? g_src : none, ctx->needs_input_grad(1) ? g_tar : none, none, none};
    }
};

at::Tensor rect_scalar_autograd(const at::Tensor& src, const at::Tensor& tar, double scale,
                                double div) {
    if (!any_requires_grad({&src, &tar})) {
        at::AutoDispatchBelowADInplaceOrView below;
        return call_rect_scalar(src, tar, scale, div);
    }
    return RectScalarFunction::apply(src, tar, scale, div);
}

at::Tensor call_aca(const at::Tensor& src, const at::Tensor& tar, bool normalize) {
    static auto op = c10::Dispatcher::singleton()
                         .findSchemaOrThrow("sks_amd::aca", "")
                         .typed<at::Tensor(const at::Tensor&, const at::Tensor&, bool)>();
    return op.call(src, tar, normalize);
}

std::tuple<at::Tensor, at::Tensor> call_aca_backward(const at::Tensor& src, const at::Tensor& tar,
                                                     const at::Tensor& grad, bool need_src,
                                                     bool need_tar) {
    static auto op = c10::Dispatcher::singleton()
                         .findSchemaOrThrow("sks_amd::aca_backward", "")
                         .typed<std::tuple<at::Tensor, at::Tensor>(
                             const at::Tensor&, const at::Tensor&, const at::Tensor&, bool, bool)>();
    return op.call(src, tar, grad, need_src, need_tar);
}

// ACA_vanilla is differentiable in the reference (ATen autograd through its statements,
// .py:322-382); the normalised form is the C++ API's (ACA_SKS.cpp:94-98), which nothing
// differentiates, so it is refused rather than given a gradient the reference never defines.
class AcaFunction : public torch::autograd::Function<AcaFunction> {
   public:
    static at::Tensor forward(AutogradContext* ctx, const at::Tensor& src, const at::Tensor& tar) {
        at::AutoDispatchBelowADInplaceOrView below;
        ctx->save_for_backward({src, tar});
        return call_aca(src, tar, false);
    }

    static variable_list backward(AutogradContext* ctx, variable_list grads) {
        const auto saved = ctx->get_saved_variables();
        const bool need_src = ctx->needs_input_grad(0), need_tar = ctx->needs_input_grad(1);
        auto [g_src, g_tar] =
            call_aca_backward(saved[0], saved[1], grads[0].contiguous(), need_src, need_tar);
        at::Tensor none;
        return {need_src ? g_src : none, need_tar ? g_tar : none};
    }
};

// One policy for the three forms nothing in the reference differentiates (aca with
// normalize=True, solve, sks): an input that requires grad while grad mode is on is refused,
// naming the differentiable form, instead of a result whose graph is silently cut.  Under
// torch.no_grad() or on detached inputs they run as inference.
at::Tensor aca_autograd(const at::Tensor& src, const at::Tensor& tar, bool normalize) {
    const bool grad = any_requires_grad({&src, &tar});
    TORCH_CHECK(!(grad && normalize),
                "sks_amd::aca: normalize=True (the C++ API's H/H[8], ACA_SKS.cpp:94-98) has no "
                "backward in the reference; call it on detached inputs or under torch.no_grad(), "
                "or use normalize=False (ACA_vanilla's form, Modules_Runtime_Test.py:312-388), "
                "which is differentiable");
    if (!grad) {
        at::AutoDispatchBelowADInplaceOrView below;
        return call_aca(src, tar, normalize);
    }
    return AcaFunction::apply(src, tar);
}

// sks_amd::solve is the C++ API's batch mirror (sks::runKernel_*, normalised by default):
// nothing differentiates it in the reference, so inputs that require grad are refused.
at::Tensor solve_autograd(const at::Tensor& src, const at::Tensor& tar, int64_t algo,
                          bool normalize, int64_t layout) {
    TORCH_CHECK(!any_requires_grad({&src, &tar}),
                "sks_amd::solve has no backward (the C++ API it mirrors, ACA_SKS.cpp, is not "
                "differentiated by the reference); call it on detached inputs or under "
                "torch.no_grad(), or use sks_amd::aca (normalize=False) for gradients");
    static auto op = c10::Dispatcher::singleton()
                         .findSchemaOrThrow("sks_amd::solve", "")
                         .typed<at::Tensor(const at::Tensor&, const at::Tensor&, int64_t, bool,
                                           int64_t)>();
    at::AutoDispatchBelowADInplaceOrView below;
    return op.call(src, tar, algo, normalize, layout);
}

at::Tensor call_sks(const at::Tensor& src, const at::Tensor& tar, bool normalize) {
    static auto op = c10::Dispatcher::singleton()
                         .findSchemaOrThrow("sks_amd::sks", "")
                         .typed<at::Tensor(const at::Tensor&, const at::Tensor&, bool)>();
    return op.call(src, tar, normalize);
}

// The reference has no differentiable SKS (its PyTorch file composes ACA only, .py:286-388),
// so an input that requires grad is refused here instead of reaching autograd's
// not-implemented fallback (a warning now, an error at .backward()).
at::Tensor sks_autograd(const at::Tensor& src, const at::Tensor& tar, bool normalize) {
    TORCH_CHECK(!any_requires_grad({&src, &tar}),
                "sks_amd::sks has no backward (the reference differentiates ACA only: "
                "Modules_Runtime_Test.py:286-388); call it on detached inputs or under "
                "torch.no_grad(), or use sks_amd::aca (normalize=False) for gradients");
    at::AutoDispatchBelowADInplaceOrView below;
    return call_sks(src, tar, normalize);
}

at::Tensor call_offsets(const at::Tensor& corner, const at::Tensor& offsets, double w, double h) {
    static auto op = c10::Dispatcher::singleton()
                         .findSchemaOrThrow("sks_amd::tensor_aca_offsets", "")
                         .typed<at::Tensor(const at::Tensor&, const at::Tensor&, double, double)>();
    return op.call(corner, offsets, w, h);
}

class OffsetsFunction : public torch::autograd::Function<OffsetsFunction> {
   public:
    static at::Tensor forward(AutogradContext* ctx, const at::Tensor& corner,
                              const at::Tensor& offsets, double w, double h) {
        at::AutoDispatchBelowADInplaceOrView below;
        ctx->save_for_backward({corner, offsets});
        ctx->saved_data["w"] = w;
        ctx->saved_data["h"] = h;
        return call_offsets(corner, offsets, w, h);
    }

    static variable_list backward(AutogradContext* ctx, variable_list grads) {
        const auto saved = ctx->get_saved_variables();
        const bool need_c = ctx->needs_input_grad(0);
        auto [g_off, g_cor] =
            call_offsets_backward(saved[0], saved[1], grads[0].contiguous(),
                             ctx->saved_data["w"].toDouble(), ctx->saved_data["h"].toDouble(),
                             need_c);
        at::Tensor none;
        return {need_c ? g_cor : none, ctx->needs_input_grad(1) ? g_off : none, none, none};
    }
};

at::Tensor offsets_autograd(const at::Tensor& corner, const at::Tensor& offsets, double w,
                            double h) {
    if (!any_requires_grad({&corner, &offsets})) {
        at::AutoDispatchBelowADInplaceOrView below;
        return call_offsets(corner, offsets, w, h);
    }
    return OffsetsFunction::apply(corner, offsets, w, h);
}

}  // namespace

TORCH_LIBRARY(sks_amd, m) {
    m.def("aca(Tensor src, Tensor tar, bool normalize=False) -> Tensor");
    m.def("aca.out(Tensor src, Tensor tar, bool normalize=False, *, Tensor(a!) out) -> Tensor(a!)");
    m.def("sks(Tensor src, Tensor tar, bool normalize=False) -> Tensor");
    m.def("sks.out(Tensor src, Tensor tar, bool normalize=False, *, Tensor(a!) out) -> Tensor(a!)");
    m.def("solve(Tensor src, Tensor tar, int algo, bool normalize, int layout) -> Tensor");
    m.def("solve.out(Tensor src, Tensor tar, int algo, bool normalize, int layout, *, "
          "Tensor(a!) out) -> Tensor(a!)");
    m.def("tensor_aca_rect(Tensor src, Tensor tar, Tensor scale, Tensor div, int order=0) -> "
          "Tensor");
    m.def("tensor_aca_rect.out(Tensor src, Tensor tar, Tensor scale, Tensor div, int order=0, *, "
          "Tensor(a!) out) -> Tensor(a!)");
    m.def("tensor_aca_rect.scalar(Tensor src, Tensor tar, float scale, float div) -> Tensor");
    m.def("tensor_aca_rect.scalar_out(Tensor src, Tensor tar, float scale, float div, *, "
          "Tensor(a!) out) -> Tensor(a!)");
    m.def("tensor_aca_rect_backward(Tensor src, Tensor tar, Tensor grad, Tensor scale, "
          "Tensor div, bool need_src, bool need_scale_div, int aten_threads=0, int order=0) -> "
          "(Tensor, Tensor, Tensor, Tensor)");
    m.def("aca_backward(Tensor src, Tensor tar, Tensor grad, bool need_src, bool need_tar) -> "
          "(Tensor, Tensor)");
    m.def("tensor_aca_offsets(Tensor corner, Tensor offsets, float width, float height) -> Tensor");
    m.def("tensor_aca_offsets.out(Tensor corner, Tensor offsets, float width, float height, *, "
          "Tensor(a!) out) -> Tensor(a!)");
    m.def("tensor_aca_offsets_backward(Tensor corner, Tensor offsets, Tensor grad, float width, "
          "float height, bool need_corner) -> (Tensor, Tensor)");
}

TORCH_LIBRARY_IMPL(sks_amd, CUDA, m) {
    m.impl("solve", solve);
    m.impl("solve.out", solve_out);
    m.impl("aca", quad<0>);
    m.impl("aca.out", quad_out<0>);
    m.impl("aca_backward", aca_backward);
    m.impl("sks", quad<1>);
    m.impl("sks.out", quad_out<1>);
    m.impl("tensor_aca_rect", rect);
    m.impl("tensor_aca_rect.out", rect_out);
    m.impl("tensor_aca_rect.scalar", rect_scalar);
    m.impl("tensor_aca_rect.scalar_out", rect_scalar_out);
    m.impl("tensor_aca_rect_backward", rect_backward);
    m.impl("tensor_aca_offsets", offsets_fwd);
    m.impl("tensor_aca_offsets.out", offsets_out);
    m.impl("tensor_aca_offsets_backward", offsets_backward);
}

TORCH_LIBRARY_IMPL(sks_amd, Meta, m) {
    m.impl("solve", [](const at::Tensor& s, const at::Tensor& t, int64_t, bool, int64_t layout) {
        return at::empty(solve_shape(s, t, layout), t.options());
    });
    m.impl("aca", [](const at::Tensor& s, const at::Tensor& t, bool) { return meta_b33(t); });
    m.impl("sks", [](const at::Tensor& s, const at::Tensor& t, bool) { return meta_b33(t); });
    m.impl("tensor_aca_rect", [](const at::Tensor& s, const at::Tensor& t, const at::Tensor& sc,
                                 const at::Tensor& dv, int64_t order) {
        order_of(order);
        check_rect(s, t);
        bcast_of(sc, t.size(0), "scale");  // the shapes the reference composition accepts
        bcast_of(dv, t.size(0), "div");
        return meta_b33(t);
    });
    m.impl("tensor_aca_rect.scalar",
           [](const at::Tensor& s, const at::Tensor& t, double, double) { return meta_b33(t); });
    m.impl("tensor_aca_offsets", [](const at::Tensor& c, const at::Tensor& o, double, double) {
        return meta_b33(o);
    });
    m.impl("tensor_aca_rect_backward",
           [](const at::Tensor& s, const at::Tensor& t, const at::Tensor&, const at::Tensor& sc,
              const at::Tensor& dv, bool need_src, bool need_sd, int64_t, int64_t) {
               const int64_t B = t.size(0);
               return std::make_tuple(need_src ? at::empty({B, 3, 4}, t.options())
                                               : at::empty({0}, t.options()),
                                      at::empty({B, 3, 4}, t.options()),
                                      need_sd ? at::empty(sc.sizes(), t.options())
                                              : at::empty({0}, t.options()),
                                      need_sd ? at::empty(dv.sizes(), t.options())
                                              : at::empty({0}, t.options()));
           });
    m.impl("aca_backward", [](const at::Tensor& s, const at::Tensor& t, const at::Tensor&,
                              bool need_src, bool need_tar) {
        return std::make_tuple(need_src ? at::empty(s.sizes(), s.options()) : at::empty({0}, s.options()),
                               need_tar ? at::empty(t.sizes(), t.options()) : at::empty({0}, t.options()));
    });
    m.impl("tensor_aca_offsets_backward",
           [](const at::Tensor& c, const at::Tensor& o, const at::Tensor&, double, double,
              bool need_c) {
               return std::make_tuple(at::empty(o.sizes(), o.options()),
                                      need_c ? at::empty({o.size(0), 2}, o.options())
                                             : at::empty({0}, o.options()));
           });
}

TORCH_LIBRARY_IMPL(sks_amd, Autograd, m) {
    m.impl("aca", aca_autograd);
    m.impl("sks", sks_autograd);
    m.impl("solve", solve_autograd);
    m.impl("tensor_aca_rect", rect_autograd);
    m.impl("tensor_aca_rect.scalar", rect_scalar_autograd);
    m.impl("tensor_aca_offsets", offsets_autograd);
}
