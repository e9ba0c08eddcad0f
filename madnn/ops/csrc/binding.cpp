// torch.ops.madnn.* registration for the hand-written gfx950 kernels.
//
// The kernels live in bucket.hip / optim.hip / norm.hip behind a C ABI; this
// file only validates tensors, fetches the current HIP stream and launches.
// Registered for the CUDA dispatch key, which is what ROCm PyTorch uses for
// HIP device tensors.  CPU tensors never reach this file: the Python layer
// (madnn/ops/__init__.py) routes CPU tensors to the eager reference.
#include <torch/library.h>
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <hip/hip_runtime.h>

#include <vector>

#include "attn.h"

extern "C" {
hipError_t madnn_bucket_pack(void* const*, const int64_t*, const int64_t*, int, void*, int, int, float, hipStream_t);
hipError_t madnn_bucket_unpack(void* const*, const int64_t*, const int64_t*, int, void*, int, int, float, hipStream_t);
hipError_t madnn_flat_scale_cast(const void*, void*, int64_t, int, int, float, hipStream_t);
hipError_t madnn_sgd_step(float*, const void*, int, float*, void*, int, int64_t, float, float, float, float, int, int,
                          float, const float*, hipStream_t);
hipError_t madnn_adam_step(float*, const void*, int, float*, float*, void*, int, int64_t, float, float, float, float,
                           float, int, float, float, float, const float*, hipStream_t);
int madnn_sqnorm_grid(int64_t);
hipError_t madnn_sqnorm_partial(const void*, int, int64_t, float, float*, int, hipStream_t);
hipError_t madnn_norm_finalize(const float*, int, float, float*, hipStream_t);
hipError_t madnn_norm_fwd(const void*, const void*, const void*, const void*, void*, void*, float*, float*, int64_t,
                          int, float, int, int, int, hipStream_t);
int64_t madnn_norm_bwd_workspace(int64_t, int);
hipError_t madnn_norm_bwd(const void*, const void*, const void*, const float*, const float*, const void*, void*, void*,
                          void*, void*, int, float*, int64_t, int, int, int, int, hipStream_t);
int madnn_bn_supported(int);
int madnn_bn_partial_rows(int64_t, int);
hipError_t madnn_bn_fwd(const void*, const void*, void*, unsigned char*, int64_t, int, int, int, int, float, float,
                        const float*, const float*, float*, float*, int64_t*, float*, float*, float*, float*, float*,
                        const float*, int, hipStream_t);
int madnn_bias_grad_supported(int64_t, int);
int madnn_bias_grad_rows(int64_t, int, int);
hipError_t madnn_bias_grad(const void*, const void*, void*, int64_t, int, int, float*, void*, int, int, hipStream_t);
hipError_t madnn_gelu_fwd(const void*, void*, int64_t, int, int, hipStream_t);
hipError_t madnn_rope_qkv(const void*, void*, const float*, const float*, int64_t, int, int, int, int, int, hipStream_t);
hipError_t madnn_swiglu_fwd(const void*, void*, int64_t, int, hipStream_t);
hipError_t madnn_swiglu_bwd(const void*, const void*, void*, int64_t, int, hipStream_t);
int madnn_attn_supported(int);
hipError_t madnn_attn_fwd(const MadnnAttnArgs*, int, int, hipStream_t);
hipError_t madnn_attn_bwd(const MadnnAttnArgs*, int, int, hipStream_t);
int64_t madnn_attn_colsum_rows(int, int);
hipError_t madnn_attn_colsum_finalize(const float*, int64_t, int64_t, void*, int, hipStream_t);
int madnn_maxpool_supported(int64_t, int, int);
hipError_t madnn_maxpool_fwd(const void*, void*, void*, int, int, int, int, int, int, int, int, int, int, hipStream_t);
int madnn_pool_bn_supported(int64_t, int);
int madnn_pool_bn_bwd_rows(int64_t, int);
hipError_t madnn_pool_bn_fwd(const void*, const float*, const float*, void*, void*, int, int, int, int, int, int, int,
                             hipStream_t);
hipError_t madnn_pool_bn_bwd(const void*, const void*, const void*, const float*, const float*, const float*,
                             const float*, const float*, void*, float*, float*, float*, float*, int, int, int, int, int,
                             int, int, hipStream_t);
hipError_t madnn_maxpool_bwd(const void*, const void*, void*, int, int, int, int, int, int, int, int, int, int,
                             hipStream_t);
hipError_t madnn_xent_fwd(const void*, int, const int64_t*, int64_t, int64_t, int64_t, int, int, float*, float*,
                          hipStream_t);
hipError_t madnn_xent_bwd(const void*, int, const int64_t*, const float*, int64_t, int64_t, int64_t, int, int, int64_t,
                          const float*, void*, hipStream_t);
int madnn_xent_fused_chunks(int64_t);
hipError_t madnn_xent_fused(const void*, int, const int64_t*, int64_t, int64_t, int64_t, int, int, int64_t,
                            const float*, float*, void*, hipStream_t);
hipError_t madnn_xent_rescale(void*, int, int64_t, const float*, hipStream_t);
hipError_t madnn_bn_bwd(const void*, const void*, const unsigned char*, int, void*, void*, int64_t, int, int, int,
                        const float*, const float*, const float*, const float*, const float*, float*, float*, float*,
                        float*, hipStream_t);
hipError_t madnn_bn_fwd_dual(const void*, const void*, void*, unsigned char*, int64_t, int, float, float, const float*,
                             const float*, float*, float*, int64_t*, float*, float*, float*, float*, const float*, int,
                             float, float, const float*, const float*, float*, float*, int64_t*, float*, float*,
                             float*, float*, const float*, int, float*, hipStream_t);
hipError_t madnn_bn_bwd_dual(const void*, const void*, const void*, const unsigned char*, void*, void*, int64_t, int,
                             const float*, const float*, const float*, const float*, const float*, const float*,
                             float*, float*, float*, float*, float*, float*, hipStream_t);
int madnn_conv1x1_supported(int64_t, int64_t);
int madnn_conv1x1_stat_rows(int64_t, int64_t, int64_t);
hipError_t madnn_conv1x1_fwd(const void*, const void*, void*, float*, int64_t, int64_t, int64_t, hipStream_t);
hipError_t madnn_conv1x1_dgrad(const void*, const void*, void*, const void*, int64_t, int64_t, int64_t, const void*,
                               const float*, const float*, float*, hipStream_t, const unsigned char* = nullptr);
int madnn_conv1x1_dgrad_rows(int64_t, int64_t, int64_t);
int64_t madnn_conv1x1_wgrad_ws(int64_t, int64_t, int64_t);
hipError_t madnn_conv1x1_wgrad(const void*, const void*, void*, int, float*, int64_t, int64_t, int64_t, hipStream_t);
hipError_t madnn_bn_coef(const void*, int64_t, int, float, float, const float*, const float*, float*, float*, int64_t*,
                         float*, float*, float*, float*, float*, const float*, int, hipStream_t);
int madnn_stem_supported(int, int);
int madnn_stem_stat_rows(int, int, int);
hipError_t madnn_stem_fwd(const void*, const void*, void*, float*, int, int, int, hipStream_t);
int64_t madnn_stem_wgrad_ws(int, int, int);
hipError_t madnn_stem_wgrad(const void*, const void*, float*, float*, int, int, int, hipStream_t);
int madnn_gemm_supported(int64_t, int64_t, int64_t, int64_t, int64_t);
int madnn_conv3x3_supported(int, int, int, int);
int madnn_conv3x3_stat_rows(int64_t);
hipError_t madnn_conv3x3_fwd(const void*, const void*, void*, float*, int, int, int, int, int, hipStream_t);
int madnn_conv3x3_s2_supported(int, int, int, int);
int madnn_conv3x3_s2_stat_rows(int, int, int);
hipError_t madnn_conv3x3_fwd_s2(const void*, const void*, void*, float*, int, int, int, int, int, hipStream_t);
int64_t madnn_conv3x3_wgrad_ws(int, int, int, int, int);
hipError_t madnn_conv3x3_fwd_bnb(const void*, const void*, void*, float*, const void*, const float*, const float*, int,
                                 int, int, int, int, hipStream_t);
hipError_t madnn_bn_bwd_ext(const void*, const void*, void*, int64_t, int, int, const float*, const float*,
                            const float*, const float*, const float*, float*, float*, float*, const float*, int, float*,
                            hipStream_t);
int madnn_bn_prereduce_floats(int);
hipError_t madnn_conv3x3_wgrad(const void*, const void*, float*, void*, int, int, int, int, int, int, hipStream_t);
hipError_t madnn_linear_fwd(const void*, const void*, const void*, int, const void*, void*, void*, int, int64_t,
                            int64_t, int64_t, hipStream_t);
hipError_t madnn_linear_dgrad(const void*, const void*, const void*, void*, int64_t, int64_t, int64_t, hipStream_t);
int madnn_wgrad_splits(int64_t, int64_t, int64_t);
hipError_t madnn_linear_wgrad4h(const void*, const void*, void*, float*, int, int, int64_t, int64_t, int64_t,
                                hipStream_t);
hipError_t madnn_linear_wgrad4(const void*, const void*, void*, float*, int, int, int64_t, int64_t, int64_t,
                               hipStream_t);
hipError_t madnn_linear_wgrad(const void*, const void*, void*, float*, int, int, int64_t, int64_t, int64_t,
                              hipStream_t);
int madnn_gemmp_supported(int64_t, int64_t, int64_t, int);
hipError_t madnn_linear_fwd_p(const void*, const void*, const void*, int, void*, void*, int, int64_t, int64_t,
                              int64_t, hipStream_t);
hipError_t madnn_linear_dgrad_p(const void*, const void*, const void*, void*, float*, int64_t, int64_t, int64_t, int,
                                hipStream_t);
hipError_t madnn_colsum_finalize(const float*, int, int64_t, void*, int, hipStream_t);
hipError_t madnn_hwq_wait(const int*, int, int64_t, int*, hipStream_t);
hipError_t madnn_hwq_set(int*, int, hipStream_t);
hipError_t madnn_hwq_batch(const int*, const int*, int, int*, int*, int, int64_t, int*, const int*, hipStream_t);
hipError_t madnn_hwq_spin(int64_t, hipStream_t);
}

namespace {

int dt_code(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return 0;
    case at::kBFloat16: return 1;
    case at::kHalf: return 2;
    default: TORCH_CHECK(false, "madnn: unsupported dtype ", t.scalar_type());
  }
  return -1;
}

hipStream_t cur_stream(const at::Tensor& t) {
  // ROCm PyTorch labels HIP devices "cuda": use the masquerading stream/guard API.
  return at::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.device().index()).stream();
}

void check(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, "madnn HIP kernel ", what, " failed: ", hipGetErrorString(e));
}

void check_dev(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "madnn: ", name, " must be a HIP device tensor");
}

// A tensor whose storage is one dense block (any stride permutation, e.g.
// channels_last) can be packed as raw memory in its physical order.
void check_dense(const at::Tensor& t) {
  TORCH_CHECK(t.is_non_overlapping_and_dense(), "madnn bucket op: tensor must be non-overlapping and dense");
}

void bucket_copy(bool pack, at::TensorList tensors, const at::Tensor& flat, at::IntArrayRef offsets, double scale) {
  check_dev(flat, "flat");
  TORCH_CHECK(flat.is_contiguous(), "flat bucket must be contiguous");
  TORCH_CHECK(tensors.size() == offsets.size(), "tensors/offsets length mismatch");
  if (tensors.empty()) return;
  at::hip::HIPGuardMasqueradingAsCUDA guard(flat.device());
  const int tdt = dt_code(tensors[0]);
  std::vector<void*> ptrs;
  std::vector<int64_t> numels, offs;
  ptrs.reserve(tensors.size());
  for (size_t i = 0; i < tensors.size(); ++i) {
    const auto& t = tensors[i];
    check_dev(t, "bucket tensor");
    check_dense(t);
    TORCH_CHECK(dt_code(t) == tdt, "bucket tensors must share one dtype");
    TORCH_CHECK(offsets[i] >= 0 && offsets[i] + t.numel() <= flat.numel(), "bucket offset out of range");
    ptrs.push_back(t.data_ptr());
    numels.push_back(t.numel());
    offs.push_back(offsets[i]);
  }
  auto fn = pack ? madnn_bucket_pack : madnn_bucket_unpack;
  check(fn(ptrs.data(), offs.data(), numels.data(), (int)ptrs.size(), flat.data_ptr(), tdt, dt_code(flat),
           (float)scale, cur_stream(flat)),
        pack ? "bucket_pack" : "bucket_unpack");
}

void bucket_pack(at::TensorList srcs, at::Tensor flat, at::IntArrayRef offsets, double scale) {
  bucket_copy(true, srcs, flat, offsets, scale);
}

void bucket_unpack(at::TensorList dsts, at::Tensor flat, at::IntArrayRef offsets, double scale) {
  bucket_copy(false, dsts, flat, offsets, scale);
}

void flat_scale_cast(const at::Tensor& src, at::Tensor dst, double scale) {
  check_dev(src, "src");
  check_dev(dst, "dst");
  TORCH_CHECK(src.is_contiguous() && dst.is_contiguous(), "flat_scale_cast needs contiguous tensors");
  TORCH_CHECK(src.numel() == dst.numel(), "flat_scale_cast size mismatch");
  at::hip::HIPGuardMasqueradingAsCUDA guard(src.device());
  check(madnn_flat_scale_cast(src.data_ptr(), dst.data_ptr(), src.numel(), dt_code(src), dt_code(dst), (float)scale,
                              cur_stream(src)),
        "flat_scale_cast");
}

const float* opt_scale(const c10::optional<at::Tensor>& s) {
  if (!s.has_value()) return nullptr;
  TORCH_CHECK(s->scalar_type() == at::kFloat && s->is_cuda(), "device scale must be a float HIP tensor");
  return s->data_ptr<float>();
}

void sgd_step(at::Tensor master, const at::Tensor& grad, const c10::optional<at::Tensor>& mom,
              const c10::optional<at::Tensor>& model, double lr, double momentum, double dampening,
              double weight_decay, bool nesterov, bool first_step, double grad_scale,
              const c10::optional<at::Tensor>& dscale) {
  check_dev(master, "master");
  TORCH_CHECK(master.scalar_type() == at::kFloat && master.is_contiguous(), "master must be contiguous fp32");
  TORCH_CHECK(grad.is_contiguous() && grad.numel() == master.numel(), "grad must be contiguous and match master");
  if (momentum != 0.0) TORCH_CHECK(mom.has_value() && mom->numel() == master.numel(), "momentum buffer required");
  if (model.has_value()) TORCH_CHECK(model->is_contiguous() && model->numel() == master.numel(), "model copy size");
  at::hip::HIPGuardMasqueradingAsCUDA guard(master.device());
  check(madnn_sgd_step(master.data_ptr<float>(), grad.data_ptr(), dt_code(grad),
                       mom.has_value() ? mom->data_ptr<float>() : nullptr,
                       model.has_value() ? model->data_ptr() : nullptr, model.has_value() ? dt_code(*model) : -1,
                       master.numel(), (float)lr, (float)momentum, (float)dampening, (float)weight_decay,
                       nesterov ? 1 : 0, first_step ? 1 : 0, (float)grad_scale, opt_scale(dscale),
                       cur_stream(master)),
        "sgd_step");
}

void adam_step(at::Tensor master, const at::Tensor& grad, at::Tensor m1, at::Tensor m2,
               const c10::optional<at::Tensor>& model, double lr, double beta1, double beta2, double eps,
               double weight_decay, bool adamw, int64_t step, double grad_scale,
               const c10::optional<at::Tensor>& dscale) {
  check_dev(master, "master");
  TORCH_CHECK(master.scalar_type() == at::kFloat && master.is_contiguous(), "master must be contiguous fp32");
  TORCH_CHECK(grad.is_contiguous() && grad.numel() == master.numel(), "grad must be contiguous and match master");
  TORCH_CHECK(m1.numel() == master.numel() && m2.numel() == master.numel(), "adam state size");
  if (model.has_value()) TORCH_CHECK(model->is_contiguous() && model->numel() == master.numel(), "model copy size");
  TORCH_CHECK(step >= 1, "adam step must be >= 1");
  at::hip::HIPGuardMasqueradingAsCUDA guard(master.device());
  const double bc1 = 1.0 - std::pow(beta1, (double)step);
  const double bc2 = 1.0 - std::pow(beta2, (double)step);
  check(madnn_adam_step(master.data_ptr<float>(), grad.data_ptr(), dt_code(grad), m1.data_ptr<float>(),
                        m2.data_ptr<float>(), model.has_value() ? model->data_ptr() : nullptr,
                        model.has_value() ? dt_code(*model) : -1, master.numel(), (float)lr, (float)beta1,
                        (float)beta2, (float)eps, (float)weight_decay, adamw ? 1 : 0, (float)bc1,
                        (float)std::sqrt(bc2), (float)grad_scale, opt_scale(dscale), cur_stream(master)),
        "adam_step");
}

// Returns a 2-element fp32 device tensor [global L2 norm, clip coefficient].
at::Tensor grad_norm(at::TensorList flats, double max_norm, double scale) {
  TORCH_CHECK(!flats.empty(), "grad_norm needs at least one tensor");
  at::hip::HIPGuardMasqueradingAsCUDA guard(flats[0].device());
  std::vector<int> grids;
  int total = 0;
  for (const auto& f : flats) {
    check_dev(f, "grad");
    TORCH_CHECK(f.is_contiguous(), "grad_norm inputs must be contiguous");
    grids.push_back(madnn_sqnorm_grid(f.numel()));
    total += grids.back();
  }
  auto opts = flats[0].options().dtype(at::kFloat);
  at::Tensor partial = at::empty({std::max(total, 1)}, opts);
  at::Tensor out = at::empty({2}, opts);
  hipStream_t s = cur_stream(flats[0]);
  int off = 0;
  for (size_t i = 0; i < flats.size(); ++i) {
    check(madnn_sqnorm_partial(flats[i].data_ptr(), dt_code(flats[i]), flats[i].numel(), (float)scale,
                               partial.data_ptr<float>() + off, grids[i], s),
          "sqnorm_partial");
    off += grids[i];
  }
  if (total == 0) partial.zero_();
  check(madnn_norm_finalize(partial.data_ptr<float>(), std::max(total, 1), (float)max_norm, out.data_ptr<float>(), s),
        "norm_finalize");
  return out;
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> norm_fwd(const at::Tensor& x,
                                                                    const c10::optional<at::Tensor>& res,
                                                                    const at::Tensor& w,
                                                                    const c10::optional<at::Tensor>& b, double eps,
                                                                    bool rms) {
  check_dev(x, "x");
  TORCH_CHECK(x.is_contiguous(), "norm input must be contiguous");
  const int64_t H = w.numel();
  TORCH_CHECK(x.size(-1) == H && w.is_contiguous(), "norm weight / hidden size mismatch");
  TORCH_CHECK(H % 8 == 0 && H <= 16384, "madnn norm kernel needs H % 8 == 0 and H <= 16384, got ", H);
  const int64_t rows = x.numel() / H;
  at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  at::Tensor y = at::empty_like(x);
  at::Tensor sum;
  if (res.has_value()) {
    TORCH_CHECK(res->sizes() == x.sizes() && res->is_contiguous() && res->scalar_type() == x.scalar_type(),
                "residual must match x");
    sum = at::empty_like(x);
  }
  auto fopts = x.options().dtype(at::kFloat);
  at::Tensor mean = rms ? at::empty({0}, fopts) : at::empty({rows}, fopts);
  at::Tensor rstd = at::empty({rows}, fopts);
  if (b.has_value()) TORCH_CHECK(b->numel() == H && b->scalar_type() == w.scalar_type(), "norm bias mismatch");
  check(madnn_norm_fwd(x.data_ptr(), res.has_value() ? res->data_ptr() : nullptr, w.data_ptr(),
                       b.has_value() ? b->data_ptr() : nullptr, y.data_ptr(), sum.defined() ? sum.data_ptr() : nullptr,
                       rms ? nullptr : mean.data_ptr<float>(), rstd.data_ptr<float>(), rows, (int)H, (float)eps,
                       rms ? 1 : 0, dt_code(x), dt_code(w), cur_stream(x)),
        "norm_fwd");
  if (!sum.defined()) sum = at::empty({0}, x.options());
  return {y, sum, mean, rstd};
}

// colsum: also the column sums of dx over the rows (the producing Linear's bias gradient), in bf16
// when colsum_bf16 (the Linear's bias dtype) else fp32
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> norm_bwd(const at::Tensor& dy, const at::Tensor& x,
                                                                    const at::Tensor& w, const at::Tensor& mean,
                                                                    const at::Tensor& rstd,
                                                                    const c10::optional<at::Tensor>& dres, bool rms,
                                                                    bool has_bias, bool colsum, bool colsum_bf16) {
  check_dev(x, "x");
  const int64_t H = w.numel();
  const int64_t rows = x.numel() / H;
  TORCH_CHECK(dy.is_contiguous() && x.is_contiguous() && dy.sizes() == x.sizes(), "norm_bwd: dy/x mismatch");
  at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  at::Tensor dyc = dy.scalar_type() == x.scalar_type() ? dy : dy.to(x.scalar_type());
  at::Tensor dx = at::empty_like(x);
  at::Tensor dw = at::empty_like(w);
  at::Tensor db = has_bias ? at::empty_like(w) : at::empty({0}, w.options());
  at::Tensor ws = at::empty({madnn_norm_bwd_workspace(rows, (int)H)}, x.options().dtype(at::kFloat));
  at::Tensor dr;
  if (dres.has_value() && dres->defined()) {
    dr = dres->scalar_type() == x.scalar_type() ? dres->contiguous() : dres->to(x.scalar_type()).contiguous();
  }
  const auto cdt = colsum_bf16 ? at::kBFloat16 : at::kFloat;
  at::Tensor cs = colsum ? at::empty({H}, x.options().dtype(cdt)) : at::empty({0}, x.options().dtype(cdt));
  check(madnn_norm_bwd(dyc.data_ptr(), x.data_ptr(), w.data_ptr(), rms ? nullptr : mean.data_ptr<float>(),
                       rstd.data_ptr<float>(), dr.defined() ? dr.data_ptr() : nullptr, dx.data_ptr(), dw.data_ptr(),
                       has_bias ? db.data_ptr() : nullptr, colsum ? cs.data_ptr() : nullptr, colsum_bf16 ? 1 : 0,
                       ws.data_ptr<float>(), rows, (int)H, rms ? 1 : 0, dt_code(x), dt_code(w), cur_stream(x)),
        "norm_bwd");
  return {dx, dw, db, cs};
}

// ---- K5 fused BatchNorm(+add)(+ReLU), NHWC -------------------------------
// x viewed as a dense [M, C] matrix: 2-D [N, C] contiguous or 4-D channels_last.
int64_t bn_rows(const at::Tensor& x, int64_t C) {
  if (x.dim() == 2) {
    TORCH_CHECK(x.is_contiguous(), "bn: 2-D input must be contiguous");
  } else {
    TORCH_CHECK(x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast),
                "bn: 4-D input must be channels_last");
  }
  TORCH_CHECK(x.size(1) == C, "bn: channel mismatch");
  return x.numel() / C;
}

const float* optf(const c10::optional<at::Tensor>& t) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous(), "bn: affine/stat tensors must be fp32");
  return t->data_ptr<float>();
}

float* optf_mut(const c10::optional<at::Tensor>& t) { return const_cast<float*>(optf(t)); }

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor> bn_fwd(
    const at::Tensor& x, const c10::optional<at::Tensor>& res, const c10::optional<at::Tensor>& w,
    const c10::optional<at::Tensor>& b, const c10::optional<at::Tensor>& run_mean,
    const c10::optional<at::Tensor>& run_var, const c10::optional<at::Tensor>& nbt, bool training, double momentum,
    double eps, bool relu, const c10::optional<at::Tensor>& partial) {
  check_dev(x, "x");
  const int64_t C = x.size(1);
  TORCH_CHECK(madnn_bn_supported((int)C), "bn kernel needs C % 8 == 0 and C <= 2048, got ", C);
  const int64_t M = bn_rows(x, C);
  at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  at::Tensor y = at::empty_like(x);
  if (res.has_value()) TORCH_CHECK(res->sizes() == x.sizes() && res->strides() == x.strides(), "bn residual layout");
  if (!training) TORCH_CHECK(run_mean.has_value() && run_var.has_value(), "bn eval needs running stats");
  auto fo = x.options().dtype(at::kFloat);
  at::Tensor save_mean = at::empty({C}, fo), save_invstd = at::empty({C}, fo);
  at::Tensor scale = at::empty({C}, fo), shift = at::empty({C}, fo);
  // statistics produced upstream (K9 conv epilogue): [rows, 2, C] partial sums
  const bool ext = training && partial.has_value() && partial->defined() && partial->numel() > 0;
  if (ext) {
    TORCH_CHECK(partial->scalar_type() == at::kFloat && partial->is_contiguous() && partial->dim() == 3 &&
                    partial->size(1) == 2 && partial->size(2) == C,
                "bn: partial statistics must be fp32 [rows, 2, C]");
  }
  at::Tensor ws = at::empty({training && !ext ? (int64_t)madnn_bn_partial_rows(M, (int)C) * 2 * C
                                              : (int64_t)madnn_bn_prereduce_floats((int)C)},
                            fo);
  // training with a fused residual + ReLU: 1-bit ReLU mask for the backward passes
  const bool need_mask = training && relu && res.has_value();
  at::Tensor mask = at::empty({need_mask ? x.numel() / 8 : 0}, x.options().dtype(at::kByte));
  int64_t* nb = nullptr;
  if (nbt.has_value() && nbt->defined()) {
    TORCH_CHECK(nbt->scalar_type() == at::kLong && nbt->is_cuda(), "num_batches_tracked must be an int64 device tensor");
    nb = nbt->data_ptr<int64_t>();
  }
  check(madnn_bn_fwd(x.data_ptr(), res.has_value() ? res->data_ptr() : nullptr, y.data_ptr(),
                     need_mask ? mask.data_ptr<uint8_t>() : nullptr, M, (int)C, dt_code(x),
                     relu ? 1 : 0, training ? 1 : 0, (float)eps, (float)momentum, optf(w), optf(b),
                     training ? optf_mut(run_mean) : const_cast<float*>(optf(run_mean)), optf_mut(run_var),
                     training ? nb : nullptr, save_mean.data_ptr<float>(), save_invstd.data_ptr<float>(),
                     scale.data_ptr<float>(), shift.data_ptr<float>(), ws.data_ptr<float>(),
                     ext ? partial->data_ptr<float>() : nullptr, ext ? (int)partial->size(0) : 0, cur_stream(x)),
        "bn_fwd");
  return {y, save_mean, save_invstd, scale, shift, mask};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> bn_bwd(
    const at::Tensor& dy, const at::Tensor& x, const c10::optional<at::Tensor>& mask, bool has_res,
    const c10::optional<at::Tensor>& w, const at::Tensor& save_mean, const at::Tensor& save_invstd,
    const at::Tensor& scale, const at::Tensor& shift, bool relu, bool need_wgrad, bool write_dres) {
  check_dev(x, "x");
  const int64_t C = x.size(1);
  const int64_t M = bn_rows(x, C);
  at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  at::Tensor dyc = dy;
  if (dy.strides() != x.strides() || dy.scalar_type() != x.scalar_type()) {
    dyc = at::empty_like(x);
    dyc.copy_(dy);
  }
  at::Tensor dx = at::empty_like(x);
  // !write_dres (ReLU + residual only): the residual's gradient (dy masked by the ReLU) is left to
  // the consumer, which reads dy and the bit mask itself (conv1x1_dgrad resmask)
  TORCH_CHECK(write_dres || (relu && has_res), "bn_bwd: write_dres=False needs ReLU + residual");
  at::Tensor dres = has_res && write_dres ? at::empty_like(x) : at::Tensor();
  const uint8_t* mk = nullptr;
  if (relu && has_res) {
    TORCH_CHECK(mask.has_value() && mask->numel() == x.numel() / 8, "bn_bwd: ReLU bit mask required");
    mk = mask->data_ptr<uint8_t>();
  }
  auto fo = x.options().dtype(at::kFloat);
  at::Tensor dw = at::empty({C}, fo), db = at::empty({C}, fo);
  at::Tensor coef = at::empty({3 * C}, fo);
  at::Tensor ws = at::empty({(int64_t)madnn_bn_partial_rows(M, (int)C) * 2 * C}, fo);
  check(madnn_bn_bwd(dyc.data_ptr(), x.data_ptr(), mk, has_res ? 1 : 0, dx.data_ptr(),
                     dres.defined() ? dres.data_ptr() : nullptr, M, (int)C, dt_code(x), relu ? 1 : 0, optf(w),
                     save_mean.data_ptr<float>(), save_invstd.data_ptr<float>(), scale.data_ptr<float>(),
                     shift.data_ptr<float>(), need_wgrad ? dw.data_ptr<float>() : nullptr,
                     need_wgrad ? db.data_ptr<float>() : nullptr, coef.data_ptr<float>(), ws.data_ptr<float>(),
                     cur_stream(x)),
        "bn_bwd");
  if (!dres.defined()) dres = at::empty({0}, x.options());
  return {dx, dw, db, dres};
}

// relu(BN(x) + BN_r(r)) in training (ResNet's bn3 with the downsample BatchNorm folded in).
// Returns y, the ReLU bit mask and (mean, invstd, scale, shift) of each BN: 10 tensors.
std::vector<at::Tensor> bn_fwd_dual(const at::Tensor& x, const at::Tensor& r, const c10::optional<at::Tensor>& w,
                                    const c10::optional<at::Tensor>& b, const c10::optional<at::Tensor>& run_mean,
                                    const c10::optional<at::Tensor>& run_var, const c10::optional<at::Tensor>& nbt,
                                    double momentum, double eps, const c10::optional<at::Tensor>& partial,
                                    const c10::optional<at::Tensor>& w_r, const c10::optional<at::Tensor>& b_r,
                                    const c10::optional<at::Tensor>& run_mean_r,
                                    const c10::optional<at::Tensor>& run_var_r,
                                    const c10::optional<at::Tensor>& nbt_r, double momentum_r, double eps_r,
                                    const c10::optional<at::Tensor>& partial_r) {
  check_dev(x, "x");
  check_dev(r, "r");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && r.scalar_type() == at::kBFloat16, "bn_fwd_dual: bf16 only");
  const int64_t C = x.size(1);
  TORCH_CHECK(madnn_bn_supported((int)C), "bn kernel needs C % 8 == 0 and C <= 2048, got ", C);
  const int64_t M = bn_rows(x, C);
  TORCH_CHECK(r.sizes() == x.sizes() && r.strides() == x.strides(), "bn_fwd_dual: residual layout");
  at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  auto fo = x.options().dtype(at::kFloat);
  auto ext = [&](const c10::optional<at::Tensor>& p) -> const float* {
    if (!p.has_value() || !p->defined() || p->numel() == 0) return nullptr;
    TORCH_CHECK(p->scalar_type() == at::kFloat && p->is_contiguous() && p->dim() == 3 && p->size(1) == 2 &&
                    p->size(2) == C,
                "bn: partial statistics must be fp32 [rows, 2, C]");
    return p->data_ptr<float>();
  };
  auto nbp = [](const c10::optional<at::Tensor>& t) -> int64_t* {
    if (!t.has_value() || !t->defined()) return nullptr;
    TORCH_CHECK(t->scalar_type() == at::kLong && t->is_cuda(), "num_batches_tracked must be an int64 device tensor");
    return t->data_ptr<int64_t>();
  };
  std::vector<at::Tensor> out;
  out.push_back(at::empty_like(x));
  out.push_back(at::empty({x.numel() / 8}, x.options().dtype(at::kByte)));
  for (int k = 0; k < 8; ++k) out.push_back(at::empty({C}, fo));
  at::Tensor ws = at::empty({std::max<int64_t>((int64_t)madnn_bn_partial_rows(M, (int)C) * 2 * C,
                                               (int64_t)madnn_bn_prereduce_floats((int)C))},
                            fo);
  const float* pe = ext(partial);
  const float* pr = ext(partial_r);
  check(madnn_bn_fwd_dual(x.data_ptr(), r.data_ptr(), out[0].data_ptr(), out[1].data_ptr<uint8_t>(), M, (int)C,
                          (float)eps, (float)momentum, optf(w), optf(b), optf_mut(run_mean), optf_mut(run_var),
                          nbp(nbt), out[2].data_ptr<float>(), out[3].data_ptr<float>(), out[4].data_ptr<float>(),
                          out[5].data_ptr<float>(), pe, pe ? (int)partial->size(0) : 0, (float)eps_r,
                          (float)momentum_r, optf(w_r), optf(b_r), optf_mut(run_mean_r), optf_mut(run_var_r),
                          nbp(nbt_r), out[6].data_ptr<float>(), out[7].data_ptr<float>(), out[8].data_ptr<float>(),
                          out[9].data_ptr<float>(), pr, pr ? (int)partial_r->size(0) : 0, ws.data_ptr<float>(),
                          cur_stream(x)),
        "bn_fwd_dual");
  return out;
}

// -> dx, dr, dw, db, dw_r, db_r
std::vector<at::Tensor> bn_bwd_dual(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& r,
                                    const at::Tensor& mask, const c10::optional<at::Tensor>& w,
                                    const at::Tensor& save_mean, const at::Tensor& save_invstd,
                                    const c10::optional<at::Tensor>& w_r, const at::Tensor& save_mean_r,
                                    const at::Tensor& save_invstd_r) {
  check_dev(x, "x");
  const int64_t C = x.size(1);
  const int64_t M = bn_rows(x, C);
  TORCH_CHECK(r.sizes() == x.sizes() && r.strides() == x.strides() && r.scalar_type() == x.scalar_type(),
              "bn_bwd_dual: residual layout");
  TORCH_CHECK(mask.numel() == x.numel() / 8, "bn_bwd_dual: ReLU bit mask required");
  at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  at::Tensor dyc = dy;
  if (dy.strides() != x.strides() || dy.scalar_type() != x.scalar_type()) {
    dyc = at::empty_like(x);
    dyc.copy_(dy);
  }
  auto fo = x.options().dtype(at::kFloat);
  std::vector<at::Tensor> out{at::empty_like(x), at::empty_like(x), at::empty({C}, fo), at::empty({C}, fo),
                              at::empty({C}, fo), at::empty({C}, fo)};
  at::Tensor coef = at::empty({6 * C}, fo);
  at::Tensor ws = at::empty({(int64_t)madnn_bn_partial_rows(M, (int)C) * 3 * C}, fo);
  check(madnn_bn_bwd_dual(dyc.data_ptr(), x.data_ptr(), r.data_ptr(), mask.data_ptr<uint8_t>(), out[0].data_ptr(),
                          out[1].data_ptr(), M, (int)C, optf(w), save_mean.data_ptr<float>(),
                          save_invstd.data_ptr<float>(), optf(w_r), save_mean_r.data_ptr<float>(),
                          save_invstd_r.data_ptr<float>(), out[2].data_ptr<float>(), out[3].data_ptr<float>(),
                          out[4].data_ptr<float>(), out[5].data_ptr<float>(), coef.data_ptr<float>(),
                          ws.data_ptr<float>(), cur_stream(x)),
        "bn_bwd_dual");
  return out;
}

// Training BatchNorm coefficients only (statistics pass unless `partial` is given, finalize with
// the running-stat update): -> mean, invstd, scale, shift.  The apply is left to a consumer
// kernel (K9's BatchNorm prologue).
std::vector<at::Tensor> bn_coef(const at::Tensor& x, const c10::optional<at::Tensor>& w,
                                const c10::optional<at::Tensor>& b, const c10::optional<at::Tensor>& run_mean,
                                const c10::optional<at::Tensor>& run_var, const c10::optional<at::Tensor>& nbt,
                                double momentum, double eps, const c10::optional<at::Tensor>& partial) {
  check_dev(x, "x");
  const int64_t C = x.size(1);
  TORCH_CHECK(madnn_bn_supported((int)C), "bn kernel needs C % 8 == 0 and C <= 2048, got ", C);
  const int64_t M = bn_rows(x, C);
  TORCH_CHECK(x.scalar_type() == at::kBFloat16, "bn_coef: bf16 only");
  at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  auto fo = x.options().dtype(at::kFloat);
  std::vector<at::Tensor> out;
  for (int k = 0; k < 4; ++k) out.push_back(at::empty({C}, fo));
  const bool ext = partial.has_value() && partial->defined() && partial->numel() > 0;
  if (ext) {
    TORCH_CHECK(partial->scalar_type() == at::kFloat && partial->is_contiguous() && partial->dim() == 3 &&
                    partial->size(1) == 2 && partial->size(2) == C,
                "bn: partial statistics must be fp32 [rows, 2, C]");
  }
  at::Tensor ws = at::empty({ext ? (int64_t)madnn_bn_prereduce_floats((int)C)
                                : (int64_t)madnn_bn_partial_rows(M, (int)C) * 2 * C},
                            fo);
  int64_t* nb = nullptr;
  if (nbt.has_value() && nbt->defined()) {
    TORCH_CHECK(nbt->scalar_type() == at::kLong && nbt->is_cuda(), "num_batches_tracked must be an int64 device tensor");
    nb = nbt->data_ptr<int64_t>();
  }
  check(madnn_bn_coef(x.data_ptr(), M, (int)C, (float)eps, (float)momentum, optf(w), optf(b), optf_mut(run_mean),
                      optf_mut(run_var), nb, out[0].data_ptr<float>(), out[1].data_ptr<float>(),
                      out[2].data_ptr<float>(), out[3].data_ptr<float>(), ws.data_ptr<float>(),
                      ext ? partial->data_ptr<float>() : nullptr, ext ? (int)partial->size(0) : 0, cur_stream(x)),
        "bn_coef");
  return out;
}

bool bn_supported(int64_t C) { return madnn_bn_supported((int)C) != 0; }

// ---- K9 NHWC 1x1 convolution (stride 1) on MFMA --------------------------------
// Activations: 4-D channels_last [N, C, H, W] or 2-D contiguous [M, C], bf16.
// Weight: [Cout, Cin] or [Cout, Cin, 1, 1] with contiguous rows (either memory format).
int64_t conv_rows(const at::Tensor& t, int64_t C, const char* name) {
  check_dev(t, name);
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, "conv1x1: ", name, " must be bf16");
  if (t.dim() == 2) {
    TORCH_CHECK(t.is_contiguous(), "conv1x1: 2-D ", name, " must be contiguous");
  } else {
    TORCH_CHECK(t.dim() == 4 && t.is_contiguous(at::MemoryFormat::ChannelsLast), "conv1x1: 4-D ", name,
                " must be channels_last");
  }
  TORCH_CHECK(t.size(1) == C, "conv1x1: ", name, " channel mismatch");
  return t.numel() / C;
}

at::Tensor conv_out_like(const at::Tensor& t, int64_t C) {
  if (t.dim() == 2) return at::empty({t.size(0), C}, t.options());
  return at::empty({t.size(0), C, t.size(2), t.size(3)}, t.options().memory_format(at::MemoryFormat::ChannelsLast));
}

void conv_check_w(const at::Tensor& w, int64_t cout, int64_t cin) {
  check_dev(w, "w");
  TORCH_CHECK(w.scalar_type() == at::kBFloat16, "conv1x1: weight must be bf16");
  TORCH_CHECK(w.size(0) == cout && w.numel() == cout * cin, "conv1x1: weight must be [Cout, Cin(, 1, 1)]");
  TORCH_CHECK(w.stride(0) == cin && w.stride(1) == 1, "conv1x1: weight rows must be contiguous");
  TORCH_CHECK(madnn_conv1x1_supported(cin, cout), "conv1x1: channels must be multiples of 64, got ", cin, " -> ",
              cout);
}

// y = conv(x, w); with stats: partial [rows, 2, Cout] per-channel (sum, sum of squares) of y
std::tuple<at::Tensor, at::Tensor> conv1x1_fwd(const at::Tensor& x, const at::Tensor& w, bool stats) {
  const int64_t cin = x.size(1), cout = w.size(0);
  const int64_t M = conv_rows(x, cin, "x");
  conv_check_w(w, cout, cin);
  at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  at::Tensor y = conv_out_like(x, cout);
  const int64_t rows = stats ? madnn_conv1x1_stat_rows(M, cin, cout) : 0;
  at::Tensor part = at::empty({rows, 2, cout}, x.options().dtype(at::kFloat));
  check(madnn_conv1x1_fwd(x.data_ptr(), w.data_ptr(), y.data_ptr(), stats ? part.data_ptr<float>() : nullptr, M, cin,
                          cout, cur_stream(x)),
        "conv1x1_fwd");
  return {y, part};
}

// dx = dy (*) w^T, plus `res` (a gradient of x's layout accumulated from another path) if given;
// resmask: a ReLU bit mask over res's elements (8 per byte) -- res counts only where it is set
at::Tensor conv1x1_dgrad(const at::Tensor& dy, const at::Tensor& w, const c10::optional<at::Tensor>& res,
                         const c10::optional<at::Tensor>& resmask) {
  const int64_t cout = dy.size(1), cin = w.numel() / std::max<int64_t>(cout, 1);
  const int64_t M = conv_rows(dy, cout, "dy");
  conv_check_w(w, cout, cin);
  at::hip::HIPGuardMasqueradingAsCUDA guard(dy.device());
  at::Tensor dx = conv_out_like(dy, cin);
  const bool has_res = res.has_value() && res->defined();
  if (has_res) {
    TORCH_CHECK(conv_rows(*res, cin, "res") == M && res->dim() == dy.dim(), "conv1x1_dgrad: residual layout");
  }
  const bool has_mask = resmask.has_value() && resmask->defined();
  if (has_mask) {
    TORCH_CHECK(has_res && resmask->scalar_type() == at::kByte && resmask->is_contiguous() &&
                    resmask->numel() == M * cin / 8, "conv1x1_dgrad: resmask must be a uint8 bit mask over res");
  }
  check(madnn_conv1x1_dgrad(dy.data_ptr(), w.data_ptr(), dx.data_ptr(), has_res ? res->data_ptr() : nullptr, M, cin,
                            cout, nullptr, nullptr, nullptr, nullptr, cur_stream(dy),
                            has_mask ? resmask->data_ptr<uint8_t>() : nullptr),
        "conv1x1_dgrad");
  return dx;
}

// dx = dy (*) w^T where dx is d relu(bn(bny)), plus bn's backward sums (sum g, sum g*bny) from the
// epilogue: -> (dx, partial [rows, 2, Cin])
std::tuple<at::Tensor, at::Tensor> conv1x1_dgrad_bnb(const at::Tensor& dy, const at::Tensor& w, const at::Tensor& bny,
                                                     const at::Tensor& scale, const at::Tensor& shift) {
  const int64_t cout = dy.size(1), cin = w.numel() / std::max<int64_t>(cout, 1);
  const int64_t M = conv_rows(dy, cout, "dy");
  conv_check_w(w, cout, cin);
  TORCH_CHECK(conv_rows(bny, cin, "bny") == M && bny.dim() == dy.dim(), "conv1x1_dgrad_bnb: bny layout");
  TORCH_CHECK(scale.numel() == cin && shift.numel() == cin && scale.scalar_type() == at::kFloat &&
                  shift.scalar_type() == at::kFloat && scale.is_contiguous() && shift.is_contiguous(),
              "conv1x1_dgrad_bnb: fp32 [Cin] scale / shift");
  at::hip::HIPGuardMasqueradingAsCUDA guard(dy.device());
  at::Tensor dx = conv_out_like(dy, cin);
  at::Tensor part = at::empty({madnn_conv1x1_dgrad_rows(M, cin, cout), 2, cin}, dy.options().dtype(at::kFloat));
  check(madnn_conv1x1_dgrad(dy.data_ptr(), w.data_ptr(), dx.data_ptr(), nullptr, M, cin, cout, bny.data_ptr(),
                            scale.data_ptr<float>(), shift.data_ptr<float>(), part.data_ptr<float>(), cur_stream(dy)),
        "conv1x1_dgrad_bnb");
  return {dx, part};
}

// [Cout, Cin] weight gradient, fp32 (or bf16 with out_bf16: the split reduction casts)
at::Tensor conv1x1_wgrad(const at::Tensor& dy, const at::Tensor& x, bool out_bf16) {
  const int64_t cout = dy.size(1), cin = x.size(1);
  const int64_t M = conv_rows(x, cin, "x");
  TORCH_CHECK(conv_rows(dy, cout, "dy") == M && dy.dim() == x.dim(), "conv1x1_wgrad: dy / x pixel mismatch");
  TORCH_CHECK(madnn_conv1x1_supported(cin, cout), "conv1x1: channels must be multiples of 64");
  at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  at::Tensor dw = at::empty({cout, cin}, x.options().dtype(out_bf16 ? at::kBFloat16 : at::kFloat));
  at::Tensor ws = at::empty({madnn_conv1x1_wgrad_ws(M, cin, cout)}, x.options().dtype(at::kFloat));
  check(madnn_conv1x1_wgrad(dy.data_ptr(), x.data_ptr(), dw.data_ptr(), out_bf16 ? 1 : 0, ws.data_ptr<float>(), M, cin,
                            cout, cur_stream(x)),
        "conv1x1_wgrad");
  return dw;
}

// ---- K12 MFMA GEMM (Linear layers) ------------------------------------------------------------
// x: [..., K] bf16 with contiguous rows, w: [N, K] bf16 contiguous.
void gemm_check(const at::Tensor& t, const char* name) {
  check_dev(t, name);
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, "linear: ", name, " must be bf16");
  TORCH_CHECK(t.is_contiguous(), "linear: ", name, " must be contiguous");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, "linear: ", name, " must be 16-B aligned");
}

// y = x w^T (+ bias) (-> GELU: act 1 tanh / 2 erf) (+ res); with save_aux the pre-activation is returned too
std::tuple<at::Tensor, at::Tensor> linear_fwd(const at::Tensor& x, const at::Tensor& w,
                                              const c10::optional<at::Tensor>& bias,
                                              const c10::optional<at::Tensor>& res, int64_t act, bool save_aux) {
  gemm_check(x, "x");
  gemm_check(w, "w");
  const int64_t K = x.size(-1), N = w.size(0), M = x.numel() / std::max<int64_t>(K, 1);
  TORCH_CHECK(w.dim() == 2 && w.size(1) == K, "linear: weight must be [N, K]");
  TORCH_CHECK(madnn_gemm_supported(N, M, K, K, K), "linear: unsupported shape M=", M, " N=", N, " K=", K);
  at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  std::vector<int64_t> shape(x.sizes().begin(), x.sizes().end());
  shape.back() = N;
  at::Tensor y = at::empty(shape, x.options());
  at::Tensor aux = save_aux ? at::empty(shape, x.options()) : at::empty({0}, x.options());
  const bool hb = bias.has_value() && bias->defined();
  if (hb) {
    check_dev(*bias, "bias");
    TORCH_CHECK(bias->numel() == N && bias->is_contiguous() &&
                    (bias->scalar_type() == at::kFloat || bias->scalar_type() == at::kBFloat16),
                "linear: bias must be a contiguous fp32/bf16 [N]");
  }
  const bool hr = res.has_value() && res->defined();
  if (hr) {
    gemm_check(*res, "res");
    TORCH_CHECK(res->numel() == M * N && res->size(-1) == N, "linear: residual shape");
  }
  check(madnn_linear_fwd(x.data_ptr(), w.data_ptr(), hb ? bias->data_ptr() : nullptr,
                         hb && bias->scalar_type() == at::kFloat ? 1 : 0, hr ? res->data_ptr() : nullptr, y.data_ptr(),
                         save_aux ? aux.data_ptr() : nullptr, (int)act, M, N, K, cur_stream(x)),
        "linear_fwd");
  return {y, aux};
}

// dx = dy w (+ res).  With accumulate, res itself receives the result (in-place beta = 1).
at::Tensor linear_dgrad(const at::Tensor& dy, const at::Tensor& w, const c10::optional<at::Tensor>& res,
                        bool accumulate) {
  gemm_check(dy, "dy");
  gemm_check(w, "w");
  const int64_t N = dy.size(-1), K = w.size(1), M = dy.numel() / std::max<int64_t>(N, 1);
  TORCH_CHECK(w.dim() == 2 && w.size(0) == N, "linear_dgrad: weight must be [N, K]");
  TORCH_CHECK(madnn_gemm_supported(K, M, N, K, N), "linear_dgrad: unsupported shape M=", M, " N=", N, " K=", K);
  at::hip::HIPGuardMasqueradingAsCUDA guard(dy.device());
  const bool hr = res.has_value() && res->defined();
  if (hr) {
    gemm_check(*res, "res");
    TORCH_CHECK(res->numel() == M * K && res->size(-1) == K, "linear_dgrad: residual shape");
  }
  at::Tensor dx;
  if (hr && accumulate) {
    dx = *res;
  } else {
    std::vector<int64_t> shape(dy.sizes().begin(), dy.sizes().end());
    shape.back() = K;
    dx = at::empty(shape, dy.options());
  }
  check(madnn_linear_dgrad(dy.data_ptr(), w.data_ptr(), hr ? res->data_ptr() : nullptr, dx.data_ptr(), M, N, K,
                           cur_stream(dy)),
        "linear_dgrad");
  return dx;
}

// dW[N, K] = dy[M, N]^T x[M, K] over the M tokens, split along M (fp32 slabs + reduce) so the few
// output tiles of a weight gradient fill the GPU.  With `out` the result is written there (the
// reducer's bucket slot: a grad sink), with accumulate added to its contents.  splits <= 0: auto.
at::Tensor linear_wgrad_impl(const at::Tensor& dy, const at::Tensor& x, const c10::optional<at::Tensor>& out,
                             bool accumulate, int64_t splits, int kind) {
  gemm_check(dy, "dy");
  gemm_check(x, "x");
  const int64_t N = dy.size(-1), K = x.size(-1), M = dy.numel() / std::max<int64_t>(N, 1);
  TORCH_CHECK(x.numel() == M * K, "linear_wgrad: dy / x token mismatch");
  TORCH_CHECK(M % 64 == 0 && madnn_gemm_supported(K, N, M, K, N), "linear_wgrad: unsupported shape M=", M, " N=", N,
              " K=", K);
  at::hip::HIPGuardMasqueradingAsCUDA guard(dy.device());
  at::Tensor dw;
  if (out.has_value() && out->defined()) {
    gemm_check(*out, "out");
    TORCH_CHECK(out->numel() == N * K, "linear_wgrad: out must hold N x K");
    dw = *out;
  } else {
    TORCH_CHECK(!accumulate, "linear_wgrad: accumulate needs out");
    dw = at::empty({N, K}, dy.options());
  }
  const int sp = splits > 0 ? (int)splits : madnn_wgrad_splits(M, N, K);
  at::Tensor ws = sp > 1 ? at::empty({sp, N, K}, dy.options().dtype(at::kFloat)) : at::Tensor();
  if (kind == 2) TORCH_CHECK(M % 128 == 0, "linear_wgrad4h: tokens must be a multiple of 128");
  auto fn = kind == 2 ? madnn_linear_wgrad4h : kind == 1 ? madnn_linear_wgrad4 : madnn_linear_wgrad;
  check(fn(dy.data_ptr(), x.data_ptr(), dw.data_ptr(), sp > 1 ? ws.data_ptr<float>() : nullptr, sp, accumulate ? 1 : 0,
           M, N, K, cur_stream(dy)),
        "linear_wgrad");
  return dw;
}

at::Tensor linear_wgrad(const at::Tensor& dy, const at::Tensor& x, const c10::optional<at::Tensor>& out,
                        bool accumulate, int64_t splits) {
  return linear_wgrad_impl(dy, x, out, accumulate, splits, 0);
}

// K12W (gemm.hip: one wave per SIMD, 128 x 128 per wave), same contract
at::Tensor linear_wgrad4(const at::Tensor& dy, const at::Tensor& x, const c10::optional<at::Tensor>& out,
                         bool accumulate, int64_t splits) {
  return linear_wgrad_impl(dy, x, out, accumulate, splits, 1);
}

// K12W16 (gemm.hip gemm4h_kernel: the v_mfma_f32_16x16x32_bf16 form), same contract, tokens % 128 == 0
at::Tensor linear_wgrad4h(const at::Tensor& dy, const at::Tensor& x, const c10::optional<at::Tensor>& out,
                          bool accumulate, int64_t splits) {
  return linear_wgrad_impl(dy, x, out, accumulate, splits, 2);
}

int64_t wgrad_splits(int64_t M, int64_t N, int64_t K) { return madnn_wgrad_splits(M, N, K); }

// ---- K12P persistent GEMMs with overlapped epilogues (gemmp.hip) ------------------------------
bool gemmp_supported(int64_t I, int64_t J, int64_t K, bool has_bias) {
  return madnn_gemmp_supported(I, J, K, has_bias ? 1 : 0) != 0;
}

// y = x w^T (+ bias); act 1: (gelu(pre), pre) with pre = x w^T + bias
std::tuple<at::Tensor, at::Tensor> linear_fwd_p(const at::Tensor& x, const at::Tensor& w,
                                                const c10::optional<at::Tensor>& bias, int64_t act) {
  gemm_check(x, "x");
  gemm_check(w, "w");
  const int64_t K = x.size(-1), N = w.size(0), M = x.numel() / std::max<int64_t>(K, 1);
  TORCH_CHECK(w.dim() == 2 && w.size(1) == K, "linear_p: weight must be [N, K]");
  const bool hb = bias.has_value() && bias->defined();
  TORCH_CHECK(madnn_gemmp_supported(N, M, K, hb ? 1 : 0), "linear_p: unsupported shape M=", M, " N=", N, " K=", K);
  if (hb) {
    check_dev(*bias, "bias");
    TORCH_CHECK(bias->numel() == N && bias->is_contiguous() &&
                    (bias->scalar_type() == at::kFloat || bias->scalar_type() == at::kBFloat16),
                "linear_p: bias must be a contiguous fp32/bf16 [N]");
  }
  at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  std::vector<int64_t> shape(x.sizes().begin(), x.sizes().end());
  shape.back() = N;
  at::Tensor y = at::empty(shape, x.options());
  TORCH_CHECK(act >= 0 && act <= 2, "linear_fwd_p: act 0 (none), 1 (tanh GELU) or 2 (erf GELU)");
  at::Tensor aux = act != 0 ? at::empty(shape, x.options()) : at::empty({0}, x.options());
  check(madnn_linear_fwd_p(x.data_ptr(), w.data_ptr(), hb ? bias->data_ptr() : nullptr,
                           hb && bias->scalar_type() == at::kFloat ? 1 : 0, y.data_ptr(),
                           act != 0 ? aux.data_ptr() : nullptr, (int)act, M, N, K, cur_stream(x)),
        "linear_fwd_p");
  return {y, aux};
}

// dx = dy w; with pre: (dx * gelu'(pre), column sums of that in bias_dtype) -- the GELU backward
// and c_fc's bias gradient fused into the data-gradient GEMM
std::tuple<at::Tensor, at::Tensor> linear_dgrad_p(const at::Tensor& dy, const at::Tensor& w,
                                                  const c10::optional<at::Tensor>& pre, at::ScalarType bias_dtype,
                                                  int64_t gelu_kind) {
  TORCH_CHECK(gelu_kind == 1 || gelu_kind == 2, "linear_dgrad_p: gelu_kind 1 (tanh) or 2 (erf)");
  gemm_check(dy, "dy");
  gemm_check(w, "w");
  const int64_t N = dy.size(-1), K = w.size(1), M = dy.numel() / std::max<int64_t>(N, 1);
  TORCH_CHECK(w.dim() == 2 && w.size(0) == N, "linear_dgrad_p: weight must be [N, K]");
  TORCH_CHECK(madnn_gemmp_supported(K, M, N, 0), "linear_dgrad_p: unsupported shape M=", M, " N=", N, " K=", K);
  const bool hp = pre.has_value() && pre->defined();
  if (hp) {
    gemm_check(*pre, "pre");
    TORCH_CHECK(pre->numel() == M * K && pre->size(-1) == K, "linear_dgrad_p: pre must be [M, K]");
    TORCH_CHECK(bias_dtype == at::kFloat || bias_dtype == at::kBFloat16, "linear_dgrad_p: fp32/bf16 bias grad");
  }
  at::hip::HIPGuardMasqueradingAsCUDA guard(dy.device());
  std::vector<int64_t> shape(dy.sizes().begin(), dy.sizes().end());
  shape.back() = K;
  at::Tensor dx = at::empty(shape, dy.options());
  at::Tensor db = hp ? at::empty({K}, dy.options().dtype(bias_dtype)) : at::empty({0}, dy.options());
  at::Tensor part;
  const int rows = (int)(M / 256 * 4);
  if (hp) part = at::empty({rows, K}, dy.options().dtype(at::kFloat));
  check(madnn_linear_dgrad_p(dy.data_ptr(), w.data_ptr(), hp ? pre->data_ptr() : nullptr, dx.data_ptr(),
                             hp ? part.data_ptr<float>() : nullptr, M, N, K, (int)gelu_kind, cur_stream(dy)),
        "linear_dgrad_p");
  if (hp)
    check(madnn_colsum_finalize(part.data_ptr<float>(), rows, K, db.data_ptr(), bias_dtype == at::kFloat ? 1 : 0,
                                cur_stream(dy)),
          "colsum_finalize");
  return {dx, db};
}

// ---- K13 NHWC 3x3 / stride 1 / pad 1 convolution on MFMA --------------------------------------
// x: [N, Ci, H, W] channels_last bf16; w: [Co, Ci, 3, 3] channels_last ([Co][3][3][Ci] in memory).
// stride 2 / pad 1 (K13 SD = 2): y [N, Co, H/2, W/2] channels_last (+ BN statistics partial rows)
std::tuple<at::Tensor, at::Tensor> conv3x3_fwd_s2(const at::Tensor& x, const at::Tensor& w, bool stats) {
  check_dev(x, "x");
  check_dev(w, "w");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16, "conv3x3_s2: bf16 only");
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast), "conv3x3_s2: x must be NHWC 4-D");
  TORCH_CHECK(w.dim() == 4 && w.size(2) == 3 && w.size(3) == 3 && w.size(1) == x.size(1) &&
                  w.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv3x3_s2: w must be a channels_last [Co, Ci, 3, 3]");
  const int N = (int)x.size(0), Ci = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3), Co = (int)w.size(0);
  TORCH_CHECK(madnn_conv3x3_s2_supported(H, W, Ci, Co), "conv3x3_s2: unsupported shape Ci=", Ci, " Co=", Co, " H=", H,
              " W=", W);
  at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  at::Tensor y = at::empty({N, Co, H / 2, W / 2}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int64_t rows = stats ? madnn_conv3x3_s2_stat_rows(N, H, W) : 0;
  at::Tensor part = at::empty({rows, 2, Co}, x.options().dtype(at::kFloat));
  check(madnn_conv3x3_fwd_s2(x.data_ptr(), w.data_ptr(), y.data_ptr(), stats ? part.data_ptr<float>() : nullptr, N,
                             H, W, Ci, Co, cur_stream(x)),
        "conv3x3_fwd_s2");
  return {y, part};
}

std::tuple<at::Tensor, at::Tensor> conv3x3_fwd(const at::Tensor& x, const at::Tensor& w, bool stats) {
  check_dev(x, "x");
  check_dev(w, "w");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16, "conv3x3: bf16 only");
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast), "conv3x3: x must be NHWC 4-D");
  TORCH_CHECK(w.dim() == 4 && w.size(2) == 3 && w.size(3) == 3 && w.size(1) == x.size(1) &&
                  w.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv3x3: w must be a channels_last [Co, Ci, 3, 3]");
  const int N = (int)x.size(0), Ci = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3), Co = (int)w.size(0);
  TORCH_CHECK(madnn_conv3x3_supported(H, W, Ci, Co), "conv3x3: unsupported shape Ci=", Ci, " Co=", Co, " W=", W);
  at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  at::Tensor y = at::empty({N, Co, H, W}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int64_t rows = stats ? madnn_conv3x3_stat_rows((int64_t)N * H * W) : 0;
  at::Tensor part = at::empty({rows, 2, Co}, x.options().dtype(at::kFloat));
  check(madnn_conv3x3_fwd(x.data_ptr(), w.data_ptr(), y.data_ptr(), stats ? part.data_ptr<float>() : nullptr, N, H,
                          W, Ci, Co, cur_stream(x)),
        "conv3x3_fwd");
  return {y, part};
}

// Data grad (x = output gradient, w = flipped / transposed weight) with the BatchNorm-backward sums of
// bny (the BN input feeding relu -> this conv) in the epilogue: -> (dx, partial [rows, 2, Co])
std::tuple<at::Tensor, at::Tensor> conv3x3_fwd_bnb(const at::Tensor& x, const at::Tensor& w, const at::Tensor& bny,
                                                   const at::Tensor& scale, const at::Tensor& shift) {
  check_dev(x, "x");
  check_dev(w, "w");
  check_dev(bny, "bny");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16 &&
                  bny.scalar_type() == at::kBFloat16,
              "conv3x3: bf16 only");
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast), "conv3x3: x must be NHWC 4-D");
  TORCH_CHECK(w.dim() == 4 && w.size(2) == 3 && w.size(3) == 3 && w.size(1) == x.size(1) &&
                  w.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv3x3: w must be a channels_last [Co, Ci, 3, 3]");
  const int N = (int)x.size(0), Ci = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3), Co = (int)w.size(0);
  TORCH_CHECK(bny.dim() == 4 && bny.size(0) == N && bny.size(1) == Co && bny.size(2) == H && bny.size(3) == W &&
                  bny.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv3x3_fwd_bnb: bny must be the NHWC [N, Co, H, W] BN input");
  TORCH_CHECK(scale.numel() == Co && shift.numel() == Co && scale.scalar_type() == at::kFloat &&
                  shift.scalar_type() == at::kFloat && scale.is_contiguous() && shift.is_contiguous(),
              "conv3x3_fwd_bnb: fp32 [Co] scale / shift");
  TORCH_CHECK(madnn_conv3x3_supported(H, W, Ci, Co), "conv3x3: unsupported shape Ci=", Ci, " Co=", Co, " W=", W);
  at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  at::Tensor y = at::empty({N, Co, H, W}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  at::Tensor part = at::empty({madnn_conv3x3_stat_rows((int64_t)N * H * W), 2, Co}, x.options().dtype(at::kFloat));
  check(madnn_conv3x3_fwd_bnb(x.data_ptr(), w.data_ptr(), y.data_ptr(), part.data_ptr<float>(), bny.data_ptr(),
                              scale.data_ptr<float>(), shift.data_ptr<float>(), N, H, W, Ci, Co, cur_stream(x)),
        "conv3x3_fwd_bnb");
  return {y, part};
}

// BN(+ReLU) backward from externally reduced sums (partial [G, 2, C]): -> (dx, dw, db)
std::tuple<at::Tensor, at::Tensor, at::Tensor> bn_bwd_ext(const at::Tensor& dy, const at::Tensor& x,
                                                          const c10::optional<at::Tensor>& w,
                                                          const at::Tensor& save_mean, const at::Tensor& save_invstd,
                                                          const at::Tensor& scale, const at::Tensor& shift,
                                                          const at::Tensor& partial, bool relu) {
  check_dev(x, "x");
  const int64_t C = x.size(1);
  const int64_t M = bn_rows(x, C);
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && dy.scalar_type() == at::kBFloat16 && dy.strides() == x.strides(),
              "bn_bwd_ext: bf16 dy / x of one layout");
  TORCH_CHECK(partial.scalar_type() == at::kFloat && partial.is_contiguous() && partial.dim() == 3 &&
                  partial.size(1) == 2 && partial.size(2) == C,
              "bn_bwd_ext: partial must be fp32 [rows, 2, C]");
  at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  auto fo = x.options().dtype(at::kFloat);
  at::Tensor dx = at::empty_like(x), dw = at::empty({C}, fo), db = at::empty({C}, fo), coef = at::empty({3 * C}, fo);
  at::Tensor ws = at::empty({(int64_t)madnn_bn_prereduce_floats((int)C)}, fo);
  check(madnn_bn_bwd_ext(dy.data_ptr(), x.data_ptr(), dx.data_ptr(), M, (int)C, relu ? 1 : 0, optf(w),
                         save_mean.data_ptr<float>(), save_invstd.data_ptr<float>(), scale.data_ptr<float>(),
                         shift.data_ptr<float>(), dw.data_ptr<float>(), db.data_ptr<float>(), coef.data_ptr<float>(),
                         partial.data_ptr<float>(), (int)partial.size(0), ws.data_ptr<float>(), cur_stream(x)),
        "bn_bwd_ext");
  return {dx, dw, db};
}

// dW [Co, Ci, 3, 3] (channels_last) of y = conv3x3(x, w): dy [N, Co, H, W], x [N, Ci, H, W], both NHWC bf16
at::Tensor conv3x3_wgrad(const at::Tensor& dy, const at::Tensor& x, bool out_bf16) {
  check_dev(x, "x");
  check_dev(dy, "dy");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && dy.scalar_type() == at::kBFloat16, "conv3x3_wgrad: bf16 only");
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast) && dy.dim() == 4 &&
                  dy.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv3x3_wgrad: NHWC 4-D tensors");
  TORCH_CHECK(dy.size(0) == x.size(0) && dy.size(2) == x.size(2) && dy.size(3) == x.size(3), "conv3x3_wgrad: shapes");
  const int N = (int)x.size(0), Ci = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3), Co = (int)dy.size(1);
  const int64_t nws = madnn_conv3x3_wgrad_ws(N, H, W, Ci, Co);
  TORCH_CHECK(nws > 0, "conv3x3_wgrad: unsupported shape Ci=", Ci, " Co=", Co, " H=", H, " W=", W);
  at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  at::Tensor ws = at::empty({nws}, x.options().dtype(at::kFloat));
  at::Tensor dw = at::empty({Co, Ci, 3, 3},
                            x.options().dtype(out_bf16 ? at::kBFloat16 : at::kFloat).memory_format(at::MemoryFormat::ChannelsLast));
  check(madnn_conv3x3_wgrad(dy.data_ptr(), x.data_ptr(), ws.data_ptr<float>(), dw.data_ptr(), out_bf16 ? 1 : 0, N, H, W,
                            Ci, Co, cur_stream(x)),
        "conv3x3_wgrad");
  return dw;
}

// ---- K10 ResNet stem: 7x7 / stride 2 / pad 3 convolution, 3 -> 64 channels, NHWC bf16 ---------
void stem_check_x(const at::Tensor& x) {
  check_dev(x, "x");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && x.dim() == 4 && x.size(1) == 3, "stem: x must be bf16 [N, 3, H, W]");
  TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast), "stem: x must be channels_last");
  TORCH_CHECK(madnn_stem_supported((int)x.size(2), (int)x.size(3)), "stem: unsupported image size ", x.size(2), "x",
              x.size(3));
}

// y = conv7x7s2(x, w) with w packed [64][7][8][4]; stats: partial [rows, 2, 64] (sum, sum sq) of y
std::tuple<at::Tensor, at::Tensor> stem_fwd(const at::Tensor& x, const at::Tensor& wp, bool stats) {
  stem_check_x(x);
  check_dev(wp, "wp");
  TORCH_CHECK(wp.scalar_type() == at::kBFloat16 && wp.is_contiguous() && wp.numel() == 64 * 224,
              "stem: packed weight must be contiguous bf16 [64, 7, 8, 4]");
  const int N = (int)x.size(0), H = (int)x.size(2), W = (int)x.size(3);
  const int64_t Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  at::Tensor y = at::empty({N, 64, Ho, Wo}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int64_t rows = stats ? madnn_stem_stat_rows(N, H, W) : 0;
  at::Tensor part = at::empty({rows, 2, 64}, x.options().dtype(at::kFloat));
  check(madnn_stem_fwd(x.data_ptr(), wp.data_ptr(), y.data_ptr(), stats ? part.data_ptr<float>() : nullptr, N, H, W,
                       cur_stream(x)),
        "stem_fwd");
  return {y, part};
}

// fp32 [64, 3, 7, 7] weight gradient
at::Tensor stem_wgrad(const at::Tensor& dy, const at::Tensor& x) {
  stem_check_x(x);
  check_dev(dy, "dy");
  const int N = (int)x.size(0), H = (int)x.size(2), W = (int)x.size(3);
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && dy.dim() == 4 && dy.size(0) == N && dy.size(1) == 64 &&
                  dy.size(2) == (H - 1) / 2 + 1 && dy.size(3) == (W - 1) / 2 + 1,
              "stem_wgrad: dy must be bf16 [N, 64, Ho, Wo]");
  TORCH_CHECK(dy.is_contiguous(at::MemoryFormat::ChannelsLast), "stem_wgrad: dy must be channels_last");
  at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  at::Tensor ws = at::empty({madnn_stem_wgrad_ws(N, H, W)}, x.options().dtype(at::kFloat));
  at::Tensor dw = at::empty({64, 3, 7, 7}, x.options().dtype(at::kFloat));
  check(madnn_stem_wgrad(x.data_ptr(), dy.data_ptr(), ws.data_ptr<float>(), dw.data_ptr<float>(), N, H, W,
                         cur_stream(x)),
        "stem_wgrad");
  return dw;
}

// ---- K6 fused softmax cross-entropy ------------------------------------------
// logits: [N, ld] or [B, S, ld] contiguous; V <= ld valid columns.  shift: causal
// LM (logit row (b, s) predicts target (b, s+1); the last position has no loss).
struct XentGeom {
  int64_t n_rows_all, n_loss_rows, seq, ld;
};

XentGeom xent_geom(const at::Tensor& logits, const at::Tensor& targets, bool shift) {
  TORCH_CHECK(logits.is_contiguous(), "xent: logits must be contiguous");
  TORCH_CHECK(targets.scalar_type() == at::kLong && targets.is_contiguous(), "xent: int64 contiguous targets");
  XentGeom g;
  g.ld = logits.size(-1);
  g.n_rows_all = logits.numel() / g.ld;
  TORCH_CHECK(targets.numel() == g.n_rows_all, "xent: one target per logit row");
  if (shift) {
    TORCH_CHECK(logits.dim() == 3, "xent shift mode needs [B, S, V] logits");
    g.seq = logits.size(1);
    g.n_loss_rows = logits.size(0) * (g.seq - 1);
  } else {
    g.seq = 0;
    g.n_loss_rows = g.n_rows_all;
  }
  return g;
}

std::tuple<at::Tensor, at::Tensor> xent_fwd(const at::Tensor& logits, const at::Tensor& targets, bool shift,
                                            int64_t V, int64_t ignore_index) {
  check_dev(logits, "logits");
  const XentGeom g = xent_geom(logits, targets, shift);
  TORCH_CHECK(V > 0 && V <= g.ld, "xent: bad vocabulary size");
  at::hip::HIPGuardMasqueradingAsCUDA guard(logits.device());
  auto fo = logits.options().dtype(at::kFloat);
  at::Tensor loss = at::empty({g.n_loss_rows}, fo), lse = at::empty({g.n_loss_rows}, fo);
  check(madnn_xent_fwd(logits.data_ptr(), dt_code(logits), targets.data_ptr<int64_t>(), g.n_loss_rows, g.seq, g.ld,
                       (int)V, (int)ignore_index, loss.data_ptr<float>(), lse.data_ptr<float>(), cur_stream(logits)),
        "xent_fwd");
  return {loss, lse};
}

at::Tensor xent_bwd(const at::Tensor& logits, const at::Tensor& targets, const at::Tensor& lse, bool shift, int64_t V,
                    int64_t ignore_index, const at::Tensor& gscale) {
  check_dev(logits, "logits");
  const XentGeom g = xent_geom(logits, targets, shift);
  TORCH_CHECK(gscale.scalar_type() == at::kFloat && gscale.is_cuda(), "xent: fp32 device grad scale");
  at::hip::HIPGuardMasqueradingAsCUDA guard(logits.device());
  at::Tensor grad = at::empty_like(logits);
  check(madnn_xent_bwd(logits.data_ptr(), dt_code(logits), targets.data_ptr<int64_t>(), lse.data_ptr<float>(),
                       g.n_loss_rows, g.seq, g.ld, (int)V, (int)ignore_index, g.n_rows_all, gscale.data_ptr<float>(),
                       grad.data_ptr(), cur_stream(logits)),
        "xent_bwd");
  return grad;
}

// K6f: loss rows and the finished logit gradient (scaled by gscale[0]) from one pass; 16-bit logits
// with 16-byte aligned rows only (xent_fused_ok).
bool xent_fused_ok(const at::Tensor& logits) {
  return (logits.scalar_type() == at::kBFloat16 || logits.scalar_type() == at::kHalf) && logits.is_contiguous() &&
         madnn_xent_fused_chunks(logits.size(-1)) > 0 && (reinterpret_cast<uintptr_t>(logits.data_ptr()) & 15) == 0;
}

std::tuple<at::Tensor, at::Tensor> xent_fused(const at::Tensor& logits, const at::Tensor& targets, bool shift,
                                              int64_t V, int64_t ignore_index, const at::Tensor& gscale) {
  check_dev(logits, "logits");
  const XentGeom g = xent_geom(logits, targets, shift);
  TORCH_CHECK(V > 0 && V <= g.ld, "xent: bad vocabulary size");
  TORCH_CHECK(xent_fused_ok(logits), "xent_fused: 16-bit contiguous logits with 16-byte aligned rows");
  TORCH_CHECK(gscale.scalar_type() == at::kFloat && gscale.is_cuda(), "xent: fp32 device grad scale");
  at::hip::HIPGuardMasqueradingAsCUDA guard(logits.device());
  at::Tensor loss = at::empty({g.n_loss_rows}, logits.options().dtype(at::kFloat));
  at::Tensor grad = at::empty_like(logits);
  check(madnn_xent_fused(logits.data_ptr(), dt_code(logits), targets.data_ptr<int64_t>(), g.n_loss_rows, g.seq, g.ld,
                         (int)V, (int)ignore_index, g.n_rows_all, gscale.data_ptr<float>(), loss.data_ptr<float>(),
                         grad.data_ptr(), cur_stream(logits)),
        "xent_fused");
  return {loss, grad};
}

void xent_rescale(at::Tensor grad, const at::Tensor& g) {
  check_dev(grad, "grad");
  TORCH_CHECK(grad.is_contiguous() && g.scalar_type() == at::kFloat && g.is_cuda(), "xent_rescale: bad operands");
  at::hip::HIPGuardMasqueradingAsCUDA guard(grad.device());
  check(madnn_xent_rescale(grad.data_ptr(), dt_code(grad), grad.numel(), g.data_ptr<float>(), cur_stream(grad)),
        "xent_rescale");
}

// K7 NHWC max-pool.  x: [N, C, H, W] in channels_last.  Returns (y, argmax bytes);
// argmax is empty when need_arg is false (inference).
std::tuple<at::Tensor, at::Tensor> maxpool_fwd(const at::Tensor& x, int64_t k, int64_t s, int64_t p, bool need_arg) {
  check_dev(x, "x");
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast), "maxpool: NHWC 4-D input");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(madnn_maxpool_supported(x.numel(), (int)C, (int)k), "maxpool: unsupported shape");
  TORCH_CHECK(k > 0 && s > 0 && p >= 0 && 2 * p <= k, "maxpool: bad window");
  const int64_t Ho = (H + 2 * p - k) / s + 1, Wo = (W + 2 * p - k) / s + 1;
  TORCH_CHECK(Ho > 0 && Wo > 0, "maxpool: empty output");
  at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  at::Tensor y = at::empty({N, C, Ho, Wo}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  at::Tensor arg = at::empty({need_arg ? N * Ho * Wo * C : 0}, x.options().dtype(at::kByte));
  check(madnn_maxpool_fwd(x.data_ptr(), y.data_ptr(), need_arg ? arg.data_ptr() : nullptr, (int)N, (int)H, (int)W,
                          (int)C, (int)Ho, (int)Wo, (int)k, (int)s, (int)p, dt_code(x), cur_stream(x)),
        "maxpool_fwd");
  return {y, arg};
}

at::Tensor maxpool_bwd(const at::Tensor& dy, const at::Tensor& arg, int64_t H, int64_t W, int64_t k, int64_t s,
                       int64_t p) {
  check_dev(dy, "dy");
  TORCH_CHECK(dy.dim() == 4, "maxpool_bwd: 4-D grad");
  const int64_t N = dy.size(0), C = dy.size(1), Ho = dy.size(2), Wo = dy.size(3);
  TORCH_CHECK(arg.numel() == dy.numel() && arg.scalar_type() == at::kByte, "maxpool_bwd: argmax map mismatch");
  TORCH_CHECK(Ho == (H + 2 * p - k) / s + 1 && Wo == (W + 2 * p - k) / s + 1, "maxpool_bwd: geometry mismatch");
  at::Tensor dyc = dy.contiguous(at::MemoryFormat::ChannelsLast);
  at::hip::HIPGuardMasqueradingAsCUDA guard(dy.device());
  at::Tensor dx = at::empty({N, C, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  TORCH_CHECK(madnn_maxpool_supported(dx.numel(), (int)C, (int)k), "maxpool_bwd: unsupported shape");
  check(madnn_maxpool_bwd(dyc.data_ptr(), arg.data_ptr(), dx.data_ptr(), (int)N, (int)H, (int)W, (int)C, (int)Ho,
                          (int)Wo, (int)k, (int)s, (int)p, dt_code(dy), cur_stream(dy)),
        "maxpool_bwd");
  return dx;
}

// maxpool 3x3/s2(relu(bn(y))) with the BN apply + ReLU fused into the pool (ResNet stem).
// y: bf16 NHWC raw BN input; scale/shift from bn_coef.  -> (pooled output, 1-byte argmax map)
std::tuple<at::Tensor, at::Tensor> pool_bn_fwd(const at::Tensor& y, const at::Tensor& scale, const at::Tensor& shift,
                                               int64_t p) {
  check_dev(y, "y");
  TORCH_CHECK(y.dim() == 4 && y.is_contiguous(at::MemoryFormat::ChannelsLast) && y.scalar_type() == at::kBFloat16,
              "pool_bn: bf16 NHWC 4-D input");
  const int64_t N = y.size(0), C = y.size(1), H = y.size(2), W = y.size(3);
  TORCH_CHECK(madnn_pool_bn_supported(y.numel(), (int)C) && p >= 0 && p <= 1, "pool_bn: unsupported shape");
  TORCH_CHECK(scale.numel() == C && shift.numel() == C && scale.scalar_type() == at::kFloat &&
                  shift.scalar_type() == at::kFloat && scale.is_contiguous() && shift.is_contiguous(),
              "pool_bn: fp32 [C] scale/shift");
  const int64_t Ho = (H + 2 * p - 3) / 2 + 1, Wo = (W + 2 * p - 3) / 2 + 1;
  TORCH_CHECK(Ho > 0 && Wo > 0, "pool_bn: empty output");
  at::hip::HIPGuardMasqueradingAsCUDA guard(y.device());
  at::Tensor out = at::empty({N, C, Ho, Wo}, y.options().memory_format(at::MemoryFormat::ChannelsLast));
  at::Tensor arg = at::empty({N * Ho * Wo * C}, y.options().dtype(at::kByte));
  check(madnn_pool_bn_fwd(y.data_ptr(), scale.data_ptr<float>(), shift.data_ptr<float>(), out.data_ptr(),
                          arg.data_ptr(), (int)N, (int)H, (int)W, (int)C, (int)Ho, (int)Wo, (int)p, cur_stream(y)),
        "pool_bn_fwd");
  return {out, arg};
}

// -> (dy, dw, db)
std::tuple<at::Tensor, at::Tensor, at::Tensor> pool_bn_bwd(const at::Tensor& dp, const at::Tensor& arg,
                                                           const at::Tensor& y, const c10::optional<at::Tensor>& w,
                                                           const at::Tensor& mean, const at::Tensor& invstd,
                                                           const at::Tensor& scale, const at::Tensor& shift,
                                                           int64_t p) {
  check_dev(y, "y");
  const int64_t N = y.size(0), C = y.size(1), H = y.size(2), W = y.size(3);
  const int64_t Ho = (H + 2 * p - 3) / 2 + 1, Wo = (W + 2 * p - 3) / 2 + 1;
  TORCH_CHECK(dp.dim() == 4 && dp.size(0) == N && dp.size(1) == C && dp.size(2) == Ho && dp.size(3) == Wo,
              "pool_bn_bwd: gradient shape");
  TORCH_CHECK(arg.numel() == dp.numel() && arg.scalar_type() == at::kByte, "pool_bn_bwd: argmax map mismatch");
  at::Tensor dpc = dp.to(at::kBFloat16).contiguous(at::MemoryFormat::ChannelsLast);
  at::hip::HIPGuardMasqueradingAsCUDA guard(y.device());
  auto fo = y.options().dtype(at::kFloat);
  at::Tensor dy = at::empty_like(y);
  at::Tensor dw = at::empty({C}, fo), db = at::empty({C}, fo), coef = at::empty({3 * C}, fo);
  at::Tensor ws = at::empty({(int64_t)madnn_pool_bn_bwd_rows(N * H * W, (int)C) * 2 * C}, fo);
  check(madnn_pool_bn_bwd(dpc.data_ptr(), arg.data_ptr(), y.data_ptr(), optf(w), mean.data_ptr<float>(),
                          invstd.data_ptr<float>(), scale.data_ptr<float>(), shift.data_ptr<float>(), dy.data_ptr(),
                          dw.data_ptr<float>(), db.data_ptr<float>(), coef.data_ptr<float>(), ws.data_ptr<float>(),
                          (int)N, (int)H, (int)W, (int)C, (int)Ho, (int)Wo, (int)p, cur_stream(y)),
        "pool_bn_bwd");
  return {dy, dw, db};
}

// K11 Linear bias gradient.  dy (and pre): [..., N], row-major contiguous.  Returns
// (db [N] in bias_dtype, dp) where dp = dy * gelu_tanh'(pre) when pre is given (else empty).
std::tuple<at::Tensor, at::Tensor> bias_grad(const at::Tensor& dy, const c10::optional<at::Tensor>& pre,
                                             at::ScalarType bias_dtype, int64_t gelu_kind) {
  TORCH_CHECK(gelu_kind == 1 || gelu_kind == 2, "bias_grad: gelu_kind 1 (tanh) or 2 (erf)");
  check_dev(dy, "dy");
  at::Tensor g = dy.contiguous();
  const int64_t N = g.size(-1), M = g.numel() / N;
  TORCH_CHECK(madnn_bias_grad_supported(M, (int)N), "bias_grad: last dim must be a multiple of 8");
  at::Tensor pc, dp;
  if (pre.has_value()) {
    pc = pre->contiguous();
    TORCH_CHECK(pc.sizes() == g.sizes() && pc.scalar_type() == g.scalar_type(), "bias_grad: pre mismatch");
  }
  at::hip::HIPGuardMasqueradingAsCUDA guard(dy.device());
  if (pc.defined()) dp = at::empty_like(g);
  else dp = at::empty({0}, g.options());
  const int R = madnn_bias_grad_rows(M, (int)N, pc.defined() ? 1 : 0);
  at::Tensor partial = at::empty({R, N}, g.options().dtype(at::kFloat));
  at::Tensor db = at::empty({N}, g.options().dtype(bias_dtype));
  check(madnn_bias_grad(g.data_ptr(), pc.defined() ? pc.data_ptr() : nullptr, pc.defined() ? dp.data_ptr() : nullptr,
                        M, (int)N, dt_code(g), partial.data_ptr<float>(), db.data_ptr(), dt_code(db), (int)gelu_kind,
                        cur_stream(g)),
        "bias_grad");
  return {db, dp};
}

// GELU forward (K11 family, kind 1 tanh / 2 erf): y = gelu(x), x contiguous float, numel % 8 == 0.
at::Tensor gelu_fwd(const at::Tensor& x, int64_t kind) {
  TORCH_CHECK(kind == 1 || kind == 2, "gelu_fwd: kind 1 (tanh) or 2 (erf)");
  check_dev(x, "x");
  at::Tensor xc = x.contiguous();
  TORCH_CHECK(xc.numel() % 8 == 0, "gelu_fwd: numel must be a multiple of 8");
  at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  at::Tensor y = at::empty_like(xc);
  if (xc.numel())
    check(madnn_gelu_fwd(xc.data_ptr(), y.data_ptr(), xc.numel(), dt_code(xc), (int)kind, cur_stream(xc)), "gelu_fwd");
  return y;
}

// K14 / K15 move 16 bytes per lane: every operand must start on a 16-byte boundary (a contiguous
// slice of a larger buffer need not)
static void check_aligned16(const at::Tensor& t, const char* op, const char* name) {
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, op, ": ", name, " must be 16-byte aligned");
}

// K14: heads 0..rot_heads-1 of the packed bf16 QKV [B, S, NH, D] rotated (inverse: the transpose
// rotation); in place (rope_qkv_, the backward on dQKV) or into a new packed tensor (rope_qkv, the
// v heads copied); cos / sin fp32 [>= S][D]
at::Tensor rope_qkv_impl(const at::Tensor& qkv, at::Tensor out, const at::Tensor& cos, const at::Tensor& sin,
                         int64_t rot_heads, bool inverse) {
  check_dev(qkv, "qkv");
  TORCH_CHECK(qkv.scalar_type() == at::kBFloat16 && qkv.dim() == 4 && qkv.is_contiguous(),
              "rope_qkv_: qkv must be a contiguous bf16 [B, S, heads, D]");
  const int64_t S = qkv.size(1), NH = qkv.size(2), D = qkv.size(3);
  TORCH_CHECK(D % 16 == 0 && rot_heads >= 0 && rot_heads <= NH, "rope_qkv_: D % 16 and rot_heads <= heads");
  for (const at::Tensor* t : {&cos, &sin}) {
    TORCH_CHECK(t->device() == qkv.device() && t->scalar_type() == at::kFloat && t->dim() == 2 && t->is_contiguous() &&
                    t->size(0) >= S && t->size(1) == D,
                "rope_qkv_: cos / sin must be contiguous fp32 [>= S, D] on the device");
  }
  for (const at::Tensor* t : {&qkv, const_cast<const at::Tensor*>(&out), &cos, &sin}) check_aligned16(*t, "rope_qkv", "qkv / out / cos / sin");
  at::hip::HIPGuardMasqueradingAsCUDA guard(qkv.device());
  check(madnn_rope_qkv(qkv.data_ptr(), out.data_ptr(), cos.data_ptr<float>(), sin.data_ptr<float>(), qkv.size(0) * S,
                       (int)S, (int)NH, (int)rot_heads, (int)D, inverse ? 1 : 0, cur_stream(qkv)),
        "rope_qkv");
  return out;
}

at::Tensor rope_qkv_(at::Tensor qkv, const at::Tensor& cos, const at::Tensor& sin, int64_t rot_heads, bool inverse) {
  return rope_qkv_impl(qkv, qkv, cos, sin, rot_heads, inverse);
}

at::Tensor rope_qkv(const at::Tensor& qkv, const at::Tensor& cos, const at::Tensor& sin, int64_t rot_heads,
                    bool inverse) {
  check_dev(qkv, "qkv");
  return rope_qkv_impl(qkv, at::empty_like(qkv), cos, sin, rot_heads, inverse);
}

// K15: h = silu(g) * u of the fused gate_up output gu [..., 2I] -> [..., I]
at::Tensor swiglu_fwd(const at::Tensor& gu) {
  check_dev(gu, "gu");
  TORCH_CHECK(gu.scalar_type() == at::kBFloat16 && gu.is_contiguous() && gu.size(-1) % 16 == 0,
              "swiglu: gu must be contiguous bf16 with a last dim that is a multiple of 16");
  const int64_t I = gu.size(-1) / 2, M = gu.numel() / (2 * I);
  auto shape = gu.sizes().vec();
  shape.back() = I;
  check_aligned16(gu, "swiglu", "gu");
  at::hip::HIPGuardMasqueradingAsCUDA guard(gu.device());
  at::Tensor h = at::empty(shape, gu.options());
  check(madnn_swiglu_fwd(gu.data_ptr(), h.data_ptr(), M, (int)I, cur_stream(gu)), "swiglu_fwd");
  return h;
}

// K15 backward: d[g | u] from dh [..., I] and gu [..., 2I]
at::Tensor swiglu_bwd(const at::Tensor& dh, const at::Tensor& gu) {
  check_dev(gu, "gu");
  TORCH_CHECK(gu.scalar_type() == at::kBFloat16 && gu.is_contiguous() && gu.size(-1) % 16 == 0, "swiglu_bwd: gu");
  const int64_t I = gu.size(-1) / 2, M = gu.numel() / (2 * I);
  at::Tensor d = dh.to(at::kBFloat16).contiguous();
  TORCH_CHECK(d.numel() == M * I, "swiglu_bwd: dh must have gu's rows and I columns");
  check_aligned16(gu, "swiglu_bwd", "gu");
  check_aligned16(d, "swiglu_bwd", "dh");
  at::hip::HIPGuardMasqueradingAsCUDA guard(gu.device());
  at::Tensor dgu = at::empty_like(gu);
  check(madnn_swiglu_bwd(d.data_ptr(), gu.data_ptr(), dgu.data_ptr(), M, (int)I, cur_stream(gu)), "swiglu_bwd");
  return dgu;
}

// K8 attention.  q: [B, S, H, D], k/v: [B, S, Hkv, D] bf16 views with a contiguous last dim
// (any other strides, e.g. slices of one packed QKV projection).
void attn_check(const at::Tensor& t, const char* name, int64_t D) {
  check_dev(t, name);
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, "attention: ", name, " must be bf16");
  TORCH_CHECK(t.dim() == 4 && t.size(3) == D && t.stride(3) == 1, "attention: ", name, " must be [B, S, heads, D]");
  for (int i = 0; i < 3; ++i) TORCH_CHECK(t.stride(i) % 8 == 0, "attention: ", name, " strides must be multiples of 8");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, "attention: ", name, " must be 16-byte aligned");
}

MadnnAttnArgs attn_args(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, double scale) {
  const int64_t D = q.size(3);
  TORCH_CHECK(madnn_attn_supported((int)D), "attention: head dim must be 64 or 128");
  attn_check(q, "q", D);
  attn_check(k, "k", D);
  attn_check(v, "v", D);
  TORCH_CHECK(k.sizes() == v.sizes() && k.size(0) == q.size(0) && k.size(1) == q.size(1), "attention: k/v shape");
  TORCH_CHECK(q.size(2) % k.size(2) == 0, "attention: query heads must be a multiple of kv heads");
  TORCH_CHECK(q.size(1) < (1ll << 30) && q.size(0) * q.size(2) < (1ll << 30), "attention: problem too large");
  MadnnAttnArgs a{};
  a.q = reinterpret_cast<const uint16_t*>(q.data_ptr());
  a.k = reinterpret_cast<const uint16_t*>(k.data_ptr());
  a.v = reinterpret_cast<const uint16_t*>(v.data_ptr());
  a.q_sb = q.stride(0); a.q_ss = q.stride(1); a.q_sh = q.stride(2);
  a.k_sb = k.stride(0); a.k_ss = k.stride(1); a.k_sh = k.stride(2);
  a.v_sb = v.stride(0); a.v_ss = v.stride(1); a.v_sh = v.stride(2);
  a.B = (int)q.size(0); a.S = (int)q.size(1); a.H = (int)q.size(2); a.Hkv = (int)k.size(2);
  a.scale = (float)scale;
  a.scale_log2 = (float)(scale * 1.4426950408889634);
  return a;
}

std::tuple<at::Tensor, at::Tensor> attn_fwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                                            bool causal, double scale) {
  MadnnAttnArgs a = attn_args(q, k, v, scale);
  at::hip::HIPGuardMasqueradingAsCUDA guard(q.device());
  at::Tensor o = at::empty({q.size(0), q.size(1), q.size(2), q.size(3)}, q.options());
  at::Tensor lse = at::empty({q.size(0), q.size(2), q.size(1)}, q.options().dtype(at::kFloat));
  a.o = reinterpret_cast<uint16_t*>(o.data_ptr());
  a.lse = lse.data_ptr<float>();
  a.o_sb = o.stride(0); a.o_ss = o.stride(1); a.o_sh = o.stride(2);
  check(madnn_attn_fwd(&a, (int)q.size(3), causal ? 1 : 0, cur_stream(q)), "attn_fwd");
  return {o, lse};
}

// Writes dq/dk/dv into the given (possibly strided, e.g. one packed dQKV buffer) outputs.
void attn_bwd(const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
              const at::Tensor& o, const at::Tensor& lse, const at::Tensor& dq, const at::Tensor& dk,
              const at::Tensor& dv, bool causal, double scale, const c10::optional<at::Tensor>& colsum) {
  MadnnAttnArgs a = attn_args(q, k, v, scale);
  const int64_t D = q.size(3);
  TORCH_CHECK(o.is_contiguous() && o.sizes() == q.sizes(), "attn_bwd: o must be contiguous [B, S, H, D]");
  at::Tensor doc = dout.contiguous();
  TORCH_CHECK(doc.sizes() == o.sizes() && doc.scalar_type() == at::kBFloat16, "attn_bwd: grad shape/dtype");
  attn_check(dq, "dq", D);
  attn_check(dk, "dk", D);
  attn_check(dv, "dv", D);
  TORCH_CHECK(dq.sizes() == q.sizes() && dk.sizes() == k.sizes() && dv.sizes() == v.sizes(), "attn_bwd: grad shapes");
  TORCH_CHECK(lse.is_contiguous() && lse.numel() == q.size(0) * q.size(1) * q.size(2), "attn_bwd: lse");
  at::hip::HIPGuardMasqueradingAsCUDA guard(q.device());
  at::Tensor delta = at::empty_like(lse);
  a.o = reinterpret_cast<uint16_t*>(o.data_ptr());
  a.lse = lse.data_ptr<float>();
  a.dout = reinterpret_cast<const uint16_t*>(doc.data_ptr());
  a.delta = delta.data_ptr<float>();
  a.o_sb = o.stride(0); a.o_ss = o.stride(1); a.o_sh = o.stride(2);
  a.dq = reinterpret_cast<uint16_t*>(dq.data_ptr());
  a.dk = reinterpret_cast<uint16_t*>(dk.data_ptr());
  a.dv = reinterpret_cast<uint16_t*>(dv.data_ptr());
  a.dq_sb = dq.stride(0); a.dq_ss = dq.stride(1); a.dq_sh = dq.stride(2);
  a.dk_sb = dk.stride(0); a.dk_ss = dk.stride(1); a.dk_sh = dk.stride(2);
  a.dv_sb = dv.stride(0); a.dv_ss = dv.stride(1); a.dv_sh = dv.stride(2);
  // colsum (optional, fp32 or bf16 [(H + 2 Hkv) D]): the column sums of dq | dk | dv over all B * S rows
  const bool cs = colsum.has_value() && colsum->defined();
  at::Tensor cpart;
  int64_t R = 0, C = 0;
  if (cs) {
    C = (q.size(2) + 2 * k.size(2)) * D;
    TORCH_CHECK((colsum->scalar_type() == at::kFloat || colsum->scalar_type() == at::kBFloat16) &&
                    colsum->is_contiguous() && colsum->numel() == C,
                "attn_bwd: colsum must be a contiguous fp32 / bf16 [(H + 2 Hkv) * D]");
    R = madnn_attn_colsum_rows(a.B, a.S);
    cpart = at::empty({R, C}, q.options().dtype(at::kFloat));
    a.cpart = cpart.data_ptr<float>();
  }
  check(madnn_attn_bwd(&a, (int)D, causal ? 1 : 0, cur_stream(q)), "attn_bwd");
  if (cs)
    check(madnn_attn_colsum_finalize(a.cpart, R, C, colsum->data_ptr(), colsum->scalar_type() == at::kBFloat16 ? 1 : 0,
                                     cur_stream(q)),
          "attn_colsum");
}

// Hardware-queue aliasing probe (probe.hip): bounded flag wait / flag set on the current stream.
void hwq_wait(const at::Tensor& flag, int64_t expect, int64_t timeout_us, at::Tensor out) {
  check_dev(flag, "flag");
  check_dev(out, "out");
  TORCH_CHECK(flag.scalar_type() == at::kInt && out.scalar_type() == at::kInt && out.numel() >= 2 &&
                  out.is_contiguous() && timeout_us > 0 && timeout_us <= 2000000,
              "hwq_wait: int32 flag, int32 out[>=2], 0 < timeout_us <= 2 s");
  at::hip::HIPGuardMasqueradingAsCUDA guard(flag.device());
  check(madnn_hwq_wait(flag.data_ptr<int>(), (int)expect, timeout_us, out.data_ptr<int>(), cur_stream(flag)),
        "hwq_wait");
}

void hwq_set(at::Tensor flag, int64_t val) {
  check_dev(flag, "flag");
  TORCH_CHECK(flag.scalar_type() == at::kInt, "hwq_set: int32 flag");
  at::hip::HIPGuardMasqueradingAsCUDA guard(flag.device());
  check(madnn_hwq_set(flag.data_ptr<int>(), (int)val, cur_stream(flag)), "hwq_set");
}

// Pipeline replay (probe.hip): one rendezvous batch of P2P messages / a compute stand-in.
void hwq_batch(const at::Tensor& kinds, const at::Tensor& msgs, at::Tensor a, at::Tensor b, int64_t epoch,
               int64_t timeout_us, at::Tensor ok, const at::Tensor& ok_index) {
  for (const at::Tensor* t : {&kinds, &msgs, static_cast<const at::Tensor*>(&a), static_cast<const at::Tensor*>(&b),
                              static_cast<const at::Tensor*>(&ok), &ok_index}) {
    check_dev(*t, "hwq_batch operand");
    TORCH_CHECK(t->scalar_type() == at::kInt && t->is_contiguous(), "hwq_batch: contiguous int32 operands");
  }
  const int64_t n = kinds.numel();
  TORCH_CHECK(msgs.numel() == n && ok_index.numel() == n && timeout_us > 0 && timeout_us <= 2000000,
              "hwq_batch: kinds / msgs / ok_index of one length, 0 < timeout_us <= 2 s");
  at::hip::HIPGuardMasqueradingAsCUDA guard(a.device());
  check(madnn_hwq_batch(kinds.data_ptr<int>(), msgs.data_ptr<int>(), (int)n, a.data_ptr<int>(), b.data_ptr<int>(),
                        (int)epoch, timeout_us, ok.data_ptr<int>(), ok_index.data_ptr<int>(), cur_stream(a)),
        "hwq_batch");
}

void hwq_spin(const at::Tensor& like, int64_t spin_us) {
  check_dev(like, "like");
  TORCH_CHECK(spin_us >= 0 && spin_us <= 100000, "hwq_spin: 0 <= spin_us <= 100 ms");
  at::hip::HIPGuardMasqueradingAsCUDA guard(like.device());
  check(madnn_hwq_spin(spin_us, cur_stream(like)), "hwq_spin");
}

}  // namespace

TORCH_LIBRARY(madnn, m) {
  m.def("hwq_batch(Tensor kinds, Tensor msgs, Tensor(a!) a, Tensor(b!) b, int epoch, int timeout_us, Tensor(c!) ok, "
        "Tensor ok_index) -> ()");
  m.def("hwq_spin(Tensor like, int spin_us) -> ()");
  m.def("hwq_wait(Tensor flag, int expect, int timeout_us, Tensor(a!) out) -> ()");
  m.def("hwq_set(Tensor(a!) flag, int val) -> ()");
  m.def(
      "bn_fwd(Tensor x, Tensor? res, Tensor? w, Tensor? b, Tensor(a!)? run_mean, Tensor(b!)? run_var, "
      "Tensor(c!)? nbt, bool training, float momentum, float eps, bool relu, Tensor? partial=None) -> (Tensor, Tensor, "
      "Tensor, Tensor, Tensor, Tensor)");
  m.def("xent_fwd(Tensor logits, Tensor targets, bool shift, int V, int ignore_index) -> (Tensor, Tensor)");
  m.def(
      "xent_bwd(Tensor logits, Tensor targets, Tensor lse, bool shift, int V, int ignore_index, Tensor gscale) -> "
      "Tensor");
  m.def(
      "xent_fused(Tensor logits, Tensor targets, bool shift, int V, int ignore_index, Tensor gscale) -> "
      "(Tensor, Tensor)");
  m.def("xent_rescale(Tensor(a!) grad, Tensor g) -> ()");
  m.def(
      "bn_bwd(Tensor dy, Tensor x, Tensor? mask, bool has_res, Tensor? w, Tensor save_mean, Tensor save_invstd, "
      "Tensor scale, Tensor shift, bool relu, bool need_wgrad, bool write_dres=True) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def(
      "bn_fwd_dual(Tensor x, Tensor r, Tensor? w, Tensor? b, Tensor(a!)? run_mean, Tensor(b!)? run_var, "
      "Tensor(c!)? nbt, float momentum, float eps, Tensor? partial, Tensor? w_r, Tensor? b_r, "
      "Tensor(d!)? run_mean_r, Tensor(e!)? run_var_r, Tensor(f!)? nbt_r, float momentum_r, float eps_r, "
      "Tensor? partial_r) -> Tensor[]");
  m.def(
      "bn_bwd_dual(Tensor dy, Tensor x, Tensor r, Tensor mask, Tensor? w, Tensor save_mean, Tensor save_invstd, "
      "Tensor? w_r, Tensor save_mean_r, Tensor save_invstd_r) -> Tensor[]");
  m.def("attn_fwd(Tensor q, Tensor k, Tensor v, bool causal, float scale) -> (Tensor, Tensor)");
  m.def(
      "attn_bwd(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor o, Tensor lse, Tensor(a!) dq, Tensor(b!) dk, "
      "Tensor(c!) dv, bool causal, float scale, Tensor(d!)? colsum=None) -> ()");
  m.def("conv1x1_fwd(Tensor x, Tensor w, bool stats) -> (Tensor, Tensor)");
  m.def("conv1x1_dgrad(Tensor dy, Tensor w, Tensor? res=None, Tensor? resmask=None) -> Tensor");
  m.def("conv1x1_dgrad_bnb(Tensor dy, Tensor w, Tensor bny, Tensor scale, Tensor shift) -> (Tensor, Tensor)");
  m.def(
      "conv3x3_fwd_bnb(Tensor x, Tensor w, Tensor bny, Tensor scale, Tensor shift) -> (Tensor, Tensor)");
  m.def(
      "bn_bwd_ext(Tensor dy, Tensor x, Tensor? w, Tensor save_mean, Tensor save_invstd, Tensor scale, Tensor shift, "
      "Tensor partial, bool relu) -> (Tensor, Tensor, Tensor)");
  m.def("conv1x1_wgrad(Tensor dy, Tensor x, bool out_bf16=False) -> Tensor");
  m.def(
      "bn_coef(Tensor x, Tensor? w, Tensor? b, Tensor(a!)? run_mean, Tensor(b!)? run_var, Tensor(c!)? nbt, "
      "float momentum, float eps, Tensor? partial=None) -> Tensor[]");
  m.def("stem_fwd(Tensor x, Tensor wp, bool stats) -> (Tensor, Tensor)");
  m.def("linear_fwd(Tensor x, Tensor w, Tensor? bias, Tensor? res, int act, bool save_aux) -> (Tensor, Tensor)");
  m.def("linear_dgrad(Tensor dy, Tensor w, Tensor? res, bool accumulate) -> Tensor");
  m.def("linear_wgrad(Tensor dy, Tensor x, Tensor? out, bool accumulate, int splits) -> Tensor");
  m.def("linear_wgrad4(Tensor dy, Tensor x, Tensor? out, bool accumulate, int splits) -> Tensor");
  m.def("linear_wgrad4h(Tensor dy, Tensor x, Tensor? out, bool accumulate, int splits) -> Tensor");
  m.def("wgrad_splits(int M, int N, int K) -> int", &wgrad_splits);
  m.def("gemmp_supported(int I, int J, int K, bool has_bias) -> bool", &gemmp_supported);
  m.def("linear_fwd_p(Tensor x, Tensor w, Tensor? bias, int act) -> (Tensor, Tensor)");
  m.def("linear_dgrad_p(Tensor dy, Tensor w, Tensor? pre, ScalarType bias_dtype, int gelu_kind=1) -> (Tensor, Tensor)");
  m.def("conv3x3_fwd(Tensor x, Tensor w, bool stats) -> (Tensor, Tensor)");
  m.def("conv3x3_fwd_s2(Tensor x, Tensor w, bool stats) -> (Tensor, Tensor)");
  m.def("conv3x3_wgrad(Tensor dy, Tensor x, bool out_bf16) -> Tensor");
  m.def("stem_wgrad(Tensor dy, Tensor x) -> Tensor");
  m.def("bias_grad(Tensor dy, Tensor? pre, ScalarType bias_dtype, int gelu_kind=1) -> (Tensor, Tensor)");
  m.def("gelu_fwd(Tensor x, int kind=1) -> Tensor");
  m.def("rope_qkv_(Tensor(a!) qkv, Tensor cos, Tensor sin, int rot_heads, bool inverse) -> Tensor(a!)");
  m.def("rope_qkv(Tensor qkv, Tensor cos, Tensor sin, int rot_heads, bool inverse) -> Tensor");
  m.def("swiglu_fwd(Tensor gu) -> Tensor");
  m.def("swiglu_bwd(Tensor dh, Tensor gu) -> Tensor");
  m.def("maxpool_fwd(Tensor x, int k, int s, int p, bool need_arg) -> (Tensor, Tensor)");
  m.def("pool_bn_fwd(Tensor y, Tensor scale, Tensor shift, int p) -> (Tensor, Tensor)");
  m.def(
      "pool_bn_bwd(Tensor dp, Tensor arg, Tensor y, Tensor? w, Tensor mean, Tensor invstd, Tensor scale, Tensor shift, "
      "int p) -> (Tensor, Tensor, Tensor)");
  m.def("maxpool_bwd(Tensor dy, Tensor arg, int H, int W, int k, int s, int p) -> Tensor");
  m.def("bucket_pack(Tensor[] srcs, Tensor(a!) flat, int[] offsets, float scale) -> ()");
  m.def("bucket_unpack(Tensor(a!)[] dsts, Tensor flat, int[] offsets, float scale) -> ()");
  m.def("flat_scale_cast(Tensor src, Tensor(a!) dst, float scale) -> ()");
  m.def(
      "sgd_step(Tensor(a!) master, Tensor grad, Tensor(b!)? mom, Tensor(c!)? model, float lr, float momentum, "
      "float dampening, float weight_decay, bool nesterov, bool first_step, float grad_scale, Tensor? dscale) -> ()");
  m.def(
      "adam_step(Tensor(a!) master, Tensor grad, Tensor(b!) m1, Tensor(c!) m2, Tensor(d!)? model, float lr, "
      "float beta1, float beta2, float eps, float weight_decay, bool adamw, int step, float grad_scale, "
      "Tensor? dscale) -> ()");
  m.def("grad_norm(Tensor[] flats, float max_norm, float scale) -> Tensor");
  m.def("norm_fwd(Tensor x, Tensor? res, Tensor w, Tensor? b, float eps, bool rms) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def(
      "norm_bwd(Tensor dy, Tensor x, Tensor w, Tensor mean, Tensor rstd, Tensor? dres, bool rms, bool has_bias, "
      "bool colsum=False, bool colsum_bf16=False) -> (Tensor, Tensor, Tensor, Tensor)");
}

TORCH_LIBRARY_IMPL(madnn, CUDA, m) {
  m.impl("bucket_pack", bucket_pack);
  m.impl("bucket_unpack", bucket_unpack);
  m.impl("flat_scale_cast", flat_scale_cast);
  m.impl("sgd_step", sgd_step);
  m.impl("adam_step", adam_step);
  m.impl("grad_norm", grad_norm);
  m.impl("norm_fwd", norm_fwd);
  m.impl("norm_bwd", norm_bwd);
  m.impl("bn_fwd", bn_fwd);
  m.impl("bn_bwd", bn_bwd);
  m.impl("bn_fwd_dual", bn_fwd_dual);
  m.impl("bn_coef", bn_coef);
  m.impl("conv3x3_fwd_bnb", conv3x3_fwd_bnb);
  m.impl("conv1x1_dgrad_bnb", conv1x1_dgrad_bnb);
  m.impl("bn_bwd_ext", bn_bwd_ext);
  m.impl("bn_bwd_dual", bn_bwd_dual);
  m.impl("xent_fwd", xent_fwd);
  m.impl("xent_bwd", xent_bwd);
  m.impl("xent_fused", xent_fused);
  m.impl("xent_rescale", xent_rescale);
  m.impl("maxpool_fwd", maxpool_fwd);
  m.impl("pool_bn_fwd", pool_bn_fwd);
  m.impl("pool_bn_bwd", pool_bn_bwd);
  m.impl("bias_grad", bias_grad);
  m.impl("gelu_fwd", gelu_fwd);
  m.impl("rope_qkv_", rope_qkv_);
  m.impl("rope_qkv", rope_qkv);
  m.impl("swiglu_fwd", swiglu_fwd);
  m.impl("swiglu_bwd", swiglu_bwd);
  m.impl("attn_fwd", attn_fwd);
  m.impl("attn_bwd", attn_bwd);
  m.impl("maxpool_bwd", maxpool_bwd);
  m.impl("conv1x1_fwd", conv1x1_fwd);
  m.impl("conv1x1_dgrad", conv1x1_dgrad);
  m.impl("conv1x1_wgrad", conv1x1_wgrad);
  m.impl("stem_fwd", stem_fwd);
  m.impl("stem_wgrad", stem_wgrad);
  m.impl("linear_fwd", linear_fwd);
  m.impl("linear_dgrad", linear_dgrad);
  m.impl("linear_wgrad", linear_wgrad);
  m.impl("linear_wgrad4", linear_wgrad4);
  m.impl("linear_wgrad4h", linear_wgrad4h);
  m.impl("linear_fwd_p", linear_fwd_p);
  m.impl("linear_dgrad_p", linear_dgrad_p);
  m.impl("conv3x3_fwd", conv3x3_fwd);
  m.impl("conv3x3_fwd_s2", conv3x3_fwd_s2);
  m.impl("conv3x3_wgrad", conv3x3_wgrad);
  m.impl("hwq_wait", hwq_wait);
  m.impl("hwq_set", hwq_set);
  m.impl("hwq_batch", hwq_batch);
  m.impl("hwq_spin", hwq_spin);
}
