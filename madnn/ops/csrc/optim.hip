// K1 FusedSGD and K2 FusedAdam/AdamW over flat fp32 master buffers, plus a
// two-stage gradient L2-norm (for clipping without a host sync).
//
// Reference origin: Torch7's accUpdateGradParameters, i.e. a gradient step
// fused into the weight update (reference datamodule.lua:142).
// Here the optimizer walks one flat bucket per launch:
//   read  grad (f32 or bf16), fp32 master, fp32 state
//   write fp32 master, fp32 state, and the bf16 model copy the forward uses
// so the bf16 parameters never need a separate cast kernel.  All streams are
// 16-byte-per-lane vector accesses; grid = a few waves per CU, grid-stride.
// An optional device-side scale (e.g. the clip coefficient produced by the
// norm kernels below) multiplies the gradient without a host round trip.
#include "common.h"

namespace madnn {

constexpr int kOptThreads = 256;
constexpr int kOptVec = 8;

struct SGDHyper {
  float lr, momentum, dampening, weight_decay, grad_scale;
  int nesterov, first_step;
};

struct AdamHyper {
  float lr, beta1, beta2, eps, weight_decay, grad_scale;
  float bias_corr1, bias_corr2_sqrt;  // 1 - b1^t, sqrt(1 - b2^t)
  int adamw;
};

// MDT < 0 => no model copy.
template <int GDT, int MDT>
__global__ __launch_bounds__(kOptThreads) void sgd_kernel(float* __restrict__ master, const void* __restrict__ grad,
                                                          float* __restrict__ mom, void* __restrict__ model,
                                                          int64_t n, SGDHyper h, const float* __restrict__ dscale) {
  const float gs = h.grad_scale * (dscale ? dscale[0] : 1.0f);
  const int64_t stride = (int64_t)gridDim.x * kOptThreads * kOptVec;
  for (int64_t i = ((int64_t)blockIdx.x * kOptThreads + threadIdx.x) * kOptVec; i < n; i += stride) {
    if (i + kOptVec <= n) {
      float p[8], g[8], m[8];
      load8<kF32>(master, i, p);
      load8<GDT>(grad, i, g);
      if (h.momentum != 0.f && !h.first_step) load8<kF32>(mom, i, m);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float gj = g[j] * gs;
        if (h.weight_decay != 0.f) gj += h.weight_decay * p[j];
        if (h.momentum != 0.f) {
          m[j] = h.first_step ? gj : h.momentum * m[j] + (1.f - h.dampening) * gj;
          gj = h.nesterov ? gj + h.momentum * m[j] : m[j];
        }
        p[j] -= h.lr * gj;
      }
      store8<kF32>(master, i, p);
      if (h.momentum != 0.f) store8<kF32>(mom, i, m);
      if constexpr (MDT >= 0) store8<MDT>(model, i, p);
    } else {
      for (int64_t k = i; k < n; ++k) {
        float pk = master[k];
        float gj = Elem<GDT>::load(static_cast<const typename Elem<GDT>::T*>(grad), k) * gs;
        if (h.weight_decay != 0.f) gj += h.weight_decay * pk;
        if (h.momentum != 0.f) {
          float mk = h.first_step ? gj : h.momentum * mom[k] + (1.f - h.dampening) * gj;
          mom[k] = mk;
          gj = h.nesterov ? gj + h.momentum * mk : mk;
        }
        pk -= h.lr * gj;
        master[k] = pk;
        if constexpr (MDT >= 0) Elem<MDT>::store(static_cast<typename Elem<MDT>::T*>(model), k, pk);
      }
    }
  }
}

template <int GDT, int MDT>
__global__ __launch_bounds__(kOptThreads) void adam_kernel(float* __restrict__ master, const void* __restrict__ grad,
                                                           float* __restrict__ m1, float* __restrict__ m2,
                                                           void* __restrict__ model, int64_t n, AdamHyper h,
                                                           const float* __restrict__ dscale) {
  const float gs = h.grad_scale * (dscale ? dscale[0] : 1.0f);
  const float step = h.lr / h.bias_corr1;
  const float decay = h.adamw ? (1.f - h.lr * h.weight_decay) : 1.f;
  const float l2 = h.adamw ? 0.f : h.weight_decay;
  const float inv_bc2 = 1.f / h.bias_corr2_sqrt;
  const int64_t stride = (int64_t)gridDim.x * kOptThreads * kOptVec;
  for (int64_t i = ((int64_t)blockIdx.x * kOptThreads + threadIdx.x) * kOptVec; i < n; i += stride) {
    if (i + kOptVec <= n) {
      float p[8], g[8], a[8], b[8];
      load8<kF32>(master, i, p);
      load8<GDT>(grad, i, g);
      load8<kF32>(m1, i, a);
      load8<kF32>(m2, i, b);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float gj = g[j] * gs + l2 * p[j];
        a[j] = h.beta1 * a[j] + (1.f - h.beta1) * gj;
        b[j] = h.beta2 * b[j] + (1.f - h.beta2) * gj * gj;
        const float denom = __builtin_sqrtf(b[j]) * inv_bc2 + h.eps;
        p[j] = p[j] * decay - step * a[j] / denom;
      }
      store8<kF32>(master, i, p);
      store8<kF32>(m1, i, a);
      store8<kF32>(m2, i, b);
      if constexpr (MDT >= 0) store8<MDT>(model, i, p);
    } else {
      for (int64_t k = i; k < n; ++k) {
        float pk = master[k];
        float gj = Elem<GDT>::load(static_cast<const typename Elem<GDT>::T*>(grad), k) * gs + l2 * pk;
        float ak = h.beta1 * m1[k] + (1.f - h.beta1) * gj;
        float bk = h.beta2 * m2[k] + (1.f - h.beta2) * gj * gj;
        const float denom = __builtin_sqrtf(bk) * inv_bc2 + h.eps;
        pk = pk * decay - step * ak / denom;
        master[k] = pk; m1[k] = ak; m2[k] = bk;
        if constexpr (MDT >= 0) Elem<MDT>::store(static_cast<typename Elem<MDT>::T*>(model), k, pk);
      }
    }
  }
}

// Stage 1: per-workgroup partial sum of squares (no atomics; the partial slab
// is reduced by stage 2 — MI355X_MICROARCH.md "Global float atomics").
template <int DT>
__global__ __launch_bounds__(256) void sqnorm_partial_kernel(const void* __restrict__ x, int64_t n, float scale,
                                                             float* __restrict__ partial) {
  __shared__ float red[256 / kWave];
  float acc = 0.f;
  const int64_t stride = (int64_t)gridDim.x * 256 * 8;
  for (int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8; i < n; i += stride) {
    if (i + 8 <= n) {
      float v[8];
      load8<DT>(x, i, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += v[j] * v[j];
    } else {
      for (int64_t k = i; k < n; ++k) {
        float v = Elem<DT>::load(static_cast<const typename Elem<DT>::T*>(x), k);
        acc += v * v;
      }
    }
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < 256 / kWave; ++w) s += red[w];
    partial[blockIdx.x] = s * scale * scale;
  }
}

// Stage 2: one workgroup reduces the partials; writes [norm, clip_coef].
__global__ __launch_bounds__(256) void norm_finalize_kernel(const float* __restrict__ partial, int np, float max_norm,
                                                            float* __restrict__ out) {
  __shared__ float red[256 / kWave];
  float acc = 0.f;
  for (int i = threadIdx.x; i < np; i += 256) acc += partial[i];
  acc = wave_sum(acc);
  if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int w = 0; w < 256 / kWave; ++w) s += red[w];
    const float norm = __builtin_sqrtf(s);
    out[0] = norm;
    float coef = 1.f;
    if (max_norm > 0.f) {
      coef = max_norm / (norm + 1e-6f);
      coef = coef < 1.f ? coef : 1.f;
    }
    out[1] = coef;
  }
}

}  // namespace madnn

#define MADNN_DISPATCH_MODEL(mdt, NAME, ...)                                     \
  switch (mdt) {                                                                 \
    case -1: { constexpr int NAME = -1; __VA_ARGS__; break; }                    \
    case ::madnn::kF32: { constexpr int NAME = ::madnn::kF32; __VA_ARGS__; break; } \
    case ::madnn::kBF16: { constexpr int NAME = ::madnn::kBF16; __VA_ARGS__; break; } \
    case ::madnn::kF16: { constexpr int NAME = ::madnn::kF16; __VA_ARGS__; break; } \
    default: return hipErrorInvalidValue;                                        \
  }

// optimizer launch knob (madnn_optim_tune key 0): workgroups per CU of the SGD / Adam passes
static int g_opt_wg = 4;

extern "C" {

int madnn_optim_tune(int key, int value) {
  if (key != 0) return -1;
  const int old = g_opt_wg;
  if (value > 0) g_opt_wg = value;
  return old;
}

hipError_t madnn_sgd_step(float* master, const void* grad, int grad_dt, float* mom, void* model, int model_dt,
                          int64_t n, float lr, float momentum, float dampening, float weight_decay, int nesterov,
                          int first_step, float grad_scale, const float* dscale, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  madnn::SGDHyper h{lr, momentum, dampening, weight_decay, grad_scale, nesterov, first_step};
  const int grid = madnn::stream_grid(n, madnn::kOptThreads * madnn::kOptVec, g_opt_wg * madnn::kNumCU);
  MADNN_DISPATCH_DT(grad_dt, GDT, MADNN_DISPATCH_MODEL(model_dt, MDT, {
    hipLaunchKernelGGL((madnn::sgd_kernel<GDT, MDT>), dim3(grid), dim3(madnn::kOptThreads), 0, stream, master, grad,
                       mom, model, n, h, dscale);
  }));
  return hipGetLastError();
}

hipError_t madnn_adam_step(float* master, const void* grad, int grad_dt, float* m1, float* m2, void* model,
                           int model_dt, int64_t n, float lr, float beta1, float beta2, float eps, float weight_decay,
                           int adamw, float bias_corr1, float bias_corr2_sqrt, float grad_scale, const float* dscale,
                           hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  madnn::AdamHyper h{lr, beta1, beta2, eps, weight_decay, grad_scale, bias_corr1, bias_corr2_sqrt, adamw};
  const int grid = madnn::stream_grid(n, madnn::kOptThreads * madnn::kOptVec, g_opt_wg * madnn::kNumCU);
  MADNN_DISPATCH_DT(grad_dt, GDT, MADNN_DISPATCH_MODEL(model_dt, MDT, {
    hipLaunchKernelGGL((madnn::adam_kernel<GDT, MDT>), dim3(grid), dim3(madnn::kOptThreads), 0, stream, master, grad,
                       m1, m2, model, n, h, dscale);
  }));
  return hipGetLastError();
}

int madnn_sqnorm_grid(int64_t n) { return madnn::stream_grid(n, 256 * 8, 2 * madnn::kNumCU); }

hipError_t madnn_sqnorm_partial(const void* x, int dt, int64_t n, float scale, float* partial, int grid,
                                hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  MADNN_DISPATCH_DT(dt, DT, {
    hipLaunchKernelGGL((madnn::sqnorm_partial_kernel<DT>), dim3(grid), dim3(256), 0, stream, x, n, scale, partial);
  });
  return hipGetLastError();
}

hipError_t madnn_norm_finalize(const float* partial, int np, float max_norm, float* out, hipStream_t stream) {
  hipLaunchKernelGGL(madnn::norm_finalize_kernel, dim3(1), dim3(256), 0, stream, partial, np, max_norm, out);
  return hipGetLastError();
}

}  // extern "C"
