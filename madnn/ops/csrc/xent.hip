// K6 — fused softmax cross-entropy for language-model heads (bf16 logits).
//
// The eager path for a [N, V] bf16 logit matrix (GPT-2: N = 16k tokens,
// V = 50257; Llama-3: V = 128256) materialises an fp32 copy, a log-softmax,
// and in backward a softmax-backward plus casts: ~25 GB of HBM traffic per
// step on the GPT-2-medium config (profiles/r1_gpt2m_*).  Here:
//   forward : ONE read of the logits; a workgroup owns a row, every lane keeps
//             an online (max, sum-exp) pair over its 16-byte chunks, pairs are
//             merged by wave shuffles then across the 4 waves in LDS; writes
//             per-row loss and log-sum-exp (fp32).
//   backward: ONE read + ONE write: grad = (exp(z - lse) - onehot) * g_row,
//             zero for ignored rows, for padded vocabulary columns and (causal
//             shift) for the last position of every sequence — so the caller
//             never slices/pads the logit matrix.
// Rows need not be 16-byte aligned (V = 50257 is odd): each lane walks an
// aligned vector body with a scalar head/tail.
#include "common.h"

namespace madnn {

constexpr int kXentThreads = 256;

struct XentRows {
  int64_t n_loss_rows;  // rows that carry a loss term
  int64_t seq;          // shift mode: sequence length S (loss row r -> logit row r + r/(S-1)); 0 = no shift
  int64_t ld;           // row stride of the logit matrix (>= V, padded vocab allowed)
  int V;                // valid vocabulary columns
  int ignore_index;
};

__device__ __forceinline__ int64_t logit_row_of(int64_t r, int64_t seq) {
  return seq > 1 ? r + r / (seq - 1) : r;
}

__device__ __forceinline__ void merge(float& m, float& s, float m2, float s2) {
  const float mm = fmaxf(m, m2);
  s = (m == -INFINITY ? 0.f : s * __expf(m - mm)) + (m2 == -INFINITY ? 0.f : s2 * __expf(m2 - mm));
  m = mm;
}

template <int XDT>
__global__ __launch_bounds__(kXentThreads) void xent_fwd_kernel(const void* __restrict__ logits,
                                                                const int64_t* __restrict__ targets, XentRows R,
                                                                float* __restrict__ loss, float* __restrict__ lse) {
  __shared__ float sm[kXentThreads / kWave], ss[kXentThreads / kWave];
  const int64_t r = blockIdx.x;
  if (r >= R.n_loss_rows) return;
  const int64_t lr = logit_row_of(r, R.seq);
  const int64_t tgt = targets[R.seq > 1 ? lr + 1 : lr];
  using E = Elem<XDT>;
  const typename E::T* row = static_cast<const typename E::T*>(logits) + lr * R.ld;
  // aligned body [h, h + nv*8)
  const int esz = sizeof(typename E::T);
  const uintptr_t a = reinterpret_cast<uintptr_t>(row);
  int h = (int)(((16 - (a & 15)) & 15) / esz);
  if (h > R.V) h = R.V;
  const int nv = (R.V - h) / 8;
  float m = -INFINITY, s = 0.f;
  for (int i = threadIdx.x; i < h; i += kXentThreads) merge(m, s, E::load(row, i), 1.f);
  for (int i = threadIdx.x; i < nv; i += kXentThreads) {
    float v[8];
    load8<XDT>(row, h + i * 8, v);
    float lm = v[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) lm = fmaxf(lm, v[j]);
    float ls = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) ls += __expf(v[j] - lm);
    merge(m, s, lm, ls);
  }
  for (int i = h + nv * 8 + threadIdx.x; i < R.V; i += kXentThreads) merge(m, s, E::load(row, i), 1.f);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float m2 = __shfl_xor(m, off, kWave), s2 = __shfl_xor(s, off, kWave);
    merge(m, s, m2, s2);
  }
  const int w = threadIdx.x / kWave;
  if ((threadIdx.x & (kWave - 1)) == 0) {
    sm[w] = m;
    ss[w] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = sm[0], S = ss[0];
    for (int k = 1; k < kXentThreads / kWave; ++k) merge(M, S, sm[k], ss[k]);
    const float l = M + __logf(S);
    lse[r] = l;
    loss[r] = (tgt == R.ignore_index || tgt < 0 || tgt >= R.V) ? 0.f : l - E::load(row, tgt);
  }
}

// grad over ALL rows of the logit matrix (n_rows_all x ld).
template <int XDT>
__global__ __launch_bounds__(kXentThreads) void xent_bwd_kernel(const void* __restrict__ logits,
                                                                const int64_t* __restrict__ targets,
                                                                const float* __restrict__ lse, XentRows R,
                                                                int64_t n_rows_all, const float* __restrict__ gscale,
                                                                void* __restrict__ grad) {
  const int64_t lr = blockIdx.x;
  if (lr >= n_rows_all) return;
  using E = Elem<XDT>;
  // which loss row (if any) owns this logit row
  int64_t r = lr;
  bool has = true;
  if (R.seq > 1) {
    const int64_t b = lr / R.seq, p = lr % R.seq;
    has = p < R.seq - 1;
    r = b * (R.seq - 1) + p;
  }
  int64_t tgt = -1;
  float g = 0.f, l = 0.f;
  if (has) {
    tgt = targets[R.seq > 1 ? lr + 1 : lr];
    if (tgt == R.ignore_index || tgt < 0 || tgt >= R.V) has = false;
    else {
      g = gscale[0];
      l = lse[r];
    }
  }
  const typename E::T* row = static_cast<const typename E::T*>(logits) + lr * R.ld;
  typename E::T* grow = static_cast<typename E::T*>(grad) + lr * R.ld;
  const int esz = sizeof(typename E::T);
  const uintptr_t a = reinterpret_cast<uintptr_t>(row);
  int h = (int)(((16 - (a & 15)) & 15) / esz);
  if (h > R.ld) h = (int)R.ld;
  const int nv = (int)((R.ld - h) / 8);
  auto val = [&](int64_t j, float z) -> float {
    if (!has || j >= R.V) return 0.f;
    return (__expf(z - l) - (j == tgt ? 1.f : 0.f)) * g;
  };
  for (int i = threadIdx.x; i < h; i += kXentThreads) E::store(grow, i, val(i, E::load(row, i)));
  for (int i = threadIdx.x; i < nv; i += kXentThreads) {
    const int64_t j0 = h + (int64_t)i * 8;
    float v[8];
    if (has) load8<XDT>(row, j0, v);
    else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = 0.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = val(j0 + j, v[j]);
    store8<XDT>(grow, j0, v);
  }
  for (int64_t i = h + (int64_t)nv * 8 + threadIdx.x; i < R.ld; i += kXentThreads)
    E::store(grow, i, val(i, E::load(row, i)));
}

}  // namespace madnn

extern "C" {

hipError_t madnn_xent_fwd(const void* logits, int dt, const int64_t* targets, int64_t n_loss_rows, int64_t seq,
                          int64_t ld, int V, int ignore_index, float* loss, float* lse, hipStream_t stream) {
  if (n_loss_rows <= 0) return hipSuccess;
  madnn::XentRows R{n_loss_rows, seq, ld, V, ignore_index};
  MADNN_DISPATCH_DT(dt, XDT, {
    hipLaunchKernelGGL((madnn::xent_fwd_kernel<XDT>), dim3((unsigned)n_loss_rows), dim3(madnn::kXentThreads), 0,
                       stream, logits, targets, R, loss, lse);
  });
  return hipGetLastError();
}

hipError_t madnn_xent_bwd(const void* logits, int dt, const int64_t* targets, const float* lse, int64_t n_loss_rows,
                          int64_t seq, int64_t ld, int V, int ignore_index, int64_t n_rows_all, const float* gscale,
                          void* grad, hipStream_t stream) {
  if (n_rows_all <= 0) return hipSuccess;
  madnn::XentRows R{n_loss_rows, seq, ld, V, ignore_index};
  MADNN_DISPATCH_DT(dt, XDT, {
    hipLaunchKernelGGL((madnn::xent_bwd_kernel<XDT>), dim3((unsigned)n_rows_all), dim3(madnn::kXentThreads), 0,
                       stream, logits, targets, lse, R, n_rows_all, gscale, grad);
  });
  return hipGetLastError();
}

}  // extern "C"
