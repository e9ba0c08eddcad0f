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

// K6f — forward and backward in ONE pass (16-bit logits, 16-byte aligned rows, ld <= 8 * CH * 512):
// the workgroup's 512 lanes hold the whole row in registers (CH 16-byte chunks each), reduce max and
// sum-exp across the block (the exponentials replace the logits in the registers, as bf16), then
// write the row's gradient (softmax - onehot) * gscale[0] straight from the registers.  The backward
// pass then reads nothing: one read + one write of the logit matrix in total instead of two reads +
// one write (GPT-2 medium b64: 6.6 GB less HBM traffic per step).
// gscale is 1 / (number of loss rows) at forward time; the upstream gradient is applied by
// xent_rescale_kernel, whose workgroups all exit at once when it is 1 (plain loss.backward()).
constexpr int kXentFusedThreads = 512;

template <int XDT>
__device__ __forceinline__ float h2f(unsigned short u) {
  return XDT == kBF16 ? bf16_to_f32(u) : f16_to_f32(u);
}

// Whole 8-element chunks inside the vocabulary take v_exp_f32 directly (exp2f adds a denormal range
// reduction: the result is < 2^-126 of the row max only where it cannot matter to the sum) and test the
// vocabulary end once per chunk instead of per element (GPT-2 medium b64 step +0.32 %,
// profiles/r4_ab_xent_fast_exp_gpt2m_b64.log); only the chunk that straddles it is tested per element
template <int XDT, int CH>
__global__ __launch_bounds__(kXentFusedThreads) void xent_fused_kernel(const void* __restrict__ logits,
                                                                      const int64_t* __restrict__ targets,
                                                                      XentRows R, const float* __restrict__ gscale,
                                                                      float* __restrict__ loss,
                                                                      void* __restrict__ grad) {
  constexpr int kW = kXentFusedThreads / kWave;
  constexpr float kLog2e = 1.4426950408889634f, kLn2 = 0.6931471805599453f;
  __shared__ float red[2][kW];
  const int64_t lr = blockIdx.x;
  int64_t r = lr;
  bool loss_row = true;
  if (R.seq > 1) {
    const int64_t b = lr / R.seq, p = lr % R.seq;
    loss_row = p < R.seq - 1;
    r = b * (R.seq - 1) + p;
  }
  int64_t tgt = -1;
  bool has = loss_row;
  if (has) {
    tgt = targets[R.seq > 1 ? lr + 1 : lr];
    if (tgt == R.ignore_index || tgt < 0 || tgt >= R.V) has = false;
  }
  const unsigned short* row = static_cast<const unsigned short*>(logits) + lr * R.ld;
  unsigned short* grow = static_cast<unsigned short*>(grad) + lr * R.ld;
  const int nch = (int)(R.ld / 8);
  const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid / kWave;
  if (!has) {  // block-uniform: a zero gradient row
    if (loss_row && tid == 0) loss[r] = 0.f;
    const u16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int c = tid; c < nch; c += kXentFusedThreads) *reinterpret_cast<u16x8*>(grow + 8 * c) = z;
    return;
  }
  u16x8 buf[CH];
#pragma unroll
  for (int k = 0; k < CH; ++k) {
    const int c = tid + k * kXentFusedThreads;
    if (c < nch) buf[k] = *reinterpret_cast<const u16x8*>(row + 8 * c);
  }
  float m = -INFINITY;
#pragma unroll
  for (int k = 0; k < CH; ++k) {
    const int c = tid + k * kXentFusedThreads;
    if (c < nch) {
      if (8 * c + 8 <= R.V) {
#pragma unroll
        for (int j = 0; j < 8; ++j) m = fmaxf(m, h2f<XDT>(buf[k][j]));
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (8 * c + j < R.V) m = fmaxf(m, h2f<XDT>(buf[k][j]));
      }
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, kWave));
  if (lane == 0) red[0][w] = m;
  __syncthreads();
  m = red[0][0];
#pragma unroll
  for (int k = 1; k < kW; ++k) m = fmaxf(m, red[0][k]);
  const float ml = m * kLog2e;  // row max in log2 units
  // e = exp(z - max), summed in fp32; e (bf16) replaces z in the registers, so the gradient pass is
  // one multiply per element (no second exp: the VALU work, not HBM, bounded the first version)
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < CH; ++k) {
    const int c = tid + k * kXentFusedThreads;
    if (c < nch) {
      u16x8 eb;
      if (8 * c + 8 <= R.V) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float e = __builtin_amdgcn_exp2f(fmaf(h2f<XDT>(buf[k][j]), kLog2e, -ml));
          s += e;
          eb[j] = f32_to_bf16(e);
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float e = 8 * c + j < R.V ? exp2f(fmaf(h2f<XDT>(buf[k][j]), kLog2e, -ml)) : 0.f;
          s += e;
          eb[j] = f32_to_bf16(e);
        }
      }
      buf[k] = eb;
    }
  }
  s = wave_sum(s);
  if (lane == 0) red[1][w] = s;
  __syncthreads();
  s = 0.f;
#pragma unroll
  for (int k = 0; k < kW; ++k) s += red[1][k];
  const float l2 = ml + log2f(s);  // log-sum-exp in log2 units
  if (tid == 0) loss[r] = l2 * kLn2 - h2f<XDT>(row[tgt]);
  const float g = gscale[0];
  const float gs = g / s;  // softmax = e / s
#pragma unroll
  for (int k = 0; k < CH; ++k) {
    const int c = tid + k * kXentFusedThreads;
    if (c < nch) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int64_t col = 8 * (int64_t)c + j;
        v[j] = bf16_to_f32(buf[k][j]) * gs - (col == tgt ? g : 0.f);
      }
      store8<XDT>(grow, 8 * (int64_t)c, v);
    }
  }
}

// grad *= g[0] in place; every workgroup returns at once when g[0] == 1.
template <int XDT>
__global__ __launch_bounds__(256) void xent_rescale_kernel(void* __restrict__ grad, int64_t n8,
                                                           const float* __restrict__ g) {
  const float s = g[0];
  if (s == 1.f) return;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    float v[8];
    load8<XDT>(grad, 8 * i, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] *= s;
    store8<XDT>(grad, 8 * i, v);
  }
}

}  // namespace madnn

extern "C" {

// chunks per lane the fused kernel needs for a row of ld 16-bit elements (0 = not supported)
int madnn_xent_fused_chunks(int64_t ld) {
  if (ld % 8) return 0;
  const int64_t nch = ld / 8;
  for (int ch : {4, 8, 16, 32})
    if (nch <= (int64_t)ch * madnn::kXentFusedThreads) return ch;
  return 0;
}

hipError_t madnn_xent_fused(const void* logits, int dt, const int64_t* targets, int64_t n_loss_rows, int64_t seq,
                            int64_t ld, int V, int ignore_index, int64_t n_rows_all, const float* gscale, float* loss,
                            void* grad, hipStream_t stream) {
  if (n_rows_all <= 0) return hipSuccess;
  const int ch = madnn_xent_fused_chunks(ld);
  if (dt == madnn::kF32 || ch == 0 || (reinterpret_cast<uintptr_t>(logits) & 15) ||
      (reinterpret_cast<uintptr_t>(grad) & 15))
    return hipErrorInvalidValue;
  madnn::XentRows R{n_loss_rows, seq, ld, V, ignore_index};
  const dim3 grid((unsigned)n_rows_all), block(madnn::kXentFusedThreads);
#define MADNN_XF(XDT, CH)                                                                                         \
  hipLaunchKernelGGL((madnn::xent_fused_kernel<XDT, CH>), grid, block, 0, stream, logits, targets, R, gscale, loss, \
                     grad)
#define MADNN_XF_CH(XDT)                  \
  switch (ch) {                           \
    case 4: MADNN_XF(XDT, 4); break;      \
    case 8: MADNN_XF(XDT, 8); break;      \
    case 16: MADNN_XF(XDT, 16); break;    \
    default: MADNN_XF(XDT, 32); break;    \
  }
  if (dt == madnn::kBF16) {
    MADNN_XF_CH(madnn::kBF16)
  } else {
    MADNN_XF_CH(madnn::kF16)
  }
#undef MADNN_XF_CH
#undef MADNN_XF
  return hipGetLastError();
}

hipError_t madnn_xent_rescale(void* grad, int dt, int64_t numel, const float* g, hipStream_t stream) {
  if (numel <= 0) return hipSuccess;
  if (numel % 8 || (reinterpret_cast<uintptr_t>(grad) & 15)) return hipErrorInvalidValue;
  const int64_t n8 = numel / 8;
  const int grid = madnn::stream_grid(n8, 256);
  MADNN_DISPATCH_DT(dt, XDT, {
    hipLaunchKernelGGL((madnn::xent_rescale_kernel<XDT>), dim3(grid), dim3(256), 0, stream, grad, n8, g);
  });
  return hipGetLastError();
}

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
