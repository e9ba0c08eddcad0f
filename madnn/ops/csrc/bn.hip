// K5 — fused BatchNorm (+ residual add) (+ ReLU) for channels_last (NHWC)
// activations, training and inference, forward and backward.
//
// Why: on the first MI355X profile of ResNet-50 (profiles/r1_resnet50_dp1_*)
// MIOpen's NHWC bf16 BatchNorm kernels took 35 % of the step and the separate
// ReLU / residual-add / ReLU-backward passes another 24 %.  All of it is
// HBM-bound streaming, so the win is in passes: this file does
//   forward : 1 read for the statistics + 1 read/1 write for
//             y = relu(x*scale + shift + residual)
//   backward: 1 read (dy, x[, res]) for the two channel reductions + 1 read /
//             1 write for dx (and d_residual), the ReLU mask recomputed from x
//             instead of stored.
// Layout: an NHWC tensor is a dense [M = N*H*W, C] matrix.  A lane owns 8
// consecutive channels (16-byte bf16 access), TPR = C/8 lanes cover a row and
// a 256-lane workgroup covers RPI = 256/TPR rows per iteration; grid-stride over
// rows.  Channel sums are reduced across the workgroup's row slots in LDS and
// written as ONE fp32 partial row per workgroup; a finalize kernel reduces the
// partial slab column-parallel in double (no float atomics: MI355X_MICROARCH.md
// "Global float atomics") and produces the per-channel affine coefficients, the
// running-stat update and the num_batches_tracked increment (so no extra host
// launches per layer).
#include <type_traits>

#include "common.h"

namespace madnn {

constexpr int kBnThreads = 256;
constexpr int kFinSlices = 32;   // finalize: 32 channels x 32 partial-row slices per 1024-lane block

struct BnGeom {
  int tpr, rpi;
};

// Run-time tunables of the two elementwise apply passes (round-1 A/B sweeps
// through madnn_bn_tune).
//  reverse: walk the tensor from its far end.  The pass before an apply (statistics /
//    backward reduction, or the conv that produced x) streams the same tensors front to back,
//    so its last ~100-250 MB are still in the 256 MiB Infinity Cache: a back-to-front apply
//    reads those first instead of evicting them on the way (MI355X_MICROARCH.md "Infinity
//    Cache"); the consumer of the apply's output (the next conv) then starts on lines the
//    apply wrote last.
//  wg_per_cu: grid = wg_per_cu x 256 CUs workgroups of 256 lanes.  At <= 8 (32 waves per CU)
//    every workgroup is resident at once, so the whole grid walks the tensor as one front;
//    above 8 the later workgroups only start when the first ones finish, which splits each
//    pass into several interleaved sweeps and spoils the reuse order.
//  hoist: load each lane's per-channel coefficients once per walk when its channels never change
//    (grid stride a multiple of C); 0 reloads them per chunk (A/B)
//  (re-measured at batch 2048 after the coefficient hoisting, profiles/r2_ab_bn_wg*.json: 4 workgroups
//  per CU beat 8 by 1.2 % and 16 lost 0.7 %; against 4, 3 gained 1.6 %, 2 gained 1.3 %, 6 lost 0.7 %;
//  the reverse walk is neutral there, 0.1 %)
struct BnTune {
  int reverse = 1;
  int wg_per_cu = 3;
  int hoist = 1;
  int partials_per_cu = 2;  // reduction passes (statistics, backward sums): workgroups = partial rows per CU
  //                            (ResNet-50 b512, profiles/r4_ab_bn_partials_*: 1 -1.8 %, 4 -0.5 % against 2)
};
inline BnTune& bn_tune() {
  static BnTune t;
  return t;
}
// walk flags passed to the apply kernels: bit 0 reverse, bit 1 no coefficient hoisting (two / four
// chunks per trip were measured slower at every launch shape and removed)
inline int bn_walk_flags() { return (bn_tune().reverse ? 1 : 0) | (bn_tune().hoist ? 0 : 2); }

// grid-stride walk of [0, total) in 8-element lane chunks, forward or back-to-front; c0 tracks
// the channel of the chunk without a 64-bit modulo per step
struct StripeWalk {
  int64_t i, di, n;
  int c0, dc, C;
  __device__ StripeWalk(int64_t total, int C_, bool reverse) : C(C_) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x * 8;
    const int sC = (int)(stride % C);
    const int64_t i0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8;
    n = i0 < total ? (total - 1 - i0) / stride + 1 : 0;
    i = reverse && n > 0 ? i0 + (n - 1) * stride : i0;
    di = reverse ? -stride : stride;
    c0 = (int)(i % C);
    dc = reverse ? C - sC : sC;
  }
  __device__ void next() {
    --n;
    i += di;
    c0 = (c0 + dc >= C) ? c0 + dc - C : c0 + dc;
  }
};

__host__ __device__ inline BnGeom bn_geom(int C) {
  BnGeom g;
  g.tpr = C / 8;
  g.rpi = kBnThreads / g.tpr;
  return g;
}

// partial[blk][0:C] = sum x, partial[blk][C:2C] = sum x^2
template <int XDT>
__global__ __launch_bounds__(kBnThreads) void bn_stats_kernel(const void* __restrict__ x, int64_t M, int C,
                                                               float* __restrict__ partial) {
  extern __shared__ __attribute__((aligned(16))) float slab[];  // [rpi][2][C]
  const BnGeom g = bn_geom(C);
  const int t = threadIdx.x;
  const int cg = t % g.tpr;
  const int rs = t / g.tpr;
  const bool active = rs < g.rpi;
  float s[8], q[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = q[j] = 0.f;
  if (active) {
    const int64_t step = (int64_t)gridDim.x * g.rpi;
    int64_t r = (int64_t)blockIdx.x * g.rpi + rs;
    // 4 rows in flight per lane: memory-level parallelism for the HBM stream
    for (; r + 3 * step < M; r += 4 * step) {
      float v[4][8];
#pragma unroll
      for (int u = 0; u < 4; ++u) load8<XDT>(x, (r + u * step) * C + cg * 8, v[u]);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          s[j] += v[u][j];
          q[j] += v[u][j] * v[u][j];
        }
    }
    for (; r < M; r += step) {
      float v[8];
      load8<XDT>(x, r * C + cg * 8, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s[j] += v[j];
        q[j] += v[j] * v[j];
      }
    }
  }
  if (g.rpi == 1) {
    if (active) {
      store8<kF32>(partial, (int64_t)blockIdx.x * 2 * C + cg * 8, s);
      store8<kF32>(partial, (int64_t)blockIdx.x * 2 * C + C + cg * 8, q);
    }
    return;
  }
  if (active) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      slab[(rs * 2 + 0) * C + cg * 8 + j] = s[j];
      slab[(rs * 2 + 1) * C + cg * 8 + j] = q[j];
    }
  }
  __syncthreads();
  for (int c = t; c < 2 * C; c += kBnThreads) {
    const int which = c / C, ch = c % C;
    float a = 0.f;
    for (int r = 0; r < g.rpi; ++r) a += slab[(r * 2 + which) * C + ch];
    partial[(int64_t)blockIdx.x * 2 * C + c] = a;
  }
}

// Reduce [G][2][C] partials per channel (double), then:
//   mean, invstd -> save_mean/save_invstd
//   scale = w*invstd, shift = b - mean*scale
//   running stats update (unbiased var), nbt += 1
__global__ __launch_bounds__(1024) void bn_stats_finalize_kernel(
    const float* __restrict__ partial, int G, int C, int64_t M, float eps, float momentum,
    const float* __restrict__ w, const float* __restrict__ b, float* __restrict__ save_mean,
    float* __restrict__ save_invstd, float* __restrict__ scale, float* __restrict__ shift,
    float* __restrict__ run_mean, float* __restrict__ run_var, int64_t* __restrict__ nbt) {
  __shared__ double red[2][kFinSlices][33];
  const int lc = threadIdx.x & 31, ls = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + lc;
  double s = 0.0, q = 0.0;
  if (c < C) {
    // independent loads in flight: the slab read is latency-bound, not bandwidth-bound
    float fs[4] = {0.f, 0.f, 0.f, 0.f}, fq[4] = {0.f, 0.f, 0.f, 0.f};
    int k = ls;
    for (; k + 3 * kFinSlices < G; k += 4 * kFinSlices) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        fs[u] = partial[(int64_t)(k + u * kFinSlices) * 2 * C + c];
        fq[u] = partial[(int64_t)(k + u * kFinSlices) * 2 * C + C + c];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        s += fs[u];
        q += fq[u];
      }
    }
    for (; k < G; k += kFinSlices) {
      s += partial[(int64_t)k * 2 * C + c];
      q += partial[(int64_t)k * 2 * C + C + c];
    }
  }
  red[0][ls][lc] = s;
  red[1][ls][lc] = q;
  __syncthreads();
  if (ls == 0 && c < C) {
    s = q = 0.0;
    for (int k = 0; k < kFinSlices; ++k) {
      s += red[0][k][lc];
      q += red[1][k][lc];
    }
    const double mean = s / (double)M;
    double var = q / (double)M - mean * mean;
    if (var < 0.0) var = 0.0;
    const float invstd = (float)(1.0 / sqrt(var + (double)eps));
    save_mean[c] = (float)mean;
    save_invstd[c] = invstd;
    const float wc = w ? w[c] : 1.f, bc = b ? b[c] : 0.f;
    scale[c] = wc * invstd;
    shift[c] = bc - (float)mean * wc * invstd;
    if (run_mean) {
      const double unbiased = M > 1 ? var * (double)M / (double)(M - 1) : var;
      run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * (float)mean;
      run_var[c] = (1.f - momentum) * run_var[c] + momentum * (float)unbiased;
    }
  }
  if (nbt && blockIdx.x == 0 && threadIdx.x == 0) nbt[0] += 1;
}

// eval-mode coefficients from running statistics
__global__ void bn_eval_coef_kernel(int C, float eps, const float* __restrict__ w, const float* __restrict__ b,
                                    const float* __restrict__ run_mean, const float* __restrict__ run_var,
                                    float* __restrict__ scale, float* __restrict__ shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float invstd = 1.f / __builtin_sqrtf(run_var[c] + eps);
  const float wc = w ? w[c] : 1.f, bc = b ? b[c] : 0.f;
  scale[c] = wc * invstd;
  shift[c] = bc - run_mean[c] * wc * invstd;
}

// y = act(x*scale + shift + res)
// RELU && RES: also write the ReLU mask as bits (1 byte per 8 elements), so the
// backward passes need neither the residual nor the affine recompute for it.
// RAFF: the residual is itself a BatchNorm input (ResNet's downsample path): res is read raw and
// normalised in place, res*rscale + rshift, so the downsample BN never materialises its output.
template <int XDT, bool RELU, bool RES, bool RAFF = false>
__global__ __launch_bounds__(256) void bn_apply_kernel(const void* __restrict__ x, const void* __restrict__ res,
                                                       const float* __restrict__ scale,
                                                       const float* __restrict__ shift, void* __restrict__ y,
                                                       unsigned char* __restrict__ mask, int64_t total, int C,
                                                       int reverse, const float* __restrict__ rscale = nullptr,
                                                       const float* __restrict__ rshift = nullptr) {
  static_assert(!RAFF || RES, "a residual BatchNorm needs the residual");
  StripeWalk w(total, C, (reverse & 1) != 0);
  // When the grid stride is a multiple of C (always, for C dividing 256 x 8), every lane keeps its
  // channels for the whole walk: the coefficients are loaded once instead of per chunk (they were
  // 4x the data bytes in vector-memory requests)
  const bool fixed = (reverse & 2) == 0 && (w.dc == 0 || w.dc == C);
  float sc[8], sh[8], rs[8], rh[8];
  auto coef = [&](int c0) {
    load8<kF32>(scale, c0, sc);
    load8<kF32>(shift, c0, sh);
    if constexpr (RAFF) {
      load8<kF32>(rscale, c0, rs);
      load8<kF32>(rshift, c0, rh);
    }
  };
  if (fixed && w.n > 0) coef(w.c0);
  auto body = [&](int64_t i, float (&v)[8], float (&r)[8]) {
    if constexpr (RAFF) {
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] = r[j] * rs[j] + rh[j];
    }
    unsigned bits = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float z = v[j] * sc[j] + sh[j];
      if constexpr (RES) z += r[j];
      if constexpr (RELU) {
        bits |= (z > 0.f ? 1u : 0u) << j;
        z = z > 0.f ? z : 0.f;
      }
      v[j] = z;
    }
    store8<XDT>(y, i, v);
    if constexpr (RELU && RES) {
      if (mask) mask[i >> 3] = (unsigned char)bits;
    }
  };
  for (; w.n > 0; w.next()) {
    const int64_t i = w.i;
    if (!fixed) coef(w.c0);
    float v[8], r[8];
    load8<XDT>(x, i, v);
    if constexpr (RES) load8<XDT>(res, i, r);
    body(i, v, r);
  }
}

// Backward reduction: g = dy * [z > 0] (ReLU mask recomputed from x),
// partial[blk][0:C] = sum g, partial[blk][C:2C] = sum g * x
// MASKED (RELU && residual): the ReLU mask comes from the forward's bit mask;
// plain RELU recomputes it from x (which is read anyway).
// RAFF (residual BatchNorm, see bn_apply_kernel): the residual's raw input r gets its own
// reduction from the same g, partial[blk][2C:3C] = sum g * r, so one pass serves both BNs.
template <int XDT, bool RELU, bool MASKED, bool RAFF = false>
__global__ __launch_bounds__(kBnThreads) void bn_bwd_reduce_kernel(
    const void* __restrict__ dy, const void* __restrict__ x, const unsigned char* __restrict__ mask,
    const float* __restrict__ scale, const float* __restrict__ shift, int64_t M, int C,
    float* __restrict__ partial, const void* __restrict__ rin = nullptr) {
  static_assert(!RAFF || MASKED, "a residual BatchNorm comes with the fused residual + ReLU mask");
  constexpr int NS = RAFF ? 3 : 2;  // sums per channel
  extern __shared__ __attribute__((aligned(16))) float slab[];
  const BnGeom g = bn_geom(C);
  const int t = threadIdx.x;
  const int cg = t % g.tpr;
  const int rs = t / g.tpr;
  const bool active = rs < g.rpi;
  float sg[8], sgx[8], sgr[8], sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) sg[j] = sgx[j] = sgr[j] = 0.f;
  if (active) {
    if constexpr (RELU && !MASKED) {
      load8<kF32>(scale, cg * 8, sc);
      load8<kF32>(shift, cg * 8, sh);
    }
    const int64_t step = (int64_t)gridDim.x * g.rpi;
    int64_t r = (int64_t)blockIdx.x * g.rpi + rs;
    auto body = [&](const float (&dv)[8], const float (&xv)[8], const float (&rv)[8], unsigned bits) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float gj = dv[j];
        if constexpr (RELU) {
          if constexpr (MASKED) {
            gj = ((bits >> j) & 1u) ? gj : 0.f;
          } else {
            const float z = xv[j] * sc[j] + sh[j];
            gj = z > 0.f ? gj : 0.f;
          }
        }
        sg[j] += gj;
        sgx[j] += gj * xv[j];
        if constexpr (RAFF) sgr[j] += gj * rv[j];
      }
    };
    for (; r + step < M; r += 2 * step) {  // 2 rows x (dy, x[, r][, mask]) in flight per lane
      float dv[2][8], xv[2][8], rv[2][8];
      unsigned mb[2] = {0u, 0u};
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        load8<XDT>(dy, (r + u * step) * C + cg * 8, dv[u]);
        load8<XDT>(x, (r + u * step) * C + cg * 8, xv[u]);
        if constexpr (RAFF) load8<XDT>(rin, (r + u * step) * C + cg * 8, rv[u]);
        if constexpr (MASKED) mb[u] = mask[((r + u * step) * C + cg * 8) >> 3];
      }
      body(dv[0], xv[0], rv[0], mb[0]);
      body(dv[1], xv[1], rv[1], mb[1]);
    }
    for (; r < M; r += step) {
      float dv[8], xv[8], rv[8];
      load8<XDT>(dy, r * C + cg * 8, dv);
      load8<XDT>(x, r * C + cg * 8, xv);
      if constexpr (RAFF) load8<XDT>(rin, r * C + cg * 8, rv);
      unsigned mb = 0u;
      if constexpr (MASKED) mb = mask[(r * C + cg * 8) >> 3];
      body(dv, xv, rv, mb);
    }
  }
  if (g.rpi == 1) {
    if (active) {
      store8<kF32>(partial, (int64_t)blockIdx.x * NS * C + cg * 8, sg);
      store8<kF32>(partial, (int64_t)blockIdx.x * NS * C + C + cg * 8, sgx);
      if constexpr (RAFF) store8<kF32>(partial, (int64_t)blockIdx.x * NS * C + 2 * C + cg * 8, sgr);
    }
    return;
  }
  if (active) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      slab[(rs * NS + 0) * C + cg * 8 + j] = sg[j];
      slab[(rs * NS + 1) * C + cg * 8 + j] = sgx[j];
      if constexpr (RAFF) slab[(rs * NS + 2) * C + cg * 8 + j] = sgr[j];
    }
  }
  __syncthreads();
  for (int c = t; c < NS * C; c += kBnThreads) {
    const int which = c / C, ch = c % C;
    float a = 0.f;
    for (int r = 0; r < g.rpi; ++r) a += slab[(r * NS + which) * C + ch];
    partial[(int64_t)blockIdx.x * NS * C + c] = a;
  }
}

// dbeta = sum g ; dgamma = sum g*xhat = invstd*(sum g*x - mean*sum g)
// dx = w*invstd*(g - dbeta/M - xhat*dgamma/M) = A*g + Bc*x + Cc  (per channel)
// partial rows are pstride floats apart; sum g at offset 0, sum g*x at qoff
__global__ __launch_bounds__(1024) void bn_bwd_finalize_kernel(
    const float* __restrict__ partial, int G, int C, int pstride, int qoff, int64_t M, const float* __restrict__ w,
    const float* __restrict__ mean, const float* __restrict__ invstd, float* __restrict__ dw,
    float* __restrict__ db, float* __restrict__ ca, float* __restrict__ cb, float* __restrict__ cc) {
  __shared__ double red[2][kFinSlices][33];
  const int lc = threadIdx.x & 31, ls = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + lc;
  double s = 0.0, q = 0.0;
  if (c < C) {
    // independent loads in flight: the slab read is latency-bound, not bandwidth-bound
    float fs[4] = {0.f, 0.f, 0.f, 0.f}, fq[4] = {0.f, 0.f, 0.f, 0.f};
    int k = ls;
    for (; k + 3 * kFinSlices < G; k += 4 * kFinSlices) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        fs[u] = partial[(int64_t)(k + u * kFinSlices) * pstride + c];
        fq[u] = partial[(int64_t)(k + u * kFinSlices) * pstride + qoff + c];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        s += fs[u];
        q += fq[u];
      }
    }
    for (; k < G; k += kFinSlices) {
      s += partial[(int64_t)k * pstride + c];
      q += partial[(int64_t)k * pstride + qoff + c];
    }
  }
  red[0][ls][lc] = s;
  red[1][ls][lc] = q;
  __syncthreads();
  if (ls == 0 && c < C) {
    s = q = 0.0;
    for (int k = 0; k < kFinSlices; ++k) {
      s += red[0][k][lc];
      q += red[1][k][lc];
    }
    const double mu = mean[c], is = invstd[c];
    const double dbeta = s;
    const double dgamma = is * (q - mu * s);
    if (dw) dw[c] = (float)dgamma;
    if (db) db[c] = (float)dbeta;
    const double wc = w ? w[c] : 1.0;
    const double A = wc * is;
    const double k2 = dbeta / (double)M, k3 = dgamma / (double)M;
    // dx = A*(g - k2 - (x-mu)*is*k3) = A*g - A*is*k3*x + A*(is*k3*mu - k2)
    ca[c] = (float)A;
    cb[c] = (float)(-A * is * k3);
    cc[c] = (float)(A * (is * k3 * mu - k2));
  }
}

// RAFF: dres is the residual BatchNorm's input gradient, rca*g + rcb*r + rcc, instead of g itself
template <int XDT, bool RELU, bool RES, bool RAFF = false>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(
    const void* __restrict__ dy, const void* __restrict__ x, const unsigned char* __restrict__ mask,
    const float* __restrict__ scale, const float* __restrict__ shift, const float* __restrict__ ca,
    const float* __restrict__ cb, const float* __restrict__ cc, void* __restrict__ dx, void* __restrict__ dres,
    int64_t total, int C, int reverse, const void* __restrict__ rin = nullptr,
    const float* __restrict__ rca = nullptr, const float* __restrict__ rcb = nullptr,
    const float* __restrict__ rcc = nullptr) {
  static_assert(!RAFF || (RELU && RES), "a residual BatchNorm comes with the fused residual + ReLU mask");
  StripeWalk w(total, C, (reverse & 1) != 0);
  const bool fixed = (reverse & 2) == 0 && (w.dc == 0 || w.dc == C);  // channels invariant across the walk (see bn_apply_kernel)
  float a[8], b[8], c[8], sc[8], sh[8], ra[8], rb[8], rc[8];
  auto coef = [&](int c0) {
    load8<kF32>(ca, c0, a);
    load8<kF32>(cb, c0, b);
    load8<kF32>(cc, c0, c);
    if constexpr (RELU && !RES) {
      load8<kF32>(scale, c0, sc);
      load8<kF32>(shift, c0, sh);
    }
    if constexpr (RAFF) {
      load8<kF32>(rca, c0, ra);
      load8<kF32>(rcb, c0, rb);
      load8<kF32>(rcc, c0, rc);
    }
  };
  if (fixed && w.n > 0) coef(w.c0);
  auto body = [&](int64_t i, float (&dv)[8], const float (&xv)[8], const float (&rv)[8]) {
    if constexpr (RELU && RES) {
      const unsigned bits = mask[i >> 3];
#pragma unroll
      for (int j = 0; j < 8; ++j) dv[j] = ((bits >> j) & 1u) ? dv[j] : 0.f;
    } else if constexpr (RELU) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float z = xv[j] * sc[j] + sh[j];
        dv[j] = z > 0.f ? dv[j] : 0.f;
      }
    }
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = a[j] * dv[j] + b[j] * xv[j] + c[j];
    store8<XDT>(dx, i, o);
    if constexpr (RAFF) {
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = ra[j] * dv[j] + rb[j] * rv[j] + rc[j];
      store8<XDT>(dres, i, o);
    } else if constexpr (RES) {
      if (dres != nullptr) store8<XDT>(dres, i, dv);  // null: the consumer masks dy itself (resmask)
    }
  };
  for (; w.n > 0; w.next()) {
    const int64_t i = w.i;
    if (!fixed) coef(w.c0);
    float dv[8], xv[8], rv[8];
    load8<XDT>(dy, i, dv);
    load8<XDT>(x, i, xv);
    if constexpr (RAFF) load8<XDT>(rin, i, rv);
    body(i, dv, xv, rv);
  }
}

// Producer epilogues (K13: one row per 256-pixel tile) can hand over 10^4+ partial rows; the
// finalize kernels walk rows with 32 slices per channel and turn latency-bound there.  Above
// kPreMinRows the rows are first folded to kPreS rows by a (C/32) x kPreS grid.
constexpr int kPreS = 64;
constexpr int kPreMinRows = 1024;

__global__ __launch_bounds__(1024) void partial_prereduce_kernel(const float* __restrict__ partial, int G, int C,
                                                                 int pstride, int qoff, float* __restrict__ out) {
  __shared__ float red[2][kFinSlices][33];
  const int lc = threadIdx.x & 31, ls = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + lc;
  const int lo = (int)((int64_t)G * blockIdx.y / gridDim.y), hi = (int)((int64_t)G * (blockIdx.y + 1) / gridDim.y);
  float s = 0.f, q = 0.f;
  if (c < C) {
    for (int k = lo + ls; k < hi; k += kFinSlices) {
      s += partial[(int64_t)k * pstride + c];
      q += partial[(int64_t)k * pstride + qoff + c];
    }
  }
  red[0][ls][lc] = s;
  red[1][ls][lc] = q;
  __syncthreads();
  if (ls == 0 && c < C) {
    s = q = 0.f;
    for (int k = 0; k < kFinSlices; ++k) {
      s += red[0][k][lc];
      q += red[1][k][lc];
    }
    out[((int64_t)blockIdx.y * 2) * C + c] = s;
    out[((int64_t)blockIdx.y * 2 + 1) * C + c] = q;
  }
}

// fold `part` ([G] rows of pstride floats, sums at 0 / qoff) to kPreS rows of [2][C] in `scratch`
// (kPreS * 2 * C floats) when G is large; updates G / pstride / qoff to describe the result
inline const float* prereduce(const float* part, int& G, int C, int& pstride, int& qoff, float* scratch,
                              hipStream_t stream) {
  if (G < kPreMinRows || scratch == nullptr || scratch == part) return part;
  hipLaunchKernelGGL(partial_prereduce_kernel, dim3((C + 31) / 32, kPreS), dim3(32 * kFinSlices), 0, stream, part, G,
                     C, pstride, qoff, scratch);
  G = kPreS;
  pstride = 2 * C;
  qoff = C;
  return scratch;
}

static int bn_grid_rows(int64_t M, int C) {
  const BnGeom g = bn_geom(C);
  const int64_t cap = (int64_t)bn_tune().partials_per_cu * kNumCU;
  int64_t iters = (M + g.rpi - 1) / g.rpi;
  return (int)(iters < cap ? (iters < 1 ? 1 : iters) : cap);
}

}  // namespace madnn

#define MADNN_BN_VARIANT(relu, res, RELU, RES, ...)                              \
  if (relu && res) { constexpr bool RELU = true, RES = true; __VA_ARGS__; }      \
  else if (relu) { constexpr bool RELU = true, RES = false; __VA_ARGS__; }       \
  else if (res) { constexpr bool RELU = false, RES = true; __VA_ARGS__; }        \
  else { constexpr bool RELU = false, RES = false; __VA_ARGS__; }

extern "C" {

// key 0: apply passes walk back to front (0/1), 1: apply workgroups per CU, 2: coefficient hoisting
// (0/1), 4: reduction workgroups (partial rows) per CU; value < 0 only reads.
// Key 4 sizes the partial slabs: change it only between steps (every call sizes its own workspace).
// Returns the old value (-1 for an unknown key).
int madnn_bn_tune(int key, int value) {
  int* f = key == 0   ? &madnn::bn_tune().reverse
           : key == 1 ? &madnn::bn_tune().wg_per_cu
           : key == 2 ? &madnn::bn_tune().hoist
           : key == 4 ? &madnn::bn_tune().partials_per_cu
                      : nullptr;
  if (f == nullptr) return -1;
  const int old = *f;
  if (value >= 0)
    *f = key == 1 ? (value < 1 ? 1 : value)
         : key == 4 ? (value < 1 ? 1 : value > 8 ? 8 : value)
                    : (value != 0);
  return old;
}

int madnn_bn_supported(int C) { return (C % 8 == 0 && C >= 8 && C <= 2048) ? 1 : 0; }

int madnn_bn_partial_rows(int64_t M, int C) { return madnn::bn_grid_rows(M, C); }

// scratch floats the producer-partial paths need to fold many partial rows (prereduce)
int madnn_bn_prereduce_floats(int C) { return madnn::kPreS * 2 * C; }

// Forward. training: compute batch stats (+ running update); else use running stats.
// ext_partial: [ext_rows][2][C] per-channel (sum, sum of squares) of x already produced by
// the kernel that wrote x (K9 conv1x1 epilogue); the statistics pass over x is skipped.
hipError_t madnn_bn_fwd(const void* x, const void* res, void* y, unsigned char* mask, int64_t M, int C, int xdt,
                        int relu, int training, float eps, float momentum, const float* w, const float* b,
                        float* run_mean, float* run_var, int64_t* nbt, float* save_mean, float* save_invstd,
                        float* scale, float* shift, float* workspace, const float* ext_partial, int ext_rows,
                        hipStream_t stream) {
  using namespace madnn;
  if (!madnn_bn_supported(C)) return hipErrorInvalidValue;
  if (M <= 0) return hipSuccess;
  int G = bn_grid_rows(M, C);
  const BnGeom g = bn_geom(C);
  const size_t lds = g.rpi > 1 ? (size_t)g.rpi * 2 * C * sizeof(float) : 0;
  if (training) {
    const float* part = workspace;
    if (ext_partial != nullptr && ext_rows > 0) {
      G = ext_rows;
      int ps = 2 * C, qo = C;
      part = prereduce(ext_partial, G, C, ps, qo, workspace, stream);
    } else {
      MADNN_DISPATCH_DT(xdt, XDT, {
        hipLaunchKernelGGL((bn_stats_kernel<XDT>), dim3(G), dim3(kBnThreads), lds, stream, x, M, C, workspace);
      });
      MADNN_HIP_CHECK(hipGetLastError());
    }
    hipLaunchKernelGGL(bn_stats_finalize_kernel, dim3((C + 31) / 32), dim3(32 * kFinSlices), 0, stream, part, G, C, M, eps,
                       momentum, w, b, save_mean, save_invstd, scale, shift, run_mean, run_var, nbt);
  } else {
    hipLaunchKernelGGL(bn_eval_coef_kernel, dim3((C + 255) / 256), dim3(256), 0, stream, C, eps, w, b, run_mean,
                       run_var, scale, shift);
  }
  MADNN_HIP_CHECK(hipGetLastError());
  const int64_t total = M * C;
  const int grid = stream_grid(total, 256 * 8, bn_tune().wg_per_cu * kNumCU);
  MADNN_DISPATCH_DT(xdt, XDT, MADNN_BN_VARIANT(relu, res != nullptr, RELU, RES, {
    hipLaunchKernelGGL((bn_apply_kernel<XDT, RELU, RES>), dim3(grid), dim3(256), 0, stream, x, res, scale, shift, y,
                       mask, total, C, bn_walk_flags());
  }));
  return hipGetLastError();
}

hipError_t madnn_bn_bwd(const void* dy, const void* x, const unsigned char* mask, int has_res, void* dx, void* dres,
                        int64_t M, int C, int xdt, int relu, const float* w, const float* save_mean,
                        const float* save_invstd, const float* scale, const float* shift, float* dw, float* db,
                        float* coef, float* workspace, hipStream_t stream) {
  using namespace madnn;
  if (!madnn_bn_supported(C)) return hipErrorInvalidValue;
  if (M <= 0) return hipSuccess;
  const int G = bn_grid_rows(M, C);
  const BnGeom g = bn_geom(C);
  const size_t lds = g.rpi > 1 ? (size_t)g.rpi * 2 * C * sizeof(float) : 0;
  if (relu && has_res && mask == nullptr) return hipErrorInvalidValue;
  MADNN_DISPATCH_DT(xdt, XDT, MADNN_BN_VARIANT(relu, has_res, RELU, RES, {
    hipLaunchKernelGGL((bn_bwd_reduce_kernel<XDT, RELU, RELU && RES>), dim3(G), dim3(kBnThreads), lds, stream, dy, x,
                       mask, scale, shift, M, C, workspace);
  }));
  MADNN_HIP_CHECK(hipGetLastError());
  float* ca = coef;
  float* cb = coef + C;
  float* cc = coef + 2 * C;
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 31) / 32), dim3(32 * kFinSlices), 0, stream, workspace, G, C, 2 * C, C, M, w,
                     save_mean, save_invstd, dw, db, ca, cb, cc);
  MADNN_HIP_CHECK(hipGetLastError());
  const int64_t total = M * C;
  const int grid = stream_grid(total, 256 * 8, bn_tune().wg_per_cu * kNumCU);
  MADNN_DISPATCH_DT(xdt, XDT, MADNN_BN_VARIANT(relu, has_res, RELU, RES, {
    hipLaunchKernelGGL((bn_bwd_apply_kernel<XDT, RELU, RES>), dim3(grid), dim3(256), 0, stream, dy, x, mask, scale,
                       shift, ca, cb, cc, dx, dres, total, C, bn_walk_flags());
  }));
  return hipGetLastError();
}


// Training forward of relu(BN(x) + BN_r(r)): ResNet's last bottleneck BatchNorm with the downsample
// path's BatchNorm folded into the same apply pass (bf16 only).  Each BN's statistics come from its
// producer's epilogue (ext_partial*) or a statistics pass; both finalize into their own coefficients
// and running statistics; one pass then writes y and the ReLU bit mask.
hipError_t madnn_bn_fwd_dual(const void* x, const void* r, void* y, unsigned char* mask, int64_t M, int C,
                             float eps, float momentum, const float* w, const float* b, float* run_mean,
                             float* run_var, int64_t* nbt, float* save_mean, float* save_invstd, float* scale,
                             float* shift, const float* ext_partial, int ext_rows, float eps_r, float momentum_r,
                             const float* w_r, const float* b_r, float* run_mean_r, float* run_var_r,
                             int64_t* nbt_r, float* save_mean_r, float* save_invstd_r, float* scale_r,
                             float* shift_r, const float* ext_partial_r, int ext_rows_r, float* workspace,
                             hipStream_t stream) {
  using namespace madnn;
  if (!madnn_bn_supported(C) || mask == nullptr) return hipErrorInvalidValue;
  if (M <= 0) return hipSuccess;
  const BnGeom g = bn_geom(C);
  const size_t lds = g.rpi > 1 ? (size_t)g.rpi * 2 * C * sizeof(float) : 0;
  const void* src[2] = {x, r};
  const float* ext[2] = {ext_partial, ext_partial_r};
  const int erows[2] = {ext_rows, ext_rows_r};
  const float epsv[2] = {eps, eps_r}, mom[2] = {momentum, momentum_r};
  const float* wv[2] = {w, w_r};
  const float* bv[2] = {b, b_r};
  float* rm[2] = {run_mean, run_mean_r};
  float* rv[2] = {run_var, run_var_r};
  int64_t* nb[2] = {nbt, nbt_r};
  float* sm[2] = {save_mean, save_mean_r};
  float* si[2] = {save_invstd, save_invstd_r};
  float* sc[2] = {scale, scale_r};
  float* sh[2] = {shift, shift_r};
  for (int k = 0; k < 2; ++k) {
    const float* part = workspace;
    int G = bn_grid_rows(M, C);
    if (ext[k] != nullptr && erows[k] > 0) {
      G = erows[k];
      int ps = 2 * C, qo = C;
      part = prereduce(ext[k], G, C, ps, qo, workspace, stream);
    } else {
      hipLaunchKernelGGL((bn_stats_kernel<kBF16>), dim3(G), dim3(kBnThreads), lds, stream, src[k], M, C, workspace);
      MADNN_HIP_CHECK(hipGetLastError());
    }
    hipLaunchKernelGGL(bn_stats_finalize_kernel, dim3((C + 31) / 32), dim3(32 * kFinSlices), 0, stream, part, G, C, M,
                       epsv[k], mom[k], wv[k], bv[k], sm[k], si[k], sc[k], sh[k], rm[k], rv[k], nb[k]);
    MADNN_HIP_CHECK(hipGetLastError());
  }
  const int64_t total = M * C;
  const int grid = stream_grid(total, 256 * 8, bn_tune().wg_per_cu * kNumCU);
  hipLaunchKernelGGL((bn_apply_kernel<kBF16, true, true, true>), dim3(grid), dim3(256), 0, stream, x, r, scale, shift,
                     y, mask, total, C, bn_walk_flags(), scale_r, shift_r);
  return hipGetLastError();
}

// Backward of madnn_bn_fwd_dual: one reduction pass (sum g, sum g*x, sum g*r), two finalizes, one
// apply pass writing dx and dr.  workspace: bn_partial_rows(M, C) * 3 * C floats; coef: 6 * C.
hipError_t madnn_bn_bwd_dual(const void* dy, const void* x, const void* r, const unsigned char* mask, void* dx,
                             void* dr, int64_t M, int C, const float* w, const float* save_mean,
                             const float* save_invstd, const float* w_r, const float* save_mean_r,
                             const float* save_invstd_r, float* dw, float* db, float* dw_r, float* db_r, float* coef,
                             float* workspace, hipStream_t stream) {
  using namespace madnn;
  if (!madnn_bn_supported(C) || mask == nullptr) return hipErrorInvalidValue;
  if (M <= 0) return hipSuccess;
  const int G = bn_grid_rows(M, C);
  const BnGeom g = bn_geom(C);
  const size_t lds = g.rpi > 1 ? (size_t)g.rpi * 3 * C * sizeof(float) : 0;
  hipLaunchKernelGGL((bn_bwd_reduce_kernel<kBF16, true, true, true>), dim3(G), dim3(kBnThreads), lds, stream, dy, x,
                     mask, nullptr, nullptr, M, C, workspace, r);
  MADNN_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 31) / 32), dim3(32 * kFinSlices), 0, stream, workspace, G, C,
                     3 * C, C, M, w, save_mean, save_invstd, dw, db, coef, coef + C, coef + 2 * C);
  MADNN_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 31) / 32), dim3(32 * kFinSlices), 0, stream, workspace, G, C,
                     3 * C, 2 * C, M, w_r, save_mean_r, save_invstd_r, dw_r, db_r, coef + 3 * C, coef + 4 * C,
                     coef + 5 * C);
  MADNN_HIP_CHECK(hipGetLastError());
  const int64_t total = M * C;
  const int grid = stream_grid(total, 256 * 8, bn_tune().wg_per_cu * kNumCU);
  hipLaunchKernelGGL((bn_bwd_apply_kernel<kBF16, true, true, true>), dim3(grid), dim3(256), 0, stream, dy, x, mask,
                     nullptr, nullptr, coef, coef + C, coef + 2 * C, dx, dr, total, C, bn_walk_flags(), r,
                     coef + 3 * C, coef + 4 * C, coef + 5 * C);
  return hipGetLastError();
}


// Training statistics + finalize only (see bn_coef in binding.cpp): the apply runs in a consumer.
hipError_t madnn_bn_coef(const void* x, int64_t M, int C, float eps, float momentum, const float* w, const float* b,
                         float* run_mean, float* run_var, int64_t* nbt, float* save_mean, float* save_invstd,
                         float* scale, float* shift, float* workspace, const float* ext_partial, int ext_rows,
                         hipStream_t stream) {
  using namespace madnn;
  if (!madnn_bn_supported(C)) return hipErrorInvalidValue;
  if (M <= 0) return hipSuccess;
  int G = bn_grid_rows(M, C);
  const float* part = workspace;
  if (ext_partial != nullptr && ext_rows > 0) {
    G = ext_rows;
    int ps = 2 * C, qo = C;
    part = prereduce(ext_partial, G, C, ps, qo, workspace, stream);
  } else {
    const BnGeom g = bn_geom(C);
    const size_t lds = g.rpi > 1 ? (size_t)g.rpi * 2 * C * sizeof(float) : 0;
    hipLaunchKernelGGL((bn_stats_kernel<kBF16>), dim3(G), dim3(kBnThreads), lds, stream, x, M, C, workspace);
    MADNN_HIP_CHECK(hipGetLastError());
  }
  hipLaunchKernelGGL(bn_stats_finalize_kernel, dim3((C + 31) / 32), dim3(32 * kFinSlices), 0, stream, part, G, C, M, eps,
                     momentum, w, b, save_mean, save_invstd, scale, shift, run_mean, run_var, nbt);
  return hipGetLastError();
}

// The backward finalize on its own (fused consumers with their own reduction pass: pool.hip)
hipError_t madnn_bn_bwd_finalize(const float* partial, int G, int C, int pstride, int qoff, int64_t M, const float* w,
                                 const float* mean, const float* invstd, float* dw, float* db, float* ca, float* cb,
                                 float* cc, hipStream_t stream) {
  using namespace madnn;
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 31) / 32), dim3(32 * kFinSlices), 0, stream, partial, G, C,
                     pstride, qoff, M, w, mean, invstd, dw, db, ca, cb, cc);
  return hipGetLastError();
}

// BatchNorm(+ReLU) backward whose reduction came from the producer of dy (K13's / K9's data-grad
// epilogue: partial [G][2][C] = (sum g, sum g*x)): finalize + apply only.  coef: 3 * C floats.
// scratch: madnn_bn_prereduce_floats(C) floats
hipError_t madnn_bn_bwd_ext(const void* dy, const void* x, void* dx, int64_t M, int C, int relu, const float* w,
                            const float* save_mean, const float* save_invstd, const float* scale, const float* shift,
                            float* dw, float* db, float* coef, const float* partial, int G, float* scratch,
                            hipStream_t stream) {
  using namespace madnn;
  if (!madnn_bn_supported(C) || partial == nullptr || G <= 0) return hipErrorInvalidValue;
  if (M <= 0) return hipSuccess;
  int ps = 2 * C, qo = C;
  const float* part = prereduce(partial, G, C, ps, qo, scratch, stream);
  MADNN_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 31) / 32), dim3(32 * kFinSlices), 0, stream, part, G, C, ps,
                     qo, M, w, save_mean, save_invstd, dw, db, coef, coef + C, coef + 2 * C);
  MADNN_HIP_CHECK(hipGetLastError());
  const int64_t total = M * C;
  const int grid = stream_grid(total, 256 * 8, bn_tune().wg_per_cu * kNumCU);
  if (relu) {
    hipLaunchKernelGGL((bn_bwd_apply_kernel<kBF16, true, false>), dim3(grid), dim3(256), 0, stream, dy, x, nullptr,
                       scale, shift, coef, coef + C, coef + 2 * C, dx, nullptr, total, C, bn_walk_flags());
  } else {
    hipLaunchKernelGGL((bn_bwd_apply_kernel<kBF16, false, false>), dim3(grid), dim3(256), 0, stream, dy, x, nullptr,
                       scale, shift, coef, coef + C, coef + 2 * C, dx, nullptr, total, C, bn_walk_flags());
  }
  return hipGetLastError();
}
}  // extern "C"
