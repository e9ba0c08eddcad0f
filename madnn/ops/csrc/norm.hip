// K3 — LayerNorm / RMSNorm forward + backward for gfx950 (bf16 or f32 I/O,
// fp32 statistics), with an optional fused residual add.
//
// North-star kernel; the reference has no normalisation layer
// of its own.  Layout decisions for CDNA4:
//  * TPR lanes own one row (TPR = 64 for H <= 1024: one row per wave, the row
//    reduction is a pure wave shuffle; TPR = 128/256 for wider rows, finished
//    through a 16-byte-aligned LDS slab).  Each lane keeps NC x 8 elements of
//    its row in registers, loaded with 16-byte vector accesses, so x is read
//    from HBM exactly once and the variance is an exact two-pass over registers.
//  * Backward accumulates dgamma/dbeta for its columns in registers across the
//    rows of a grid-stride loop, reduces the row groups of the workgroup in
//    LDS, and writes ONE fp32 partial row per workgroup; a second small kernel
//    reduces the partial slab column-parallel.  No float atomics anywhere
//    (MI355X_MICROARCH.md "Global float atomics": contended adds are ~1.3 TB/s
//    chip-wide and non-deterministic).
//  * The XCD swizzle is deliberately absent: there is no inter-block reuse on a
//    row-wise op (cdna_hip_programming.md T1 "Transfer: 0% on LayerNorm").
#include <type_traits>

#include "common.h"

namespace madnn {

constexpr int kNormThreads = 256;
typedef unsigned int nu32x4 __attribute__((ext_vector_type(4)));

template <int TPR>
__device__ __forceinline__ float row_sum(float v, float* red) {
  v = wave_sum(v);
  if constexpr (TPR == kWave) {
    return v;
  } else {
    constexpr int WPR = TPR / kWave;  // waves per row
    const int wid = threadIdx.x / kWave;
    const int lane = threadIdx.x & (kWave - 1);
    __syncthreads();
    if (lane == 0) red[wid] = v;
    __syncthreads();
    const int first = (wid / WPR) * WPR;
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < WPR; ++k) s += red[first + k];
    return s;
  }
}

// 8 elements of a row as loaded (one 16-byte access for bf16/f16, two for f32): the forward
// keeps the NEXT row of its grid-stride loop in flight in these while it reduces the current one
template <int DT>
struct Raw8 {
  static constexpr int N = DT == kF32 ? 2 : 1;
  nu32x4 r[N];
  __device__ __forceinline__ void load(const void* base, int64_t i) {
    const nu32x4* p = DT == kF32 ? reinterpret_cast<const nu32x4*>(static_cast<const float*>(base) + i)
                                : reinterpret_cast<const nu32x4*>(static_cast<const unsigned short*>(base) + i);
#pragma unroll
    for (int k = 0; k < N; ++k) r[k] = p[k];
  }
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int k = 0; k < N; ++k) r[k] = nu32x4{0u, 0u, 0u, 0u};
  }
  __device__ __forceinline__ void unpack(float (&v)[8]) const {
    if constexpr (DT == kF32) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = __uint_as_float(r[j >> 2][j & 3]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const unsigned short h = (unsigned short)(r[0][j >> 1] >> (16 * (j & 1)));
        v[j] = DT == kBF16 ? bf16_to_f32(h) : f16_to_f32(h);
      }
    }
  }
};

// Forward: the weight / bias columns of a lane never change across its grid-stride rows, so they
// are loaded once before the loop (loading them after the row reductions exposed an L2 round trip
// per row), and the next row's x (and residual) loads are issued before the current row's two
// reductions, so every wave keeps a row of loads in flight while it reduces.  (Two rows in flight per
// wave measured +0.05 % on the GPT-2 medium step, round 4: not kept.)
template <int XDT, int WDT, int TPR, int NC>
__global__ __launch_bounds__(kNormThreads) void norm_fwd_kernel(
    const void* __restrict__ x, const void* __restrict__ res, const void* __restrict__ w, const void* __restrict__ b,
    void* __restrict__ y, void* __restrict__ sum_out, float* __restrict__ mean_out, float* __restrict__ rstd_out,
    int64_t rows, int H, float eps, int rms) {
  __shared__ __attribute__((aligned(16))) float red[kNormThreads / kWave];
  constexpr int RPB = kNormThreads / TPR;
  const int sub = threadIdx.x / TPR;
  const int t = threadIdx.x % TPR;
  float wv[NC][8], bv[NC][8];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int col = c * TPR * 8 + t * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) wv[c][j] = bv[c][j] = 0.f;
    if (col < H) {
      load8<WDT>(w, col, wv[c]);
      if (b) load8<WDT>(b, col, bv[c]);
    }
  }
  const int64_t rstep = (int64_t)gridDim.x * RPB;
  Raw8<XDT> nx[NC], nr[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    nx[c].zero();
    nr[c].zero();
  }
  auto fetch = [&](int64_t row) {
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int col = c * TPR * 8 + t * 8;
      if (row < rows && col < H) {
        nx[c].load(x, row * H + col);
        if (res) nr[c].load(res, row * H + col);
      }
    }
  };
  int64_t row0 = (int64_t)blockIdx.x * RPB;
  fetch(row0 + sub);
  while (row0 < rows) {
    const int64_t row = row0 + sub;
    const bool live = row < rows;  // uniform per row group; all lanes still join the LDS reduction
    float v[NC][8];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      nx[c].unpack(v[c]);
      if (res) {
        float r[8];
        nr[c].unpack(r);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] += r[j];
      }
    }
    fetch(row + rstep);  // the next row flies under this row's reductions
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int col = c * TPR * 8 + t * 8;
      if (live && col < H) {
        if (res) store8<XDT>(sum_out, row * H + col, v[c]);
#pragma unroll
        for (int j = 0; j < 8; ++j) s += v[c][j];
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] = 0.f;
      }
    }
    const float inv_h = 1.f / (float)H;
    float mean = 0.f;
    if (!rms) mean = row_sum<TPR>(s, red) * inv_h;
    float q = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int col = c * TPR * 8 + t * 8;
      if (live && col < H) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = v[c][j] - mean;
          q += d * d;
        }
      }
    }
    const float rstd = __builtin_amdgcn_rsqf(row_sum<TPR>(q, red) * inv_h + eps);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int col = c * TPR * 8 + t * 8;
      if (live && col < H) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (v[c][j] - mean) * rstd * wv[c][j] + bv[c][j];
        store8<XDT>(y, row * H + col, o);
      }
    }
    if (live && t == 0) {
      if (mean_out) mean_out[row] = mean;
      rstd_out[row] = rstd;
    }
    row0 += rstep;
  }
}

// dx = rstd * (w*dy - mean(w*dy) - xhat * mean(xhat*w*dy))     (LayerNorm)
// dx = rstd * (w*dy - xhat * mean(xhat*w*dy))                  (RMSNorm)
// partial[blk][0:H] = sum_rows dy*xhat, partial[blk][H:2H] = sum_rows dy
// CS: also partial[blk][2H:3H] = sum_rows dx (the written input gradient, residual included): the
// bias gradient of the Linear that produced this norm's input (the transformer residual stream),
// so that Linear's backward needs no column-sum pass of its own (ops._LinearFn, `_madnn_colsum`).
// The weight is loaded once per lane (its columns never change across the grid-stride rows) and
// the next row's x, dy, residual gradient and statistics are loaded before this row's reductions, so
// their latency hides under them instead of following them.
template <int XDT, int WDT, int TPR, int NC, bool CS>
__global__ __launch_bounds__(kNormThreads) void norm_bwd_kernel(
    const void* __restrict__ dy, const void* __restrict__ x, const void* __restrict__ w,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in, const void* __restrict__ dres,
    void* __restrict__ dx, float* __restrict__ partial, int64_t rows, int H, int rms, int has_bias) {
  constexpr int NS = CS ? 3 : 2;  // column sums per workgroup partial row
  __shared__ __attribute__((aligned(16))) float red[kNormThreads / kWave];
  extern __shared__ __attribute__((aligned(16))) float slab[];  // [RPB][NS][NC*TPR*8] when RPB > 1
  constexpr int RPB = kNormThreads / TPR;
  const int sub = threadIdx.x / TPR;
  const int t = threadIdx.x % TPR;
  float dg[NC][8], db[NC][8], ds[CS ? NC : 1][8];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) dg[c][j] = db[c][j] = 0.f;
  if constexpr (CS) {
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int j = 0; j < 8; ++j) ds[c][j] = 0.f;
  }
  float wk[NC][8];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int col = c * TPR * 8 + t * 8;
    if (col < H) {
      load8<WDT>(w, col, wk[c]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) wk[c][j] = 0.f;
    }
  }

  // the next row's x / dy / residual gradient / statistics are loaded into these before the
  // current row's reductions (as in the forward), so a wave always has a row of loads in flight
  constexpr int NP = NC;
  Raw8<XDT> px[NP], pg[NP], pr[NP];
  float pmean = 0.f, prstd = 0.f;
#pragma unroll
  for (int c = 0; c < NP; ++c) {
    px[c].zero();
    pg[c].zero();
    pr[c].zero();
  }
  const int64_t rstep = (int64_t)gridDim.x * RPB;
  auto fetch = [&](int64_t r) {
    if (r < rows) {
      pmean = rms ? 0.f : mean_in[r];
      prstd = rstd_in[r];
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int col = c * TPR * 8 + t * 8;
      if (r < rows && col < H) {
        px[c].load(x, r * H + col);
        pg[c].load(dy, r * H + col);
        if (dres) pr[c].load(dres, r * H + col);
      }
    }
  };
  fetch((int64_t)blockIdx.x * RPB + sub);
  for (int64_t row0 = (int64_t)blockIdx.x * RPB; row0 < rows; row0 += rstep) {
    const int64_t row = row0 + sub;
    const bool live = row < rows;
    float mean, rstd;
    float xh[NC][8], wdy[NC][8], rv[NC][8];
    float xcur[NP][8], gcur[NP][8];
    mean = live ? pmean : 0.f;
    rstd = live ? prstd : 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      px[c].unpack(xcur[c]);
      pg[c].unpack(gcur[c]);
      if (dres) pr[c].unpack(rv[c]);
    }
    fetch(row + rstep);  // the next row's loads fly under this row's math and reductions
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int col = c * TPR * 8 + t * 8;
      if (live && col < H) {
        float xv[8], gv[8], wv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xv[j] = xcur[c][j];
          gv[j] = gcur[c][j];
          wv[j] = wk[c][j];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xh[c][j] = (xv[j] - mean) * rstd;
          wdy[c][j] = wv[j] * gv[j];
          s1 += xh[c][j] * wdy[c][j];
          s2 += wdy[c][j];
          dg[c][j] += gv[j] * xh[c][j];
          db[c][j] += gv[j];
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) xh[c][j] = wdy[c][j] = 0.f;
      }
    }
    const float inv_h = 1.f / (float)H;
    const float c1 = row_sum<TPR>(s1, red) * inv_h;
    const float c2 = rms ? 0.f : row_sum<TPR>(s2, red) * inv_h;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int col = c * TPR * 8 + t * 8;
      if (live && col < H) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = rstd * (wdy[c][j] - c2 - xh[c][j] * c1);
        if (dres) {
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] += rv[c][j];
        }
        store8<XDT>(dx, row * H + col, o);
        if constexpr (CS) {
          // the sum of what is written (rounded to XDT, as the Linear's own column-sum pass would read it)
#pragma unroll
          for (int j = 0; j < 8; ++j) ds[c][j] += XDT == kBF16 ? bf16_to_f32(f32_to_bf16(o[j])) : o[j];
        }
      }
    }
  }

  // Reduce the RPB row groups of this workgroup, then one partial row out.
  constexpr int W = NC * TPR * 8;
  if constexpr (RPB > 1) {
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int lc = c * TPR * 8 + t * 8 + j;
        slab[(sub * NS + 0) * W + lc] = dg[c][j];
        slab[(sub * NS + 1) * W + lc] = db[c][j];
        if constexpr (CS) slab[(sub * NS + 2) * W + lc] = ds[c][j];
      }
    __syncthreads();
    // each thread finalises a strided set of columns
    for (int lc = threadIdx.x; lc < W; lc += kNormThreads) {
      if (lc >= H) continue;
      float a = 0.f, bb = 0.f, cc = 0.f;
#pragma unroll
      for (int r = 0; r < RPB; ++r) {
        a += slab[(r * NS + 0) * W + lc];
        bb += slab[(r * NS + 1) * W + lc];
        if constexpr (CS) cc += slab[(r * NS + 2) * W + lc];
      }
      partial[(int64_t)blockIdx.x * NS * H + lc] = a;
      if (has_bias) partial[(int64_t)blockIdx.x * NS * H + H + lc] = bb;
      if constexpr (CS) partial[(int64_t)blockIdx.x * NS * H + 2 * H + lc] = cc;
    }
  } else {
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int col = c * TPR * 8 + t * 8;
      if (col < H) {
        store8<kF32>(partial, (int64_t)blockIdx.x * NS * H + col, dg[c]);
        if (has_bias) store8<kF32>(partial, (int64_t)blockIdx.x * NS * H + H + col, db[c]);
        if constexpr (CS) store8<kF32>(partial, (int64_t)blockIdx.x * NS * H + 2 * H + col, ds[c]);
      }
    }
  }
}

// Column-parallel reduction of the [G][2H] partial slab: block = 32 columns x
// 32 row-slices (1024 lanes), 4 independent loads in flight per lane — the slab
// read is latency-bound, not bandwidth-bound.
constexpr int kWgSlices = 32;

template <int WDT>
__global__ __launch_bounds__(1024) void norm_wgrad_finalize_kernel(const float* __restrict__ partial, int G, int H,
                                                                   int has_bias, void* __restrict__ dw,
                                                                   void* __restrict__ dbias, int ns,
                                                                   void* __restrict__ dsum, int dsum_bf16) {
  __shared__ float red[kWgSlices][33];
  const int lc = threadIdx.x & 31;
  const int ls = threadIdx.x >> 5;
  const int col2 = blockIdx.x * 32 + lc;  // column in [0, ns*H)
  const int64_t pitch = (int64_t)ns * H;
  float acc = 0.f;
  if (col2 < ns * H) {
    float a[4] = {0.f, 0.f, 0.f, 0.f};
    int g = ls;
    for (; g + 3 * kWgSlices < G; g += 4 * kWgSlices) {
#pragma unroll
      for (int u = 0; u < 4; ++u) a[u] += partial[(int64_t)(g + u * kWgSlices) * pitch + col2];
    }
    for (; g < G; g += kWgSlices) a[0] += partial[(int64_t)g * pitch + col2];
    acc = (a[0] + a[1]) + (a[2] + a[3]);
  }
  red[ls][lc] = acc;
  __syncthreads();
  if (ls == 0 && col2 < ns * H) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < kWgSlices; ++k) s += red[k][lc];
    if (col2 < H) Elem<WDT>::store(static_cast<typename Elem<WDT>::T*>(dw), col2, s);
    else if (col2 < 2 * H) {
      if (has_bias) Elem<WDT>::store(static_cast<typename Elem<WDT>::T*>(dbias), col2 - H, s);
    } else {
      if (dsum_bf16) {
        static_cast<uint16_t*>(dsum)[col2 - 2 * H] = f32_to_bf16(s);
      } else {
        static_cast<float*>(dsum)[col2 - 2 * H] = s;
      }
    }
  }
}

struct NormCfg { int tpr, nc; };
static NormCfg pick_cfg(int H) {
  if (H <= 512) return {64, 1};
  if (H <= 1024) return {64, 2};
  if (H <= 2048) return {128, 2};
  if (H <= 4096) return {256, 2};
  if (H <= 8192) return {256, 4};
  return {256, 8};  // <= 16384
}

#define MADNN_NORM_CFG(H, TPR, NC, ...)                                          \
  do {                                                                           \
    NormCfg _c = pick_cfg(H);                                                    \
    if (_c.tpr == 64 && _c.nc == 1) { constexpr int TPR = 64, NC = 1; __VA_ARGS__; } \
    else if (_c.tpr == 64 && _c.nc == 2) { constexpr int TPR = 64, NC = 2; __VA_ARGS__; } \
    else if (_c.tpr == 128) { constexpr int TPR = 128, NC = 2; __VA_ARGS__; }  \
    else if (_c.nc == 2) { constexpr int TPR = 256, NC = 2; __VA_ARGS__; }      \
    else if (_c.nc == 4) { constexpr int TPR = 256, NC = 4; __VA_ARGS__; }      \
    else { constexpr int TPR = 256, NC = 8; __VA_ARGS__; }                       \
  } while (0)

#define MADNN_DISPATCH_XW(xdt, wdt, XDT, WDT, ...)                               \
  if (xdt == kF32 && wdt == kF32) { constexpr int XDT = kF32, WDT = kF32; __VA_ARGS__; } \
  else if (xdt == kBF16 && wdt == kBF16) { constexpr int XDT = kBF16, WDT = kBF16; __VA_ARGS__; } \
  else if (xdt == kBF16 && wdt == kF32) { constexpr int XDT = kBF16, WDT = kF32; __VA_ARGS__; } \
  else if (xdt == kF32 && wdt == kBF16) { constexpr int XDT = kF32, WDT = kBF16; __VA_ARGS__; } \
  else return hipErrorInvalidValue;

}  // namespace madnn

// launch grids (A/B knobs, madnn_norm_tune): forward workgroups per CU (grid-stride over rows beyond),
// backward workgroups per CU (each writes one dgamma/dbeta partial row).  GPT-2 medium A/B at 64 x 1024
// (profiles/r2_ab_madnn_norm_tune_*.json): backward 4 per CU +0.9 % over 2 (8: +0.7 %).  Forward at the
// b128 shapes (bench/norm_probe.py, round 5; 98 VGPRs = 5 waves per SIMD resident): 32 per CU 103 us
// against 8 per CU 113 us at 131072 x 1024 (5.2 vs 4.8 TB/s), 48.5 vs 51.0 us at 65536 x 1024
static int g_norm_fwd_wg = 32, g_norm_bwd_wg = 4;

extern "C" {

int madnn_norm_tune(int key, int value) {
  int* f = key == 0 ? &g_norm_fwd_wg : key == 1 ? &g_norm_bwd_wg : nullptr;
  if (f == nullptr) return -1;
  const int old = *f;
  if (value > 0) *f = value;
  return old;
}

int madnn_norm_max_h() { return 16384; }

hipError_t madnn_norm_fwd(const void* x, const void* res, const void* w, const void* b, void* y, void* sum_out,
                          float* mean_out, float* rstd_out, int64_t rows, int H, float eps, int rms, int xdt, int wdt,
                          hipStream_t stream) {
  using namespace madnn;
  if (rows <= 0) return hipSuccess;
  if (H % 8 != 0 || H > 16384) return hipErrorInvalidValue;
  MADNN_DISPATCH_XW(xdt, wdt, XDT, WDT, {
    MADNN_NORM_CFG(H, TPR, NC, {
      constexpr int RPB = kNormThreads / TPR;
      int64_t blocks = (rows + RPB - 1) / RPB;
      const int grid = blocks > g_norm_fwd_wg * kNumCU ? g_norm_fwd_wg * kNumCU : (int)blocks;
      hipLaunchKernelGGL((norm_fwd_kernel<XDT, WDT, TPR, NC>), dim3(grid), dim3(kNormThreads), 0, stream, x, res, w,
                         b, y, sum_out, mean_out, rstd_out, rows, H, eps, rms);
    });
  });
  return hipGetLastError();
}

// Workspace size (floats) the backward needs for its dgamma/dbeta (/ dx column-sum) partials.
static int64_t norm_bwd_groups(int64_t rows, int H) {
  using namespace madnn;
  NormCfg c = pick_cfg(H);
  const int RPB = kNormThreads / c.tpr;
  int64_t blocks = (rows + RPB - 1) / RPB;
  int64_t G = blocks < (int64_t)g_norm_bwd_wg * kNumCU ? blocks : (int64_t)g_norm_bwd_wg * kNumCU;
  return G < 1 ? 1 : G;
}

int64_t madnn_norm_bwd_workspace(int64_t rows, int H) { return norm_bwd_groups(rows, H) * 3 * (int64_t)H; }

// dsum (optional, [H], bf16 if dsum_bf16 else fp32): column sums of dx over the rows (norm_bwd_kernel CS)
hipError_t madnn_norm_bwd(const void* dy, const void* x, const void* w, const float* mean_in, const float* rstd_in,
                          const void* dres, void* dx, void* dw, void* dbias, void* dsum, int dsum_bf16, float* workspace,
                          int64_t rows, int H, int rms, int xdt, int wdt, hipStream_t stream) {
  using namespace madnn;
  if (rows <= 0) return hipSuccess;
  if (H % 8 != 0 || H > 16384) return hipErrorInvalidValue;
  const int has_bias = dbias != nullptr;
  const int G = (int)norm_bwd_groups(rows, H);
  const int ns = dsum != nullptr ? 3 : 2;
  MADNN_DISPATCH_XW(xdt, wdt, XDT, WDT, {
    MADNN_NORM_CFG(H, TPR, NC, {
      constexpr int RPB = kNormThreads / TPR;
      const size_t lds = RPB > 1 ? (size_t)RPB * ns * NC * TPR * 8 * sizeof(float) : 0;
      if (dsum != nullptr) {
        hipLaunchKernelGGL((norm_bwd_kernel<XDT, WDT, TPR, NC, true>), dim3(G), dim3(kNormThreads), lds, stream,
                           dy, x, w, mean_in, rstd_in, dres, dx, workspace, rows, H, rms, has_bias);
      } else {
        hipLaunchKernelGGL((norm_bwd_kernel<XDT, WDT, TPR, NC, false>), dim3(G), dim3(kNormThreads), lds, stream,
                           dy, x, w, mean_in, rstd_in, dres, dx, workspace, rows, H, rms, has_bias);
      }
      MADNN_HIP_CHECK(hipGetLastError());
      const int fgrid = ((dsum != nullptr ? 3 * H : (has_bias ? 2 * H : H)) + 31) / 32;
      hipLaunchKernelGGL((norm_wgrad_finalize_kernel<WDT>), dim3(fgrid), dim3(32 * kWgSlices), 0, stream, workspace, G, H,
                         has_bias, dw, dbias, ns, dsum, dsum_bf16);
    });
  });
  return hipGetLastError();
}

}  // extern "C"
