// K11: bias gradient of a Linear layer, optionally fused with the tanh-GELU backward.
//
//   plain : db[n]  = sum_m dy[m, n]
//   GELU  : dp     = dy * gelu'(p)   (p = the pre-activation x W^T + b, written out for the GEMMs)
//           db[n]  = sum_m dp[m, n]
//
// Why: on GPT-2 medium (profiles/r1_gpt2m_dp1_k8.md) ATen spent ~30 us per Linear on the
// bias-gradient column sum (97 per step) and ran the GELU backward as its own pass, re-reading
// dp afterwards for c_fc's bias.  Both are HBM streams; here one pass reads dy (and p), writes dp
// and produces the column sums.
// Layout: [M, N] row-major, N % 8 == 0.  A lane owns 8 consecutive columns (16-byte access);
// a 256-lane workgroup covers a strip of min(2048, N) columns (blockIdx.x) in 256/(strip/8)
// row slots and walks rows with 4 in flight per lane; its row slots are summed in LDS into ONE
// fp32 partial row.  A finalize (32 columns x 32 row slices per 1024-lane block) sums the
// partial rows in a fixed order (deterministic, no float atomics) and casts to the bias dtype.
#include "common.h"
#include "gelu.h"

namespace madnn {

constexpr int kBiasLanes = 256;

// 8 elements per lane per access (16-byte loads/stores), U accesses in flight per lane,
// grid-stride over the flat tensor.  HBM-bound: reads x, writes y, nothing else.
template <int DT, int U, int GK>
__global__ __launch_bounds__(256) void gelu_fwd_kernel(const void* __restrict__ x, void* __restrict__ y,
                                                       int64_t n8) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + (U - 1) * stride < n8; i += U * stride) {
    float v[U][8];
#pragma unroll
    for (int u = 0; u < U; ++u) load8<DT>(x, (i + u * stride) * 8, v[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[u][j] = gelu_act<GK>(v[u][j]);
      store8<DT>(y, (i + u * stride) * 8, v[u]);
    }
  }
  for (; i < n8; i += stride) {
    float v[8];
    load8<DT>(x, i * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = gelu_act<GK>(v[j]);
    store8<DT>(y, i * 8, v);
  }
}

// Row slots: a 256-lane workgroup is RPI = 256 / TPR row slots of TPR = min(256, N/8) lanes,
// so narrow layers (N = 1024: TPR 128, 2 rows per step) still run 4 full waves per workgroup.
struct BiasGeom {
  int tpr, rpi, strips;
};
__host__ __device__ inline BiasGeom bias_geom(int N) {
  const int lanes = N / 8;
  const int tpr = lanes < kBiasLanes ? lanes : kBiasLanes;
  return {tpr, kBiasLanes / tpr, (lanes + tpr - 1) / tpr};
}

// U: rows per lane in flight in the main loop (the GELU variant at 2 / 8 measured -0.08 % / -0.54 % on
// the GPT-2 medium step against 4, round 4).  GELU: 0 none, kGeluTanh / kGeluErf (gelu.h)
template <int XDT, int GELU, int U = 4>
__global__ __launch_bounds__(kBiasLanes) void bias_grad_kernel(const void* __restrict__ dy,
                                                               const void* __restrict__ pre, void* __restrict__ dp,
                                                               int64_t M, int N, float* __restrict__ partial) {
  __shared__ __attribute__((aligned(16))) float slab[kBiasLanes * 8];  // [rpi][tpr * 8]
  const BiasGeom g = bias_geom(N);
  const int t = threadIdx.x;
  const int cl = t % g.tpr, rs = t / g.tpr;
  const int col = blockIdx.x * g.tpr * 8 + cl * 8;
  const bool active = rs < g.rpi && col < N;
  float s[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = 0.f;
  if (active) {
    const int64_t step = (int64_t)gridDim.y * g.rpi;
    int64_t r = (int64_t)blockIdx.y * g.rpi + rs;
    for (; r + (U - 1) * step < M; r += U * step) {
      float v[U][8];
#pragma unroll
      for (int u = 0; u < U; ++u) load8<XDT>(dy, (r + u * step) * N + col, v[u]);
      if constexpr (GELU != 0) {
        float p[U][8];
#pragma unroll
        for (int u = 0; u < U; ++u) load8<XDT>(pre, (r + u * step) * N + col, p[u]);
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[u][j] *= gelu_act_grad<GELU>(p[u][j]);
          store8<XDT>(dp, (r + u * step) * N + col, v[u]);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] += v[u][j];
    }
    for (; r < M; r += step) {
      float v[8];
      load8<XDT>(dy, r * N + col, v);
      if constexpr (GELU != 0) {
        float p[8];
        load8<XDT>(pre, r * N + col, p);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] *= gelu_act_grad<GELU>(p[j]);
        store8<XDT>(dp, r * N + col, v);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += v[j];
    }
  }
  if (g.rpi == 1) {
    if (active) store8<kF32>(partial, (int64_t)blockIdx.y * N + col, s);
    return;
  }
  if (rs < g.rpi) {
#pragma unroll
    for (int j = 0; j < 8; ++j) slab[rs * g.tpr * 8 + cl * 8 + j] = s[j];
  }
  __syncthreads();
  const int width = g.tpr * 8;
  for (int c = t; c < width; c += kBiasLanes) {
    const int n = blockIdx.x * width + c;
    if (n >= N) continue;
    float a = 0.f;
    for (int q = 0; q < g.rpi; ++q) a += slab[q * width + c];
    partial[(int64_t)blockIdx.y * N + n] = a;
  }
}

// 32 columns x 32 row slices per 1024-lane block; slices combined in a fixed order
template <int ODT>
__global__ __launch_bounds__(1024) void bias_grad_finalize_kernel(const float* __restrict__ partial, int R, int N,
                                                                  void* __restrict__ db) {
  __shared__ float red[32][33];
  const int c = threadIdx.x % 32, sl = threadIdx.x / 32;
  const int n = blockIdx.x * 32 + c;
  float a = 0.f;
  if (n < N)
    for (int r = sl; r < R; r += 32) a += partial[(int64_t)r * N + n];
  red[sl][c] = a;
  __syncthreads();
  if (sl == 0 && n < N) {
    float tot = 0.f;
    for (int q = 0; q < 32; ++q) tot += red[q][c];
    Elem<ODT>::store(static_cast<typename Elem<ODT>::T*>(db), n, tot);
  }
}

}  // namespace madnn

using namespace madnn;

// partial-row count = wg_per_cu x 256 CUs / strips (A/B knob: madnn_bias_tune).  Measured at
// M = 16384 (profiles/r1_linear_ab.json): the plain column sum is fastest at 1 workgroup per CU
// (N=1024/3072/4096: 11.6/20.2/23.3 us vs 17.4/24.2/28.6 at 4: fewer partial rows to write and
// re-read), the GELU variant, which also writes dp, at 4 (36.4/80.9/92.3 us vs 40.6/135/134 at 1).
// Round 2, GPT-2 medium at 64 x 1024 (M = 65536; profiles/r2_ab_madnn_bias_tune_*.json): the plain sum at
// 2 per CU is 1.0 % faster per step than at 1 (4: +0.8 %); the GELU variant stays at 4 (2: +0.1 %, 8: -0.4 %).
static int g_bias_wg_per_cu[2] = {2, 4};

extern "C" {

int madnn_bias_tune(int gelu, int wg_per_cu) {
  const int old = g_bias_wg_per_cu[gelu ? 1 : 0];
  if (wg_per_cu > 0) g_bias_wg_per_cu[gelu ? 1 : 0] = wg_per_cu;
  return old;
}

int madnn_bias_grad_supported(int64_t M, int N) { return N % 8 == 0 && N > 0 && M > 0; }

// partial rows R: ~wg_per_cu workgroups per CU in total, each walking >= 4 row steps
int madnn_bias_grad_rows(int64_t M, int N, int gelu) {
  const BiasGeom g = bias_geom(N);
  int64_t r = (g_bias_wg_per_cu[gelu ? 1 : 0] * kNumCU + g.strips - 1) / g.strips;
  const int64_t cap = (M + 4 * g.rpi - 1) / (4 * g.rpi);
  if (r > cap) r = cap;
  if (r < 1) r = 1;
  if (r > 4096) r = 4096;
  return (int)r;
}

// GELU forward launch knobs (madnn_gelu_tune): key 0 = workgroups per CU (grid cap), key 1 = 16-byte
// accesses in flight per lane (4, 8 or 16).  Swept at GPT-2 medium's [65536, 4096]
// (bench/stream_tune.py, profiles/r4_stream_tune.json): 1 workgroup per CU with 8 accesses in flight
// 184 us (5.8 TB/s) against 245 us at the former 8 x 4 -- one narrow sweep front through the tensor
// beats many resident waves each walking its own far-apart addresses.
static int g_gelu_wg = 1, g_gelu_unroll = 8;

int madnn_gelu_tune(int key, int value) {
  int* f = key == 0 ? &g_gelu_wg : key == 1 ? &g_gelu_unroll : nullptr;
  if (f == nullptr) return -1;
  const int old = *f;
  if (value > 0) *f = value;
  return old;
}

// kind: kGeluTanh (1) or kGeluErf (2)
hipError_t madnn_gelu_fwd(const void* x, void* y, int64_t n, int dt, int kind, hipStream_t stream) {
  if (kind != kGeluTanh && kind != kGeluErf) return hipErrorInvalidValue;
  if (n % 8) return hipErrorInvalidValue;
  const int64_t n8 = n / 8;
  const int U = g_gelu_unroll >= 16 ? 16 : g_gelu_unroll >= 8 ? 8 : 4;
  int64_t grid = (n8 + U * 256 - 1) / (U * 256);
  const int64_t cap = (int64_t)g_gelu_wg * kNumCU;  // a few waves per CU, grid-stride beyond that
  if (grid > cap) grid = cap;
  if (grid < 1) grid = 1;
#define MADNN_GELU_U(GK)                                                                                     \
  MADNN_DISPATCH_DT(dt, DT, {                                                                                \
    if (U == 16) {                                                                                           \
      hipLaunchKernelGGL((gelu_fwd_kernel<DT, 16, GK>), dim3((unsigned)grid), dim3(256), 0, stream, x, y, n8); \
    } else if (U == 8) {                                                                                     \
      hipLaunchKernelGGL((gelu_fwd_kernel<DT, 8, GK>), dim3((unsigned)grid), dim3(256), 0, stream, x, y, n8);  \
    } else {                                                                                                 \
      hipLaunchKernelGGL((gelu_fwd_kernel<DT, 4, GK>), dim3((unsigned)grid), dim3(256), 0, stream, x, y, n8);  \
    }                                                                                                        \
  })
  if (kind == kGeluErf) {
    MADNN_GELU_U(kGeluErf);
  } else {
    MADNN_GELU_U(kGeluTanh);
  }
#undef MADNN_GELU_U
  return hipGetLastError();
}

// dy, pre, dp: [M, N] of dtype xdt; partial: [R, N] fp32 with R = madnn_bias_grad_rows(M, N, pre != 0);
// db: [N] of odt; kind: the GELU whose backward runs on pre (kGeluTanh / kGeluErf)
hipError_t madnn_bias_grad(const void* dy, const void* pre, void* dp, int64_t M, int N, int xdt, float* partial,
                           void* db, int odt, int kind, hipStream_t stream) {
  if (!madnn_bias_grad_supported(M, N)) return hipErrorInvalidValue;
  if (pre != nullptr && kind != kGeluTanh && kind != kGeluErf) return hipErrorInvalidValue;
  const BiasGeom g = bias_geom(N);
  const int R = madnn_bias_grad_rows(M, N, pre != nullptr);
  const dim3 grid(g.strips, R);
  MADNN_DISPATCH_DT(xdt, XDT, {
    if (pre && kind == kGeluErf) {
      hipLaunchKernelGGL((bias_grad_kernel<XDT, kGeluErf>), grid, dim3(kBiasLanes), 0, stream, dy, pre, dp, M, N,
                         partial);
    } else if (pre) {
      hipLaunchKernelGGL((bias_grad_kernel<XDT, kGeluTanh>), grid, dim3(kBiasLanes), 0, stream, dy, pre, dp, M, N,
                         partial);
    } else {
      hipLaunchKernelGGL((bias_grad_kernel<XDT, 0>), grid, dim3(kBiasLanes), 0, stream, dy, nullptr, nullptr, M, N,
                         partial);
    }
  });
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  MADNN_DISPATCH_DT(odt, ODT, {
    hipLaunchKernelGGL((bias_grad_finalize_kernel<ODT>), dim3((N + 31) / 32), dim3(1024), 0, stream, partial, R, N,
                       db);
  });
  return hipGetLastError();
}

}  // extern "C"
