// K7: NHWC max-pooling forward/backward for gfx950 (the ResNet stem pool).
//
// PyTorch-ROCm's channels_last max_pool2d writes an int64 index per output
// element (4x the output bytes in bf16) and its backward scatters through
// those indices after a full memset of dx.  Here:
//   forward : one lane = one output pixel x 8 channels; the k*k window is read
//             with 16-byte loads, the result written with one 16-byte store and
//             the window position of each max as one byte (8 bytes per lane,
//             one 64-bit store).  Eval-mode forward skips the byte map.
//   backward: gather, not scatter: one lane = one INPUT pixel x 8 channels; it
//             visits the (at most ceil(k/s)^2) output pixels whose windows hold
//             it, and sums dy where the stored byte names its position.  Every
//             dx element is written exactly once: no memset, no atomics.
// Tie-breaking/NaN follow ATen (first max in scan order; NaN wins).
// Index math is 32-bit: the host refuses tensors with >= 2^31 elements.
#include "common.h"

namespace madnn {

template <int XDT>
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(const void* __restrict__ x, void* __restrict__ y,
                                                          uint64_t* __restrict__ arg, int N, int H, int W, int C,
                                                          int Ho, int Wo, int k, int s, int p) {
  const unsigned CG = (unsigned)C >> 3;
  const unsigned total = (unsigned)N * Ho * Wo * CG;
  for (unsigned idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += gridDim.x * blockDim.x) {
    const unsigned cg = idx % CG;
    const unsigned pix = idx / CG;
    const int ow = (int)(pix % (unsigned)Wo);
    const unsigned t = pix / (unsigned)Wo;
    const int oh = (int)(t % (unsigned)Ho);
    const int n = (int)(t / (unsigned)Ho);
    const int h0 = oh * s - p, w0 = ow * s - p;
    const int kh0 = h0 < 0 ? -h0 : 0, kw0 = w0 < 0 ? -w0 : 0;
    const int kh1 = min(k, H - h0), kw1 = min(k, W - w0);
    float best[8];
    unsigned char a[8];
    const unsigned char first = (unsigned char)(kh0 * k + kw0);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      best[j] = -__builtin_inff();
      a[j] = first;
    }
    for (int kh = kh0; kh < kh1; ++kh) {
      const unsigned rowbase = ((unsigned)(n * H + h0 + kh) * W) * C + cg * 8;
      for (int kw = kw0; kw < kw1; ++kw) {
        float v[8];
        load8<XDT>(x, rowbase + (unsigned)(w0 + kw) * C, v);
        const unsigned char pos = (unsigned char)(kh * k + kw);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (v[j] > best[j] || __builtin_isnan(v[j])) {
            best[j] = v[j];
            a[j] = pos;
          }
        }
      }
    }
    store8<XDT>(y, (int64_t)pix * C + cg * 8, best);
    if (arg) {
      uint64_t packed = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) packed |= (uint64_t)a[j] << (8 * j);
      arg[idx] = packed;
    }
  }
}

template <int XDT>
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const void* __restrict__ dy,
                                                          const uint64_t* __restrict__ arg, void* __restrict__ dx,
                                                          int N, int H, int W, int C, int Ho, int Wo, int k, int s,
                                                          int p) {
  const unsigned CG = (unsigned)C >> 3;
  const unsigned total = (unsigned)N * H * W * CG;
  for (unsigned idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += gridDim.x * blockDim.x) {
    const unsigned cg = idx % CG;
    const unsigned pix = idx / CG;
    const int w = (int)(pix % (unsigned)W);
    const unsigned t = pix / (unsigned)W;
    const int h = (int)(t % (unsigned)H);
    const int n = (int)(t / (unsigned)H);
    // output rows/cols whose window [o*s-p, o*s-p+k) contains h / w
    const int nh = h + p - (k - 1), nw = w + p - (k - 1);
    const int oh_lo = nh <= 0 ? 0 : (nh + s - 1) / s;
    const int ow_lo = nw <= 0 ? 0 : (nw + s - 1) / s;
    const int oh_hi = min(Ho - 1, (h + p) / s);
    const int ow_hi = min(Wo - 1, (w + p) / s);
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    for (int oh = oh_lo; oh <= oh_hi; ++oh) {
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        const unsigned oidx = ((unsigned)(n * Ho + oh) * Wo + ow) * CG + cg;
        const uint64_t packed = arg[oidx];
        const unsigned pos = (unsigned)((h - (oh * s - p)) * k + (w - (ow * s - p)));
        float g[8];
        load8<XDT>(dy, (int64_t)oidx * 8, g);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += (((packed >> (8 * j)) & 0xffu) == pos) ? g[j] : 0.f;
      }
    }
    store8<XDT>(dx, (int64_t)idx * 8, acc);
  }
}

// Workgroup ids are dispatched round-robin over the 8 XCDs, each with its own L2.  Adjacent
// output rows share an input row (and adjacent input rows share a dy row in backward), so
// the k3s2 kernels renumber workgroups to give each XCD one contiguous 1/8 of every
// grid-stride sweep: neighbours then hit the same L2 instead of fetching the shared row
// from HBM twice (MI355X_MICROARCH.md "XCD").  Needs gridDim.x % 8 == 0 (host guarantees).
__device__ __forceinline__ unsigned xcd_block_id(int swz) {
  if (!swz) return blockIdx.x;
  return (blockIdx.x % kNumXCD) * (gridDim.x / kNumXCD) + blockIdx.x / kNumXCD;
}

// k = 3, s = 2 (the ResNet stem pool): the generic kernels' data-dependent window loops issue
// one load at a time (9 dependent trips forward, up to 4 backward), so the pass was
// latency-bound at ~3 TB/s.  These variants compute every window address up front and
// issue all loads before the first compare, keeping 9 (forward) / 8 (backward) 16-byte
// loads in flight per lane.  Same scan order, tie-breaking and NaN rule as above.
// BNRELU: x is a raw BatchNorm input; every window element is relu(x * sc[c] + sh[c]) (the stem's
// BN apply + ReLU fused into its max-pool: the normalised stem activation never reaches HBM)
template <int XDT, bool BNRELU = false>
__global__ __launch_bounds__(256) void maxpool_k3s2_fwd_kernel(const void* __restrict__ x, void* __restrict__ y,
                                                               uint64_t* __restrict__ arg, int N, int H, int W,
                                                               int C, int Ho, int Wo, int p, int swz,
                                                               const float* __restrict__ sc = nullptr,
                                                               const float* __restrict__ sh = nullptr) {
  const unsigned CG = (unsigned)C >> 3;
  const unsigned total = (unsigned)N * Ho * Wo * CG;
  for (unsigned idx = xcd_block_id(swz) * blockDim.x + threadIdx.x; idx < total; idx += gridDim.x * blockDim.x) {
    const unsigned cg = idx % CG;
    const unsigned pix = idx / CG;
    const int ow = (int)(pix % (unsigned)Wo);
    const unsigned t = pix / (unsigned)Wo;
    const int oh = (int)(t % (unsigned)Ho);
    const int n = (int)(t / (unsigned)Ho);
    const int h0 = oh * 2 - p, w0 = ow * 2 - p;
    float v[9][8];
    bool ok[9];
    float bs[8], bh[8];
    if constexpr (BNRELU) {
      load8<kF32>(sc, cg * 8, bs);
      load8<kF32>(sh, cg * 8, bh);
    }
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int h = h0 + kh, w = w0 + kw;
        const int q = kh * 3 + kw;
        ok[q] = (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
        if (ok[q]) {
          load8<XDT>(x, ((unsigned)(n * H + h) * W + (unsigned)w) * C + cg * 8, v[q]);
        }
      }
    }
    if constexpr (BNRELU) {
#pragma unroll
      for (int q = 0; q < 9; ++q) {
        if (!ok[q]) continue;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float z = v[q][j] * bs[j] + bh[j];
          v[q][j] = z > 0.f ? z : 0.f;
        }
      }
    }
    float best[8];
    unsigned char a[8];
    unsigned char first = 0;
#pragma unroll
    for (int q = 8; q >= 0; --q)
      if (ok[q]) first = (unsigned char)q;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      best[j] = -__builtin_inff();
      a[j] = first;
    }
#pragma unroll
    for (int q = 0; q < 9; ++q) {
      if (!ok[q]) continue;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (v[q][j] > best[j] || __builtin_isnan(v[q][j])) {
          best[j] = v[q][j];
          a[j] = (unsigned char)q;
        }
      }
    }
    store8<XDT>(y, (int64_t)pix * C + cg * 8, best);
    if (arg) {
      uint64_t packed = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) packed |= (uint64_t)a[j] << (8 * j);
      arg[idx] = packed;
    }
  }
}

template <int XDT>
__global__ __launch_bounds__(256) void maxpool_k3s2_bwd_kernel(const void* __restrict__ dy,
                                                               const uint64_t* __restrict__ arg,
                                                               void* __restrict__ dx, int N, int H, int W, int C,
                                                               int Ho, int Wo, int p, int swz) {
  const unsigned CG = (unsigned)C >> 3;
  const unsigned total = (unsigned)N * H * W * CG;
  for (unsigned idx = xcd_block_id(swz) * blockDim.x + threadIdx.x; idx < total; idx += gridDim.x * blockDim.x) {
    const unsigned cg = idx % CG;
    const unsigned pix = idx / CG;
    const int w = (int)(pix % (unsigned)W);
    const unsigned t = pix / (unsigned)W;
    const int h = (int)(t % (unsigned)H);
    const int n = (int)(t / (unsigned)H);
    // the (at most 2 x 2) output pixels whose window holds (h, w): o in {o1 - 1, o1}, o1 = (h+p)/2
    const int oh1 = (h + p) >> 1, ow1 = (w + p) >> 1;
    uint64_t pk[4];
    float g[4][8];
    unsigned pos[4];
    bool ok[4];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int oh = oh1 - 1 + i, ow = ow1 - 1 + j;
        const int dh = h - (oh * 2 - p), dw = w - (ow * 2 - p);
        const int q = i * 2 + j;
        ok[q] = oh >= 0 && oh < Ho && ow >= 0 && ow < Wo && dh <= 2 && dw <= 2;
        pos[q] = (unsigned)(dh * 3 + dw);
        if (ok[q]) {
          const unsigned oidx = ((unsigned)(n * Ho + oh) * Wo + ow) * CG + cg;
          pk[q] = arg[oidx];
          load8<XDT>(dy, (int64_t)oidx * 8, g[q]);
        }
      }
    }
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (!ok[q]) continue;
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += (((pk[q] >> (8 * j)) & 0xffu) == pos[q]) ? g[q][j] : 0.f;
    }
    store8<XDT>(dx, (int64_t)idx * 8, acc);
  }
}

// Backward of maxpool_k3s2(relu(bn(y))) into the BatchNorm input, without materialising the
// pool's input gradient: each lane gathers d(pool input) for one input pixel x 8 channels exactly
// as maxpool_k3s2_bwd_kernel does, masks it with the ReLU (recomputed from y) and then
//   PHASE 0: accumulates the BN backward sums (sum g, sum g*y) -> one [2][C] partial row per
//            workgroup (the format of bn.hip's backward finalize);
//   PHASE 1: writes dy = ca*g + cb*y + cc (coefficients from that finalize).
// A lane's channel group is fixed across its grid-stride walk: 256 % CG == 0 and the stride is a
// multiple of 256 (host-checked: C / 8 divides 256).
template <int PHASE>
__global__ __launch_bounds__(256) void pool_bn_bwd_kernel(const void* __restrict__ dp, const uint64_t* __restrict__ arg,
                                                          const void* __restrict__ y, const float* __restrict__ sc,
                                                          const float* __restrict__ sh, const float* __restrict__ ca,
                                                          const float* __restrict__ cb, const float* __restrict__ cc,
                                                          void* __restrict__ dy, float* __restrict__ partial, int N,
                                                          int H, int W, int C, int Ho, int Wo, int p) {
  __shared__ float slab[256][17];  // PHASE 0: per-lane (8 sums, 8 sums) + pad
  const unsigned CG = (unsigned)C >> 3;
  const unsigned total = (unsigned)N * H * W * CG;
  const unsigned cg = threadIdx.x % CG;
  float bs[8], bh[8], s0[8], s1[8], k0[8], k1[8], k2[8];
  load8<kF32>(sc, cg * 8, bs);
  load8<kF32>(sh, cg * 8, bh);
  if constexpr (PHASE == 1) {
    load8<kF32>(ca, cg * 8, k0);
    load8<kF32>(cb, cg * 8, k1);
    load8<kF32>(cc, cg * 8, k2);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) s0[j] = s1[j] = 0.f;
  for (unsigned idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += gridDim.x * blockDim.x) {
    const unsigned pix = idx / CG;
    const int w = (int)(pix % (unsigned)W);
    const unsigned t = pix / (unsigned)W;
    const int h = (int)(t % (unsigned)H);
    const int n = (int)(t / (unsigned)H);
    const int oh1 = (h + p) >> 1, ow1 = (w + p) >> 1;
    uint64_t pk[4];
    float g[4][8];
    unsigned pos[4];
    bool ok[4];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int oh = oh1 - 1 + i, ow = ow1 - 1 + j;
        const int dh = h - (oh * 2 - p), dw = w - (ow * 2 - p);
        const int q = i * 2 + j;
        ok[q] = oh >= 0 && oh < Ho && ow >= 0 && ow < Wo && dh <= 2 && dw <= 2;
        pos[q] = (unsigned)(dh * 3 + dw);
        if (ok[q]) {
          const unsigned oidx = ((unsigned)(n * Ho + oh) * Wo + ow) * CG + cg;
          pk[q] = arg[oidx];
          load8<kBF16>(dp, (int64_t)oidx * 8, g[q]);
        }
      }
    }
    float yv[8];
    load8<kBF16>(y, (int64_t)idx * 8, yv);
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (!ok[q]) continue;
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += (((pk[q] >> (8 * j)) & 0xffu) == pos[q]) ? g[q][j] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float z = yv[j] * bs[j] + bh[j];
      acc[j] = z > 0.f ? acc[j] : 0.f;
    }
    if constexpr (PHASE == 0) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s0[j] += acc[j];
        s1[j] += acc[j] * yv[j];
      }
    } else {
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = k0[j] * acc[j] + k1[j] * yv[j] + k2[j];
      store8<kBF16>(dy, (int64_t)idx * 8, o);
    }
  }
  if constexpr (PHASE == 0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      slab[threadIdx.x][j] = s0[j];
      slab[threadIdx.x][8 + j] = s1[j];
    }
    __syncthreads();
    for (int c = threadIdx.x; c < 2 * C; c += blockDim.x) {
      const int which = c / C, ch = c % C, g8 = ch >> 3, e = ch & 7;
      float a = 0.f;
      for (int r = g8; r < 256; r += (int)CG) a += slab[r][which * 8 + e];
      partial[(int64_t)blockIdx.x * 2 * C + c] = a;
    }
  }
}

}  // namespace madnn

using namespace madnn;

// k=3/s=2 routing (A/B runs, profiles/r1_pool_ab.json): 0 generic loops,
// 1 unrolled kernels (default), 2 unrolled kernels with the XCD-contiguous workgroup numbering.
// At the stem shape (batch 512): fwd 389 / 379 / 408 us, bwd 434 / 398 / 398 us; the full
// training step is unchanged within 0.1 % by either, so the pass is not latency- or L2-reuse-
// bound in the way the kernel comments above assumed.
static int g_pool_k3s2 = 1;

extern "C" {

int madnn_maxpool_set_k3s2(int on) {
  const int old = g_pool_k3s2;
  if (on >= 0) g_pool_k3s2 = on;
  return old;
}

int madnn_maxpool_supported(int64_t numel, int C, int k) { return numel < (1ll << 31) && C % 8 == 0 && k * k <= 255; }

hipError_t madnn_maxpool_fwd(const void* x, void* y, void* arg, int N, int H, int W, int C, int Ho, int Wo, int k,
                             int s, int p, int xdt, hipStream_t stream) {
  const int64_t work = (int64_t)N * Ho * Wo * (C / 8);
  const int grid = stream_grid(work, 256, 16 * kNumCU);
  if (k == 3 && s == 2 && p <= 2 && g_pool_k3s2) {
    const int g8 = (grid + kNumXCD - 1) / kNumXCD * kNumXCD;
    MADNN_DISPATCH_DT(xdt, XDT, {
      hipLaunchKernelGGL((maxpool_k3s2_fwd_kernel<XDT>), dim3(g_pool_k3s2 == 2 ? g8 : grid), dim3(256), 0, stream, x, y,
                         static_cast<uint64_t*>(arg), N, H, W, C, Ho, Wo, p,
                         (int)(g_pool_k3s2 == 2));
    });
    return hipGetLastError();
  }
  MADNN_DISPATCH_DT(xdt, XDT, {
    hipLaunchKernelGGL((maxpool_fwd_kernel<XDT>), dim3(grid), dim3(256), 0, stream, x, y,
                       static_cast<uint64_t*>(arg), N, H, W, C, Ho, Wo, k, s, p);
  });
  return hipGetLastError();
}

hipError_t madnn_maxpool_bwd(const void* dy, const void* arg, void* dx, int N, int H, int W, int C, int Ho, int Wo,
                             int k, int s, int p, int xdt, hipStream_t stream) {
  const int64_t work = (int64_t)N * H * W * (C / 8);
  const int grid = stream_grid(work, 256, 16 * kNumCU);
  if (k == 3 && s == 2 && p <= 2 && g_pool_k3s2) {
    const int g8 = (grid + kNumXCD - 1) / kNumXCD * kNumXCD;
    MADNN_DISPATCH_DT(xdt, XDT, {
      hipLaunchKernelGGL((maxpool_k3s2_bwd_kernel<XDT>), dim3(g_pool_k3s2 == 2 ? g8 : grid), dim3(256), 0, stream, dy,
                         static_cast<const uint64_t*>(arg), dx, N, H, W, C, Ho, Wo, p,
                         (int)(g_pool_k3s2 == 2));
    });
    return hipGetLastError();
  }
  MADNN_DISPATCH_DT(xdt, XDT, {
    hipLaunchKernelGGL((maxpool_bwd_kernel<XDT>), dim3(grid), dim3(256), 0, stream, dy,
                       static_cast<const uint64_t*>(arg), dx, N, H, W, C, Ho, Wo, k, s, p);
  });
  return hipGetLastError();
}


// fused stem BN + pool grids, workgroups per CU (A/B knobs, madnn_pool_bn_tune): 0 forward, 1 backward
// reduction, 2 backward apply
static int g_pool_bn_wg[3] = {16, 8, 16};

int madnn_pool_bn_tune(int key, int value) {
  if (key < 0 || key > 2) return -1;
  const int old = g_pool_bn_wg[key];
  if (value > 0) g_pool_bn_wg[key] = value;
  return old;
}

int madnn_pool_bn_supported(int64_t numel, int C) {
  return numel < (1ll << 31) && C % 8 == 0 && C <= 2048 && 256 % (C / 8) == 0;
}

// maxpool_k3s2(relu(y * scale + shift)) (bf16 NHWC): output + 1-byte argmax per element
hipError_t madnn_pool_bn_fwd(const void* x, const float* scale, const float* shift, void* y, void* arg, int N, int H,
                             int W, int C, int Ho, int Wo, int p, hipStream_t stream) {
  if (!madnn_pool_bn_supported((int64_t)N * H * W * C, C) || p > 2) return hipErrorInvalidValue;
  const int64_t work = (int64_t)N * Ho * Wo * (C / 8);
  const int grid = stream_grid(work, 256, g_pool_bn_wg[0] * kNumCU);
  hipLaunchKernelGGL((maxpool_k3s2_fwd_kernel<kBF16, true>), dim3(grid), dim3(256), 0, stream, x, y,
                     static_cast<uint64_t*>(arg), N, H, W, C, Ho, Wo, p, 0, scale, shift);
  return hipGetLastError();
}

hipError_t madnn_bn_bwd_finalize(const float* partial, int G, int C, int pstride, int qoff, int64_t M, const float* w,
                                 const float* mean, const float* invstd, float* dw, float* db, float* ca, float* cb,
                                 float* cc, hipStream_t stream);

// partial rows the fused backward's reduction writes
int madnn_pool_bn_bwd_rows(int64_t pixels, int C) {
  const int64_t work = pixels * (C / 8);
  return stream_grid(work, 256, g_pool_bn_wg[1] * kNumCU);  // gather-latency-bound: 8 workgroups per CU in flight
}

// dy (and the BN weight/bias grads) from the pool output gradient dp: reduction, finalize, apply.
// workspace: madnn_pool_bn_bwd_rows * 2 * C floats; coef: 3 * C floats.
hipError_t madnn_pool_bn_bwd(const void* dp, const void* arg, const void* y, const float* w, const float* mean,
                             const float* invstd, const float* scale, const float* shift, void* dy, float* dw,
                             float* db, float* coef, float* workspace, int N, int H, int W, int C, int Ho, int Wo,
                             int p, hipStream_t stream) {
  if (!madnn_pool_bn_supported((int64_t)N * H * W * C, C) || p > 2) return hipErrorInvalidValue;
  const int64_t pixels = (int64_t)N * H * W;
  const int G = madnn_pool_bn_bwd_rows(pixels, C);
  const uint64_t* a = static_cast<const uint64_t*>(arg);
  hipLaunchKernelGGL((pool_bn_bwd_kernel<0>), dim3(G), dim3(256), 0, stream, dp, a, y, scale, shift, nullptr, nullptr,
                     nullptr, nullptr, workspace, N, H, W, C, Ho, Wo, p);
  MADNN_HIP_CHECK(hipGetLastError());
  MADNN_HIP_CHECK(madnn_bn_bwd_finalize(workspace, G, C, 2 * C, C, pixels, w, mean, invstd, dw, db, coef, coef + C,
                                        coef + 2 * C, stream));
  const int grid = stream_grid(pixels * (C / 8), 256, g_pool_bn_wg[2] * kNumCU);
  hipLaunchKernelGGL((pool_bn_bwd_kernel<1>), dim3(grid), dim3(256), 0, stream, dp, a, y, scale, shift, coef, coef + C,
                     coef + 2 * C, dy, nullptr, N, H, W, C, Ho, Wo, p);
  return hipGetLastError();
}

}  // extern "C"
