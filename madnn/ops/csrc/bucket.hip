// K4 — multi-tensor bucket flatten (pack) / unflatten (unpack) with fused
// scale and dtype cast, plus a flat scale/cast kernel.
//
// Replaces the reference's per-tensor synchronisation loop
// (reference datamodule.lua:211-224: one allreduceTensor + div(W) per
// parameter and per gradient) and Torch7 getParameters() flattening
// (cifar_example/sgd-torchad_nn-cifar.lua:109) with ONE launch per bucket.
//
// Design (gfx950):
//  * the tensor table travels in the kernel-argument segment (<= 4 KB), so a
//    launch needs no H2D copy and can be captured in a hipGraph;
//  * one workgroup = one 2048-element chunk of one tensor (256 lanes x 8
//    elements, 16-byte vector accesses); a wave-uniform binary search over the
//    per-tensor chunk prefix maps blockIdx -> tensor (SGPR-only);
//  * grid = total chunks (>> 256 CUs for any real bucket); scale by 1/W and the
//    dtype cast are fused into the copy, so averaging costs no extra pass.
#include "common.h"

namespace madnn {

constexpr int kMaxTensors = 48;
constexpr int kPackThreads = 256;
constexpr int kPackChunk = kPackThreads * 8;

struct TensorTable {
  void* ptr[kMaxTensors];           // per-tensor base pointer (src for pack, dst for unpack)
  int64_t off[kMaxTensors];         // element offset inside the flat buffer
  int64_t numel[kMaxTensors];
  int32_t chunk_start[kMaxTensors + 1];
  int32_t vec_ok[kMaxTensors];      // 16-byte aligned on both sides
  int32_t n;
};

template <int TDT, int FDT, bool PACK>
__global__ __launch_bounds__(kPackThreads) void bucket_copy_kernel(TensorTable tab, void* flat, float scale) {
  const int b = blockIdx.x;
  int lo = 0, hi = tab.n - 1;
  while (lo < hi) {  // wave-uniform
    int mid = (lo + hi + 1) >> 1;
    if (tab.chunk_start[mid] <= b) lo = mid; else hi = mid - 1;
  }
  const int t = lo;
  const int64_t n = tab.numel[t];
  const int64_t i = (int64_t)(b - tab.chunk_start[t]) * kPackChunk + threadIdx.x * 8;
  if (i >= n) return;
  void* tp = tab.ptr[t];
  const int64_t fo = tab.off[t];
  using TE = Elem<TDT>;
  using FE = Elem<FDT>;
  if (tab.vec_ok[t] && i + 8 <= n) {
    float v[8];
    if constexpr (PACK) {
      load8<TDT>(tp, i, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] *= scale;
      store8<FDT>(flat, fo + i, v);
    } else {
      load8<FDT>(flat, fo + i, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] *= scale;
      store8<TDT>(tp, i, v);
    }
  } else {
    for (int j = 0; j < 8 && i + j < n; ++j) {
      if constexpr (PACK) {
        float x = TE::load(static_cast<const typename TE::T*>(tp), i + j) * scale;
        FE::store(static_cast<typename FE::T*>(flat), fo + i + j, x);
      } else {
        float x = FE::load(static_cast<const typename FE::T*>(flat), fo + i + j) * scale;
        TE::store(static_cast<typename TE::T*>(tp), i + j, x);
      }
    }
  }
}

template <int SDT, int DDT>
__global__ __launch_bounds__(256) void flat_scale_cast_kernel(const void* __restrict__ src, void* __restrict__ dst,
                                                              int64_t n, float scale) {
  using SE = Elem<SDT>;
  using DE = Elem<DDT>;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * 8;
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8; i < n; i += stride) {
    if (i + 8 <= n) {
      float v[8];
      load8<SDT>(src, i, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] *= scale;
      store8<DDT>(dst, i, v);
    } else {
      for (int64_t j = i; j < n; ++j)
        DE::store(static_cast<typename DE::T*>(dst), j, SE::load(static_cast<const typename SE::T*>(src), j) * scale);
    }
  }
}

static int dt_size(int dt) { return dt == kF32 ? 4 : 2; }

// Host launcher: splits arbitrary tensor lists into <=kMaxTensors launches.
static hipError_t bucket_copy(bool pack, void* const* ptrs, const int64_t* offs, const int64_t* numels, int ntensors,
                              void* flat, int tensor_dt, int flat_dt, float scale, hipStream_t stream) {
  const int tsz = dt_size(tensor_dt), fsz = dt_size(flat_dt);
  for (int base = 0; base < ntensors; base += kMaxTensors) {
    TensorTable tab;
    int n = ntensors - base < kMaxTensors ? ntensors - base : kMaxTensors;
    int32_t chunks = 0;
    tab.n = 0;
    for (int k = 0; k < n; ++k) {
      const int64_t ne = numels[base + k];
      if (ne <= 0) continue;
      const int m = tab.n++;
      tab.ptr[m] = ptrs[base + k];
      tab.off[m] = offs[base + k];
      tab.numel[m] = ne;
      tab.chunk_start[m] = chunks;
      const uintptr_t pa = reinterpret_cast<uintptr_t>(ptrs[base + k]);
      const uintptr_t fa = reinterpret_cast<uintptr_t>(flat) + (uintptr_t)(offs[base + k] * fsz);
      tab.vec_ok[m] = ((pa % 16) == 0 && (fa % 16) == 0 && ((8 * tsz) % 16) == 0) ? 1 : 0;
      chunks += (int32_t)((ne + kPackChunk - 1) / kPackChunk);
    }
    if (tab.n == 0) continue;
    tab.chunk_start[tab.n] = chunks;
    dim3 grid(chunks), block(kPackThreads);
    MADNN_DISPATCH_DT(tensor_dt, TDT, MADNN_DISPATCH_DT(flat_dt, FDT, {
      if (pack) hipLaunchKernelGGL((bucket_copy_kernel<TDT, FDT, true>), grid, block, 0, stream, tab, flat, scale);
      else hipLaunchKernelGGL((bucket_copy_kernel<TDT, FDT, false>), grid, block, 0, stream, tab, flat, scale);
    }));
    MADNN_HIP_CHECK(hipGetLastError());
  }
  return hipSuccess;
}

}  // namespace madnn

extern "C" {

hipError_t madnn_bucket_pack(void* const* srcs, const int64_t* offs, const int64_t* numels, int n, void* flat,
                             int src_dt, int flat_dt, float scale, hipStream_t stream) {
  return madnn::bucket_copy(true, srcs, offs, numels, n, flat, src_dt, flat_dt, scale, stream);
}

hipError_t madnn_bucket_unpack(void* const* dsts, const int64_t* offs, const int64_t* numels, int n, void* flat,
                               int dst_dt, int flat_dt, float scale, hipStream_t stream) {
  return madnn::bucket_copy(false, dsts, offs, numels, n, flat, dst_dt, flat_dt, scale, stream);
}

hipError_t madnn_flat_scale_cast(const void* src, void* dst, int64_t n, int src_dt, int dst_dt, float scale,
                                 hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  const int grid = madnn::stream_grid(n, 256 * 8);
  MADNN_DISPATCH_DT(src_dt, SDT, MADNN_DISPATCH_DT(dst_dt, DDT, {
    hipLaunchKernelGGL((madnn::flat_scale_cast_kernel<SDT, DDT>), dim3(grid), dim3(256), 0, stream, src, dst, n,
                       scale);
  }));
  return hipGetLastError();
}

}  // extern "C"
