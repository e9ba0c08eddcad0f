// K14 / K15 — the Llama block's elementwise glue as single passes (bf16 I/O, fp32 math).
//
// Why: on the Llama-3 8B step (profiles/r5_llama8b_steady_steps.md) PyTorch's RoPE (chunk, neg,
// cat, two multiplies, an add -- for q and k, forward and backward) and SwiGLU (split views, silu,
// mul; their backward, then a cat of dgate / dup back into the fused gate_up gradient) took ~13 % of
// the step in ~10 elementwise launches per layer, each a full HBM pass.
//
// K14 rope_qkv: the PACKED QKV projection output [B, S, H + 2 Hkv, D] with its q and k heads rotated,
//   (x[i], x[i + D/2]) -> (x[i] c - x[i + D/2] s, x[i + D/2] c + x[i] s), c / s from the
//   host-precomputed fp32 tables [pos][D], the v heads copied, into a new packed buffer (one pass);
//   `inverse` applies the transpose rotation in place (the backward, on the attention's dQKV).  The
//   attention kernel then reads q / k / v in place and writes dQKV in place: no split, no rotated
//   q / k copies, no cat.  One lane: 8 consecutive pairs (two 16-B loads / stores).
// K15 swiglu: h = silu(g) u from the gate_up GEMM output [M, 2I] (g = columns 0..I-1, u = I..2I-1);
//   the backward writes d[g | u] = [dh u silu'(g) | dh silu(g)] straight into the packed gradient
//   the gate_up Linear's backward consumes.  silu via v_exp_f32 + v_rcp_f32.
// Reference: none (SURVEY §2.5 lists the Llama config's model zoo, not these kernels); numerics are
// checked against fp32 PyTorch in tests/test_glue_gpu.py.
#include "common.h"

namespace madnn {
namespace glue {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void unpack8(const u32x4& v, float (&f)[8]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    f[2 * j] = bf16_to_f32((unsigned short)(v[j] & 0xffffu));
    f[2 * j + 1] = bf16_to_f32((unsigned short)(v[j] >> 16));
  }
}

__device__ __forceinline__ u32x4 pack8(const float (&f)[8]) {
  u32x4 v;
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = (unsigned)f32_to_bf16(f[2 * j]) | ((unsigned)f32_to_bf16(f[2 * j + 1]) << 16);
  return v;
}

// one unit = 8 pairs of one head of one (b, s) row: heads < NR rotated, the others copied
// (in place: only the NR rotated heads are visited)
template <bool INV>
__global__ __launch_bounds__(256) void rope_qkv_kernel(const uint16_t* __restrict__ src, uint16_t* __restrict__ dst,
                                                       const float* __restrict__ cos_t, const float* __restrict__ sin_t,
                                                       int64_t units, int S, int NH, int NV, int NR, int D) {
  const int per_head = D / 16;  // units per head
  for (int64_t u = (int64_t)blockIdx.x * 256 + threadIdx.x; u < units; u += (int64_t)gridDim.x * 256) {
    const int part = (int)(u % per_head);
    const int64_t rh = u / per_head;
    const int hd = (int)(rh % NV);
    const int64_t row = rh / NV;
    const int s = (int)(row % S);
    const int64_t off = (row * NH + hd) * D + 8 * part;
    const uint16_t* x = src + off;
    uint16_t* y = dst + off;
    if (hd >= NR) {  // a v head: copied
      *reinterpret_cast<u32x4*>(y) = *reinterpret_cast<const u32x4*>(x);
      *reinterpret_cast<u32x4*>(y + D / 2) = *reinterpret_cast<const u32x4*>(x + D / 2);
      continue;
    }
    const float* cp = cos_t + (int64_t)s * D + 8 * part;
    const float* sp = sin_t + (int64_t)s * D + 8 * part;
    float a[8], b[8], o1[8], o2[8];
    unpack8(*reinterpret_cast<const u32x4*>(x), a);
    unpack8(*reinterpret_cast<const u32x4*>(x + D / 2), b);
    const f32x4 c0 = *reinterpret_cast<const f32x4*>(cp), c1 = *reinterpret_cast<const f32x4*>(cp + 4);
    const f32x4 s0 = *reinterpret_cast<const f32x4*>(sp), s1 = *reinterpret_cast<const f32x4*>(sp + 4);
    const float c[8] = {c0[0], c0[1], c0[2], c0[3], c1[0], c1[1], c1[2], c1[3]};
    const float sn[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if constexpr (INV) {
        o1[j] = fmaf(a[j], c[j], b[j] * sn[j]);
        o2[j] = fmaf(b[j], c[j], -a[j] * sn[j]);
      } else {
        o1[j] = fmaf(a[j], c[j], -b[j] * sn[j]);
        o2[j] = fmaf(b[j], c[j], a[j] * sn[j]);
      }
    }
    *reinterpret_cast<u32x4*>(y) = pack8(o1);
    *reinterpret_cast<u32x4*>(y + D / 2) = pack8(o2);
  }
}

__device__ __forceinline__ float sigmoid(float g) {
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-1.4426950408889634f * g));
}

// h[m][j] = silu(gu[m][j]) * gu[m][I + j]; one unit = 8 consecutive j
__global__ __launch_bounds__(256) void swiglu_fwd_kernel(const uint16_t* __restrict__ gu, uint16_t* __restrict__ h,
                                                         int64_t units, int I) {
  const int per_row = I / 8;
  for (int64_t u = (int64_t)blockIdx.x * 256 + threadIdx.x; u < units; u += (int64_t)gridDim.x * 256) {
    const int64_t m = u / per_row;
    const int j = (int)(u - m * per_row) * 8;
    float g[8], v[8], o[8];
    unpack8(*reinterpret_cast<const u32x4*>(gu + m * 2 * I + j), g);
    unpack8(*reinterpret_cast<const u32x4*>(gu + m * 2 * I + I + j), v);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = g[e] * sigmoid(g[e]) * v[e];
    *reinterpret_cast<u32x4*>(h + m * I + j) = pack8(o);
  }
}

// dgu[m][j] = dh u silu'(g), dgu[m][I + j] = dh silu(g), silu'(g) = s (1 + g (1 - s)), s = sigmoid(g)
__global__ __launch_bounds__(256) void swiglu_bwd_kernel(const uint16_t* __restrict__ dh,
                                                         const uint16_t* __restrict__ gu, uint16_t* __restrict__ dgu,
                                                         int64_t units, int I) {
  const int per_row = I / 8;
  for (int64_t u = (int64_t)blockIdx.x * 256 + threadIdx.x; u < units; u += (int64_t)gridDim.x * 256) {
    const int64_t m = u / per_row;
    const int j = (int)(u - m * per_row) * 8;
    float d[8], g[8], v[8], og[8], ou[8];
    unpack8(*reinterpret_cast<const u32x4*>(dh + m * I + j), d);
    unpack8(*reinterpret_cast<const u32x4*>(gu + m * 2 * I + j), g);
    unpack8(*reinterpret_cast<const u32x4*>(gu + m * 2 * I + I + j), v);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float s = sigmoid(g[e]);
      og[e] = d[e] * v[e] * s * fmaf(g[e], 1.f - s, 1.f);
      ou[e] = d[e] * g[e] * s;
    }
    *reinterpret_cast<u32x4*>(dgu + m * 2 * I + j) = pack8(og);
    *reinterpret_cast<u32x4*>(dgu + m * 2 * I + I + j) = pack8(ou);
  }
}

inline unsigned grid_for(int64_t units) {
  const int64_t g = (units + 255) / 256, cap = 8 * (int64_t)kNumCU;  // grid-stride beyond 8 WGs per CU
  return (unsigned)(g < 1 ? 1 : g > cap ? cap : g);
}

}  // namespace glue
}  // namespace madnn

using namespace madnn::glue;

extern "C" {

// src / dst: bf16 [rows = B*S][NH][D] contiguous (dst == src: in place, the NR rotated heads only);
// heads 0..NR-1 rotated (q then k), the rest copied; cos / sin: fp32 [>= S][D]
hipError_t madnn_rope_qkv(const void* src, void* dst, const float* cos_t, const float* sin_t, int64_t rows, int S,
                          int NH, int NR, int D, int inverse, hipStream_t st) {
  if (D % 16 || NR > NH || S <= 0 || rows % S) return hipErrorInvalidValue;
  const int NV = src == dst ? NR : NH;  // heads visited
  const int64_t units = rows * NV * (D / 16);
  if (units == 0) return hipSuccess;
  const uint16_t* x = static_cast<const uint16_t*>(src);
  uint16_t* y = static_cast<uint16_t*>(dst);
  if (inverse) {
    hipLaunchKernelGGL(rope_qkv_kernel<true>, dim3(grid_for(units)), dim3(256), 0, st, x, y, cos_t, sin_t, units, S,
                       NH, NV, NR, D);
  } else {
    hipLaunchKernelGGL(rope_qkv_kernel<false>, dim3(grid_for(units)), dim3(256), 0, st, x, y, cos_t, sin_t, units, S,
                       NH, NV, NR, D);
  }
  return hipGetLastError();
}

// gu: bf16 [M][2I], h: bf16 [M][I]; I % 8 == 0
hipError_t madnn_swiglu_fwd(const void* gu, void* h, int64_t M, int I, hipStream_t st) {
  if (I % 8) return hipErrorInvalidValue;
  const int64_t units = M * (I / 8);
  if (units == 0) return hipSuccess;
  hipLaunchKernelGGL(swiglu_fwd_kernel, dim3(grid_for(units)), dim3(256), 0, st, static_cast<const uint16_t*>(gu),
                     static_cast<uint16_t*>(h), units, I);
  return hipGetLastError();
}

hipError_t madnn_swiglu_bwd(const void* dh, const void* gu, void* dgu, int64_t M, int I, hipStream_t st) {
  if (I % 8) return hipErrorInvalidValue;
  const int64_t units = M * (I / 8);
  if (units == 0) return hipSuccess;
  hipLaunchKernelGGL(swiglu_bwd_kernel, dim3(grid_for(units)), dim3(256), 0, st, static_cast<const uint16_t*>(dh),
                     static_cast<const uint16_t*>(gu), static_cast<uint16_t*>(dgu), units, I);
  return hipGetLastError();
}

}  // extern "C"
