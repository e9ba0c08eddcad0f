// madnn native kernels — shared device helpers for gfx950 (CDNA4, wave64).
//
// Every kernel in this directory is written directly for MI355X: 64-lane
// wavefronts, 16-byte-per-lane vector memory access, wave-shuffle reductions
// and grid sizes that cover 256 CUs.  There is no CUDA path and no hipify.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace madnn {

constexpr int kWave = 64;          // CDNA wavefront width (never 32)
constexpr int kNumCU = 256;        // MI355X: 8 XCDs x 32 CUs
constexpr int kNumXCD = 8;

typedef __attribute__((address_space(3))) void lds_void;

// LDS-DMA (global_load_lds_dwordx4 / _dword: each lane's 16 / 4 bytes land at the wave-uniform LDS
// address `dst` + size * lane), written as inline asm (cdna_hip_programming.md §5.7 recipe: M0 set and
// restored inside the statement, s_nop 0 before the load).  Why not the builtin: hipcc treats every
// later ds_read_b64_tr_b16 as aliasing each pending builtin LDS-DMA and drains vmcnt(0) before it,
// which flushes the whole prefetch pipeline once per K step in every kernel that reads a transposed
// operand (K12 data / weight gradients, K12P data gradient, the attention backward).  hipcc does not
// count these loads: the kernels wait for them with their own counted s_waitcnt vmcnt(N) and barriers;
// the compiler's own waits for its loads stay correct (they only ever see fewer younger operations).
__device__ __forceinline__ void glds16(const void* src, lds_void* dst) {
  const unsigned lds = __builtin_amdgcn_readfirstlane((unsigned)(size_t)dst);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(lds)
               : "memory");
}
__device__ __forceinline__ void glds4(const void* src, lds_void* dst) {
  const unsigned lds = __builtin_amdgcn_readfirstlane((unsigned)(size_t)dst);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(lds)
               : "memory");
}

// dtype codes shared with the Python side (madnn/ops/_native.py)
enum DType : int { kF32 = 0, kBF16 = 1, kF16 = 2 };

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf16_to_f32(unsigned short h) {
  return __uint_as_float(((unsigned)h) << 16);
}

// Plain cast: hipcc -O3 emits v_cvt_pk_bf16_f32 on gfx950 (RNE, NaN kept NaN;
// MI355X_MICROARCH.md "Correctness boundaries").
__device__ __forceinline__ unsigned short f32_to_bf16(float f) {
  __bf16 b = static_cast<__bf16>(f);
  return __builtin_bit_cast(unsigned short, b);
}

__device__ __forceinline__ float f16_to_f32(unsigned short h) {
  _Float16 v = __builtin_bit_cast(_Float16, h);
  return static_cast<float>(v);
}

__device__ __forceinline__ unsigned short f32_to_f16(float f) {
  _Float16 v = static_cast<_Float16>(f);
  return __builtin_bit_cast(unsigned short, v);
}

// Typed scalar load/store through the dtype code (runtime-dispatched at the
// launch site with templates; these are the element converters).
template <int DT> struct Elem;
template <> struct Elem<kF32> {
  using T = float;
  static __device__ __forceinline__ float load(const T* p, int64_t i) { return p[i]; }
  static __device__ __forceinline__ void store(T* p, int64_t i, float v) { p[i] = v; }
};
template <> struct Elem<kBF16> {
  using T = unsigned short;
  static __device__ __forceinline__ float load(const T* p, int64_t i) { return bf16_to_f32(p[i]); }
  static __device__ __forceinline__ void store(T* p, int64_t i, float v) { p[i] = f32_to_bf16(v); }
};
template <> struct Elem<kF16> {
  using T = unsigned short;
  static __device__ __forceinline__ float load(const T* p, int64_t i) { return f16_to_f32(p[i]); }
  static __device__ __forceinline__ void store(T* p, int64_t i, float v) { p[i] = f32_to_f16(v); }
};

// 8 consecutive elements <-> 8 floats with one 16-byte (bf16/f16) or two
// 16-byte (f32) accesses per lane.
template <int DT>
__device__ __forceinline__ void load8(const void* base, int64_t i, float (&v)[8]) {
  if constexpr (DT == kF32) {
    const f32x4* p = reinterpret_cast<const f32x4*>(static_cast<const float*>(base) + i);
    f32x4 a = p[0], b = p[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
    u16x8 r = *reinterpret_cast<const u16x8*>(static_cast<const unsigned short*>(base) + i);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (DT == kBF16) ? bf16_to_f32(r[j]) : f16_to_f32(r[j]);
  }
}

template <int DT>
__device__ __forceinline__ void store8(void* base, int64_t i, const float (&v)[8]) {
  if constexpr (DT == kF32) {
    f32x4* p = reinterpret_cast<f32x4*>(static_cast<float*>(base) + i);
    p[0] = f32x4{v[0], v[1], v[2], v[3]};
    p[1] = f32x4{v[4], v[5], v[6], v[7]};
  } else {
    u16x8 r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = (DT == kBF16) ? f32_to_bf16(v[j]) : f32_to_f16(v[j]);
    *reinterpret_cast<u16x8*>(static_cast<unsigned short*>(base) + i) = r;
  }
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

// Memory-bound grid: enough workgroups to cover every CU several times, then
// grid-stride (cdna_hip_programming.md Guideline 11).
inline int stream_grid(int64_t work_items, int per_block, int max_blocks = 8 * kNumCU) {
  int64_t g = (work_items + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > max_blocks) g = max_blocks;
  return static_cast<int>(g);
}

}  // namespace madnn

#define MADNN_HIP_CHECK(expr)                                                   \
  do {                                                                          \
    hipError_t _e = (expr);                                                     \
    if (_e != hipSuccess) return _e;                                            \
  } while (0)

// Runtime dtype -> template dispatch for a (in, out) pair.
#define MADNN_DISPATCH_DT(dt, NAME, ...)                                        \
  switch (dt) {                                                                 \
    case ::madnn::kF32: { constexpr int NAME = ::madnn::kF32; __VA_ARGS__; break; } \
    case ::madnn::kBF16: { constexpr int NAME = ::madnn::kBF16; __VA_ARGS__; break; } \
    case ::madnn::kF16: { constexpr int NAME = ::madnn::kF16; __VA_ARGS__; break; } \
    default: return hipErrorInvalidValue;                                       \
  }
