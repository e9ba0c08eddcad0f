// Shared MFMA-tile helpers for the GEMM-shaped gfx950 kernels (K9 conv1x1).
//
// v_mfma_f32_32x32x16_bf16 operand maps (cdna_hip_programming.md §3): lane l holds
// A[row l&31][k 8(l>>5) .. +7] and B[k 8(l>>5) .. +7][col l&31]; the accumulator holds
// D[row acc_row(r, l>>5)][col l&31] in register r.  LDS tiles are XOR-swizzled so that
// the two read kinds used here are bank-conflict-free:
//   * row reads (ds_read_b128): a [R][64] bf16 tile (128-B rows), lane reads row l&31,
//     16-B chunk 2s + (l>>5) -> swz<64> (the image attn.hip uses for its K tiles);
//   * natural-order transposed reads (2 x ds_read_b64_tr_b16): a [64][C] tile (C = 64 or
//     128), lane half h reads rows 16s + 8h .. +7 of column c0 + (l&31) -> swz<C>.
// For the transposed read each 32-lane half touches 4 rows x 4 aligned 16-B chunks per
// instruction; the XOR term gives the 4 rows 4 different chunk groups, i.e. 16 distinct
// 16-B slots = all 64 banks (for 128-B rows, two rows per bank row, and for 256-B rows).
#pragma once

#include "common.h"

namespace madnn {
namespace mf {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f32x16 mfma(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// accumulator register r of lane half h -> row within the 32-row block
__device__ __forceinline__ int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// byte offset of 16-B chunk `ch` of row `row` in a tile with C bf16 per row (C = 64 or 128)
template <int C>
__device__ __forceinline__ int swz(int row, int ch) {
  static_assert(C == 64 || C == 128, "swizzled tiles have 64 or 128 columns");
  if constexpr (C == 64) {
    return row * 128 + 16 * (ch ^ ((((row >> 1) & 1) << 2) | ((row >> 2) & 3)));
  } else {
    return row * 256 + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
  }
}

// operand fragment with k along the row: 8 bf16 of row `row`, chunk `ch` of a [R][64] tile
__device__ __forceinline__ bf16x8 lds_row(const uint16_t* tile, int row, int ch) {
  return *reinterpret_cast<const bf16x8*>(reinterpret_cast<const char*>(tile) + swz<64>(row, ch));
}

// operand fragment with k down the rows of a [64][C] tile, natural k order:
// element j of lane half h = tile[r0 + 8h + j][c0 + (lane & 31)]
template <int C>
__device__ __forceinline__ bf16x8 lds_col(const uint16_t* tile, int r0, int c0, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int col = c0 + 16 * (g & 1) + 4 * (i & 3);
  const int row = r0 + 8 * (g >> 1) + (i >> 2);
  const char* base = reinterpret_cast<const char*>(tile);
  const int sub = 8 * ((col >> 2) & 1);
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + swz<C>(row, col >> 3) + sub));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + swz<C>(row + 4, col >> 3) + sub));
  const s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, r);
}

__device__ __forceinline__ void store4_bf16(uint16_t* p, float a, float b, float c, float d) {
  const unsigned lo = (unsigned)f32_to_bf16(a) | ((unsigned)f32_to_bf16(b) << 16);
  const unsigned hi = (unsigned)f32_to_bf16(c) | ((unsigned)f32_to_bf16(d) << 16);
  *reinterpret_cast<u32x2*>(p) = u32x2{lo, hi};
}

__device__ __forceinline__ float round_bf16(float v) { return bf16_to_f32(f32_to_bf16(v)); }

}  // namespace mf
}  // namespace madnn
