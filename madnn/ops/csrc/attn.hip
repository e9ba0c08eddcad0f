// K8: fused (flash-style) multi-head attention forward/backward for gfx950.
//
// Replaces PyTorch-ROCm's SDPA kernels for the transformer models (GPT-2, BERT,
// Llama; SURVEY §7 "MFMA for GEMM-shaped work").  bf16 I/O, fp32 accumulation,
// head dim 64 or 128, causal or full, grouped-query (Hkv | H), any sequence length.
// Inputs are strided [B, S, heads, D] views, so the packed QKV projection output is
// consumed in place and dQKV is written in place: no transposes, no split/cat copies.
//
// CDNA4 mapping (cdna_hip_programming.md §3, T2, T10; Appendix B "Fused attention"):
//  * every product is v_mfma_f32_32x32x16_bf16 on 64-lane waves; a workgroup is
//    4 waves (one per SIMD);
//  * "query on the lane" (forward, dQ): S^T = K.Q^T puts one query row per lane
//    (and its partner lane l^32), so the online-softmax max/sum is lane-local plus
//    one cross-half exchange, and the S^T accumulator is -- unmoved -- the B
//    operand of O^T += V^T.P^T / dQ^T += K^T.dS^T (accumulator-as-operand idiom);
//  * "key on the lane" (dK/dV): S = Q.K^T, dP = dO.V^T give P and dS with the
//    key on the lane; they are the A operands of dV += P^T.dO and dK += dS^T.Q;
//  * K/V (or Q/dO) tiles are staged global -> registers -> LDS, double-buffered
//    with one barrier per tile; the LDS image is XOR-swizzled so that BOTH the
//    row reads (ds_read_b128, MFMA operand with the head dim as k) and the
//    transposed reads (ds_read_b64_tr_b16, operand with the sequence as k) are
//    bank-conflict-free (the swizzle proofs are in the comments of swz());
//  * the backward is two kernels: dQ (query blocks; its prologue also forms delta = rowsum(dO*O)
//    for its rows and writes it out); dK/dV (key blocks, looping over the query heads of a grouped KV head) --
//    no atomics, deterministic;
//  * block -> (sequence block, batch*head) mapping is XCD-aware: the workgroups
//    dispatched to one XCD work on the same heads, so K/V tiles hit in its L2.
// Reference: the reference has no attention; this serves the
// transformer configs of BASELINE.json (GPT-2 medium, BERT-large, Llama-3 8B).
#include <type_traits>

#include "attn.h"
#include "common.h"

namespace madnn {
namespace attn {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

constexpr int kThreads = 256;  // 4 waves
constexpr int kRowsWG = 128;   // query rows per workgroup (fwd, dQ) / key rows (dK/dV)
constexpr int kTile = 64;      // keys per tile (fwd, dQ) / queries per tile (dK/dV)
constexpr float kNegBig = -1.0e30f;

__device__ __forceinline__ f32x16 mfma(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// v_exp_f32 directly (exp2f adds denormal range reduction: 4 more VALU per element; a
// softmax weight below 2^-126 is 0 either way)
__device__ __forceinline__ float ex2(float x) { return __builtin_amdgcn_exp2f(x); }

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// Byte offset of 16-B chunk `ch` of row `row` in a [64][D] bf16 LDS tile.
// D = 64 (128-B rows, 2 rows per 256-B bank row): ch ^ f(row), f = ((row>>1)&1)<<2 | (row>>2)&3.
//   ds_read_b128 groups {0-3,12-15,20-27} / {4-11,16-19,28-31} (row = lane): the 8 even and the 8
//   odd rows of each group get 8 distinct f -> 16 distinct 16-B slots.  Transposed read (rows
//   4n..4n+3, an aligned 4-chunk group per 32-lane half): rows 4n, 4n+2 differ in f bit 2, rows
//   4n+1, 4n+3 sit in the other half of the bank row -> 16 distinct slots.
// D = 128 (256-B rows): the dual-use image (b) of cdna_hip_programming.md T10.
template <int D>
__device__ __forceinline__ int swz(int row, int ch) {
  if constexpr (D == 64) {
    return row * 128 + 16 * (ch ^ ((((row >> 1) & 1) << 2) | ((row >> 2) & 3)));
  } else {
    return row * 256 + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
  }
}

// MFMA operand with the head dim as k: 8 bf16 of row `row`, chunk `ch` (ds_read_b128).
template <int D>
__device__ __forceinline__ bf16x8 lds_row(const uint16_t* tile, int row, int ch) {
  return *reinterpret_cast<const bf16x8*>(reinterpret_cast<const char*>(tile) + swz<D>(row, ch));
}

// MFMA operand with the tile's ROW index as k (two ds_read_b64_tr_b16): element j of lane half h
// is tile[r0 + 8*(j>>2) + 4h + (j&3)][c0 + (lane&31)] -- the k order in which an f32x16
// accumulator's registers 8s..8s+7 serve as the other operand (pack_acc).
template <int D>
__device__ __forceinline__ bf16x8 lds_tr(const uint16_t* tile, int r0, int c0, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int col = c0 + 16 * (g & 1) + 4 * (i & 3);
  const int row = r0 + 4 * (g >> 1) + (i >> 2);
  const char* base = reinterpret_cast<const char*>(tile);
  const int sub = 8 * ((col >> 2) & 1);
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + swz<D>(row, col >> 3) + sub));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + swz<D>(row + 8, col >> 3) + sub));
  const s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, r);
}

// registers 8s..8s+7 of an accumulator -> bf16 operand fragment (v_cvt_pk_bf16_f32)
__device__ __forceinline__ bf16x8 pack_acc(const f32x16& x, int s) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = static_cast<__bf16>(x[8 * s + j]);
  return r;
}

// accumulator register r of lane half h -> row within the 32-row block
__device__ __forceinline__ int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// 8 bf16 scaled by k and rounded back to bf16: the exp2-domain operand prescale (row constants as
// the initial accumulator, cdna_hip_programming.md 'Attention backward'): with Q (or K) prescaled by
// -c, c = scale * log2(e), an S accumulator started at a row constant r ends as r - S' (S' = the
// score in log2 units) and p = exp2(-acc) -- the negation a free source modifier -- so the per-element
// scale-and-subtract (32 v_fma per tile per lane) is gone.  Cost: the operand is rounded to bf16 once
// more (relative 2^-9 per element).
__device__ __forceinline__ bf16x8 scale_bf16x8(const bf16x8& x, float k) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = static_cast<__bf16>(static_cast<float>(x[j]) * k);
  return r;
}

__device__ __forceinline__ f32x16 splat16(float v) {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = v;
  return z;
}

// [64][D] tile: global (row stride `ld` elements, rows >= nvalid read as zeros) -> regs -> LDS.
// BUF (the backward kernels): buffer loads through a per-tile descriptor (base at row0, range = the
// nvalid - row0 rows left): rows past the end come back as zeros from the range check, so the load
// needs no branch, no zero fill and no 64-bit address arithmetic -- the per-lane byte offset is
// tile-invariant (cdna_hip_programming.md T8 / T20: the descriptor is built from wave-uniform values
// only).  Measured: backward -8 % at D = 128, neutral at D = 64; the forward kernel keeps the global
// loads (+23 % forward time at D = 128 with BUF, profiles/r4_ab_attn_valu_trees.log).
template <int D, bool BUF = false>
struct TileStage {
  static constexpr int CH = D / 8;
  static constexpr int PER = kTile * CH / kThreads;
  u32x4 r[PER];
  __device__ __forceinline__ void load(const uint16_t* base, int64_t ld, int row0, int nvalid, int tid) {
    if constexpr (BUF) {
      const int64_t left = (int64_t)max(nvalid - row0, 0) * ld * 2;
      const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<uint16_t*>(base + (int64_t)row0 * ld), 0, (int)min(left, (int64_t)0x7fffffff), 0x00020000);
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int c = tid + kThreads * i;
        const int row = c / CH, ch = c % CH;
        r[i] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)(row * ld + ch * 8) * 2, 0, 0);
      }
    } else {
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int c = tid + kThreads * i;
        const int row = c / CH, ch = c % CH;
        if (row0 + row < nvalid) {
          r[i] = *reinterpret_cast<const u32x4*>(base + (int64_t)(row0 + row) * ld + ch * 8);
        } else {
          r[i] = u32x4{0u, 0u, 0u, 0u};
        }
      }
    }
  }
  __device__ __forceinline__ void store(uint16_t* tile, int tid) const {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = tid + kThreads * i;
      const int row = c / CH, ch = c % CH;
      *reinterpret_cast<u32x4*>(reinterpret_cast<char*>(tile) + swz<D>(row, ch)) = r[i];
    }
  }
};

// Workgroup -> (sequence block, batch, head): consecutive logical ids on one XCD
// (bijective remap, cdna_hip_programming.md "XCD swizzle must be bijective").
__device__ __forceinline__ void map_block(int nblk, int heads, bool heavy_last, int& blk, int& b, int& h) {
  const int nwg = gridDim.x;
  const int id = blockIdx.x;
  const int xcd = id % 8, q8 = nwg / 8, r8 = nwg % 8;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + id / 8;
  const int bh = wg / nblk;
  blk = wg % nblk;
  if (heavy_last) blk = nblk - 1 - blk;  // causal: the longest query blocks start first
  b = bh / heads;
  h = bh % heads;
}

__device__ __forceinline__ void store4_bf16(uint16_t* p, float a, float b, float c, float d) {
  const unsigned lo = (unsigned)f32_to_bf16(a) | ((unsigned)f32_to_bf16(b) << 16);
  const unsigned hi = (unsigned)f32_to_bf16(c) | ((unsigned)f32_to_bf16(d) << 16);
  *reinterpret_cast<u32x2*>(p) = u32x2{lo, hi};
}

// ------------------------------------------------------------------ forward
// The causal / sequence-end mask is one compare of a compile-time key offset against a per-lane
// limit, and the running max is moved only when a row's max grows by more than 2^8 (lazy rescale:
// the O / l rescale pass -- 32 multiplies and an exp per lane -- is skipped on most tiles; p <= 256 is
// exact in fp32 and relative-exact in the bf16 P operand, and O / l and the LSE do not depend on
// which m is used).
constexpr float kRescaleSlack = 8.f;

// One key tile of the online softmax on the prescaled accumulators acc = mi - S' (masked: +inf; mi =
// the rows' current reference, 0 before the first tile, m = kNegBig until then): the tile's row max
// is mi - min(acc); when it passes m + slack (always on the first tile) O and l are rescaled, the
// tile's acc shifted to the new reference and the splatted reference tuple (the next tiles' initial
// accumulator) updated.  Then acc <- p = exp2(-acc) and l += the lane's part of the row sums.
template <int DB>
__device__ __forceinline__ void softmax_tile(f32x16 (&sc)[2], f32x16 (&o)[DB], float& m, float& mi, float& l,
                                             f32x16& mref) {
  float mn = sc[0][0];
#pragma unroll
  for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
    for (int r = 0; r < 16; ++r) mn = fminf(mn, sc[kb][r]);
  }
  mn = fminf(mn, __shfl_xor(mn, 32));
  const float top = mi - mn;
  if (__any(top > m + kRescaleSlack)) {
    const float mnew = fmaxf(m, top);
    const float alpha = ex2(m - mnew);
    l *= alpha;
#pragma unroll
    for (int d = 0; d < DB; ++d) {
#pragma unroll
      for (int r = 0; r < 16; ++r) o[d][r] *= alpha;
    }
    const float adj = mnew - mi;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
      for (int r = 0; r < 16; ++r) sc[kb][r] += adj;
    }
    m = mi = mnew;
    mref = splat16(mnew);
  }
  float rs = 0.f;
#pragma unroll
  for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float p = ex2(-sc[kb][r]);
      sc[kb][r] = p;
      rs += p;
    }
  }
  l += rs;
}

// D = 128 is built for 2 waves per SIMD (256 VGPRs, a few spills; 348 and one wave unbounded):
// +27 % at Llama-3 8B's shape, profiles/r5_attn_ab_occupancy.json
template <int D, bool CAUSAL>
__global__ __launch_bounds__(kThreads, D == 128 ? 2 : 1) void attn_fwd_kernel(const MadnnAttnArgs a) {
  constexpr int DS = D / 16, DB = D / 32;
  __shared__ __attribute__((aligned(16))) uint16_t sK[2][kTile * D];
  __shared__ __attribute__((aligned(16))) uint16_t sV[2][kTile * D];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, l32 = lane & 31, hh = lane >> 5;
  const int nqb = (a.S + kRowsWG - 1) / kRowsWG;
  int qblk, b, h;
  map_block(nqb, a.H, CAUSAL, qblk, b, h);
  const int hk = h / (a.H / a.Hkv);
  const int q0w = qblk * kRowsWG + wave * 32;
  const int qrow = q0w + l32;

  // -c Q^T as the B operand of S^T = K.Q^T: lane holds -c Q[qrow][16s + 8hh + j]
  bf16x8 qf[DS];
  {
    const uint16_t* qp = a.q + b * a.q_sb + h * a.q_sh + (int64_t)min(qrow, a.S - 1) * a.q_ss;
#pragma unroll
    for (int s = 0; s < DS; ++s) qf[s] = scale_bf16x8(*reinterpret_cast<const bf16x8*>(qp + 16 * s + 8 * hh), -a.scale_log2);
  }
  const uint16_t* kb_ = a.k + b * a.k_sb + hk * a.k_sh;
  const uint16_t* vb_ = a.v + b * a.v_sb + hk * a.v_sh;
  f32x16 o[DB];
#pragma unroll
  for (int d = 0; d < DB; ++d) o[d] = zero16();
  float m = kNegBig, mi = 0.f, l = 0.f;
  f32x16 mref = zero16();
  const int kv_end = CAUSAL ? min(a.S, qblk * kRowsWG + kRowsWG) : a.S;
  const int ntiles = (kv_end + kTile - 1) / kTile;

  TileStage<D> stk, stv;  // global loads (see TileStage)
  stk.load(kb_, a.k_ss, 0, a.S, tid);
  stv.load(vb_, a.v_ss, 0, a.S, tid);
  stk.store(sK[0], tid);
  stv.store(sV[0], tid);
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1;
    const bool more = t + 1 < ntiles;
    if (more) {
      stk.load(kb_, a.k_ss, (t + 1) * kTile, a.S, tid);
      stv.load(vb_, a.v_ss, (t + 1) * kTile, a.S, tid);
    }
    const int k0 = t * kTile;
    if (!CAUSAL || k0 <= q0w + 31) {
      f32x16 sc[2];
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        sc[kb] = mref;
#pragma unroll
        for (int s = 0; s < DS; ++s) sc[kb] = mfma(lds_row<D>(sK[cur], kb * 32 + l32, 2 * s + hh), qf[s], sc[kb]);
      }
      if ((k0 + kTile > a.S) || (CAUSAL && k0 + kTile - 1 > q0w)) {
        // key k0 + kb*32 + acc_row(r, hh) is valid iff its compile-time offset kb*32 + acc_row(r, 0)
        // <= lim (one compare + select per element)
        const int lim = (CAUSAL ? min(a.S - 1, qrow) : a.S - 1) - k0 - 4 * hh;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
          for (int r = 0; r < 16; ++r) sc[kb][r] = kb * 32 + acc_row(r, 0) <= lim ? sc[kb][r] : __builtin_inff();
        }
      }
      softmax_tile<DB>(sc, o, m, mi, l, mref);
      // O^T[d][q] += sum_key V[key][d] P^T[key][q]
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const bf16x8 pf = pack_acc(sc[kb], s);
#pragma unroll
          for (int d = 0; d < DB; ++d) o[d] = mfma(lds_tr<D>(sV[cur], kb * 32 + 16 * s, d * 32, lane), pf, o[d]);
        }
      }
    }
    if (more) {
      stk.store(sK[cur ^ 1], tid);
      stv.store(sV[cur ^ 1], tid);
    }
    __syncthreads();
  }
  const float lt = l + __shfl_xor(l, 32);
  const float inv = lt > 0.f ? 1.f / lt : 0.f;
  if (qrow < a.S) {
    uint16_t* op = a.o + b * a.o_sb + h * a.o_sh + (int64_t)qrow * a.o_ss;
#pragma unroll
    for (int d = 0; d < DB; ++d) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        store4_bf16(op + d * 32 + 8 * g + 4 * hh, o[d][4 * g] * inv, o[d][4 * g + 1] * inv, o[d][4 * g + 2] * inv,
                    o[d][4 * g + 3] * inv);
      }
    }
    if (hh == 0) a.lse[((int64_t)b * a.H + h) * a.S + qrow] = m + log2f(lt);
  }
}

// ------------------------------------------------------------------ backward: dQ
// The S^T accumulators start at the lane's LSE (a loop-invariant register tuple) against the -c
// prescaled Q, so p = exp2(-acc); ACCD (D = 64): the dP^T accumulators start at -delta the same way,
// so dS = P * acc costs no subtraction (at D = 128 that tuple's 16 registers cost more than the
// subtraction: -8 %, profiles/r4_ab_attn_valu_trees.log).  delta = rowsum(dO * O) is formed in the
// prologue and written for the dK/dV kernel.  Two tiles per trip (compile-time LDS buffer index).
// KSPLIT (D = 128): built for 2 waves per SIMD, the key tile's two 32-key halves run one after the
// other (one half's S / dP accumulators live) and the LSE is a per-element subtraction: 256 VGPRs
// (380 and one wave before), backward +11 % at Llama-3 8B's shape (profiles/r5_attn_ab_occupancy.json;
// at D = 64 the 2-wave build measured neutral).
template <int D, bool CAUSAL>
__global__ __launch_bounds__(kThreads, D == 128 ? 2 : 1) void attn_bwd_dq_kernel(const MadnnAttnArgs a) {
  constexpr int DS = D / 16, DB = D / 32;
  constexpr bool ACCD = D == 64, KSPLIT = D == 128;
  // K and V stages in one block: after the loop the column-sum epilogue reuses all of it as a
  // [128 rows][D] fp32 image (4 * 64 * D bf16 = 128 * D fp32)
  __shared__ __attribute__((aligned(16))) uint16_t sKV[4][kTile * D];
  uint16_t(*sK)[kTile * D] = sKV;
  uint16_t(*sV)[kTile * D] = sKV + 2;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, l32 = lane & 31, hh = lane >> 5;
  const int nqb = (a.S + kRowsWG - 1) / kRowsWG;
  int qblk, b, h;
  map_block(nqb, a.H, CAUSAL, qblk, b, h);
  const int hk = h / (a.H / a.Hkv);
  const int q0w = qblk * kRowsWG + wave * 32;
  const int qrow = q0w + l32;
  const int qc = min(qrow, a.S - 1);
  bf16x8 qf[DS], df[DS];
  // delta = rowsum(dO * O) of this lane's query row, from the dO fragments it holds anyway plus the
  // matching O halves (the two lane halves hh = 0/1 own alternate 8-column chunks); written out for
  // the dK/dV kernel that follows (no separate delta pass)
  float dl = 0.f;
  {
    const uint16_t* qp = a.q + b * a.q_sb + h * a.q_sh + (int64_t)qc * a.q_ss;
    const uint16_t* dp = a.dout + b * a.o_sb + h * a.o_sh + (int64_t)qc * a.o_ss;
    const uint16_t* op = a.o + b * a.o_sb + h * a.o_sh + (int64_t)qc * a.o_ss;
#pragma unroll
    for (int s = 0; s < DS; ++s) {
      qf[s] = scale_bf16x8(*reinterpret_cast<const bf16x8*>(qp + 16 * s + 8 * hh), -a.scale_log2);
      df[s] = *reinterpret_cast<const bf16x8*>(dp + 16 * s + 8 * hh);
      const bf16x8 ov = *reinterpret_cast<const bf16x8*>(op + 16 * s + 8 * hh);
#pragma unroll
      for (int j = 0; j < 8; ++j) dl = fmaf(static_cast<float>(df[s][j]), static_cast<float>(ov[j]), dl);
    }
    dl += __shfl_xor(dl, 32, kWave);
  }
  const int64_t srow = ((int64_t)b * a.H + h) * a.S + qc;
  const float lse = a.lse[srow];
  const f32x16 lse16 = splat16(lse);
  if (hh == 0 && qrow < a.S) a.delta[srow] = dl;
  const uint16_t* kb_ = a.k + b * a.k_sb + hk * a.k_sh;
  const uint16_t* vb_ = a.v + b * a.v_sb + hk * a.v_sh;
  f32x16 dq[DB];
#pragma unroll
  for (int d = 0; d < DB; ++d) dq[d] = zero16();
  f32x16 ndl;
#pragma unroll
  for (int r = 0; r < 16; ++r) ndl[r] = -dl;
  const int kv_end = CAUSAL ? min(a.S, qblk * kRowsWG + kRowsWG) : a.S;
  const int ntiles = (kv_end + kTile - 1) / kTile;
  TileStage<D, true> stk, stv;
  stk.load(kb_, a.k_ss, 0, a.S, tid);
  stv.load(vb_, a.v_ss, 0, a.S, tid);
  stk.store(sK[0], tid);
  stv.store(sV[0], tid);
  __syncthreads();
  int t = 0;
  auto tile = [&](auto curc) {
    constexpr int cur = decltype(curc)::value;
    const bool more = t + 1 < ntiles;
    if (more) {
      stk.load(kb_, a.k_ss, (t + 1) * kTile, a.S, tid);
      stv.load(vb_, a.v_ss, (t + 1) * kTile, a.S, tid);
    }
    const int k0 = t * kTile;
    if (KSPLIT && (!CAUSAL || k0 <= q0w + 31)) {
      // one 32-key half at a time: S, dP, dS and its dQ products, so only one half's accumulators live
      const bool edge = (k0 + kTile > a.S) || (CAUSAL && k0 + kTile - 1 > q0w);
      const int lim = (CAUSAL ? min(qrow, a.S - 1) : a.S - 1) - k0 - 4 * hh;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        f32x16 sc = zero16(), dp = zero16();
#pragma unroll
        for (int s = 0; s < DS; ++s) {
          sc = mfma(lds_row<D>(sK[cur], kb * 32 + l32, 2 * s + hh), qf[s], sc);
          dp = mfma(lds_row<D>(sV[cur], kb * 32 + l32, 2 * s + hh), df[s], dp);
        }
        if (edge) {
#pragma unroll
          for (int r = 0; r < 16; ++r) sc[r] = (kb * 32 + acc_row(r, 0) <= lim) ? sc[r] : __builtin_inff();
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) sc[r] = ex2(-sc[r] - lse) * (dp[r] - dl);
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const bf16x8 sf = pack_acc(sc, s);
#pragma unroll
          for (int d = 0; d < DB; ++d) dq[d] = mfma(lds_tr<D>(sK[cur], kb * 32 + 16 * s, d * 32, lane), sf, dq[d]);
        }
      }
    } else if (!CAUSAL || k0 <= q0w + 31) {
      f32x16 sc[2], dp[2];
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        sc[kb] = lse16;
        dp[kb] = ACCD ? ndl : zero16();
#pragma unroll
        for (int s = 0; s < DS; ++s) {
          sc[kb] = mfma(lds_row<D>(sK[cur], kb * 32 + l32, 2 * s + hh), qf[s], sc[kb]);
          dp[kb] = mfma(lds_row<D>(sV[cur], kb * 32 + l32, 2 * s + hh), df[s], dp[kb]);
        }
      }
      // masking as one wave-uniform block on the scores (exp2(-inf) = 0): interior tiles run
      // none of it (a per-element `if` costs an exec-mask branch per element)
      if ((k0 + kTile > a.S) || (CAUSAL && k0 + kTile - 1 > q0w)) {
        // key = k0 + off + 4 hh with off = kb*32 + acc_row(r, 0) a compile-time constant: the mask is
        // one compare of that constant against a per-lane limit (acc = +inf: p = 0)
        const int lim = (CAUSAL ? min(qrow, a.S - 1) : a.S - 1) - k0 - 4 * hh;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
          for (int r = 0; r < 16; ++r) sc[kb][r] = (kb * 32 + acc_row(r, 0) <= lim) ? sc[kb][r] : __builtin_inff();
        }
      }
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = ex2(-sc[kb][r]);
          sc[kb][r] = ACCD ? p * dp[kb][r] : p * (dp[kb][r] - dl);
        }
      }
      // dQ^T[d][q] += sum_key K[key][d] dS^T[key][q]
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const bf16x8 sf = pack_acc(sc[kb], s);
#pragma unroll
          for (int d = 0; d < DB; ++d) dq[d] = mfma(lds_tr<D>(sK[cur], kb * 32 + 16 * s, d * 32, lane), sf, dq[d]);
        }
      }
    }
    if (more) {
      stk.store(sK[cur ^ 1], tid);
      stv.store(sV[cur ^ 1], tid);
    }
    __syncthreads();
    ++t;
  };
  while (t + 1 < ntiles) {
    tile(std::integral_constant<int, 0>{});
    tile(std::integral_constant<int, 1>{});
  }
  if (t < ntiles) tile(std::integral_constant<int, 0>{});
  if (qrow < a.S) {
    uint16_t* qp = a.dq + b * a.dq_sb + h * a.dq_sh + (int64_t)qrow * a.dq_ss;
    const float sc = a.scale;
#pragma unroll
    for (int d = 0; d < DB; ++d) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        store4_bf16(qp + d * 32 + 8 * g + 4 * hh, dq[d][4 * g] * sc, dq[d][4 * g + 1] * sc, dq[d][4 * g + 2] * sc,
                    dq[d][4 * g + 3] * sc);
      }
    }
  }
  if (a.cpart != nullptr) {
    // column sums of the stored (bf16-rounded) dq over this workgroup's 128 query rows: every lane
    // writes its row (4 consecutive columns per 16-B chunk; chunk index XOR row & 15 so the 32 rows
    // of a half-wave spread over the banks) into the K/V block as [128][D] fp32, then D threads
    // each sum one column (shuffle trees cost ~75 us per launch at GPT-2 medium's shape)
    float* red = reinterpret_cast<float*>(&sKV[0][0]);
    const int row = wave * 32 + l32;
#pragma unroll
    for (int d = 0; d < DB; ++d) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        f32x4 v;
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = qrow < a.S ? bf16_to_f32(f32_to_bf16(dq[d][4 * g + i] * a.scale)) : 0.f;
        const int chunk = (d * 8 + 2 * g + hh) ^ (row & 15);
        *reinterpret_cast<f32x4*>(red + row * D + 4 * chunk) = v;
      }
    }
    __syncthreads();
    if (tid < D) {
      float s = 0.f;
#pragma unroll 8
      for (int r = 0; r < kRowsWG; ++r) s += red[r * D + 4 * ((tid >> 2) ^ (r & 15)) + (tid & 3)];
      const int64_t C = (int64_t)(a.H + 2 * a.Hkv) * D;
      a.cpart[((int64_t)b * nqb + qblk) * C + (int64_t)h * D + tid] = s;
    }
  }
}

// ----------------------------------------------------------- LDS-DMA tile staging (D = 64)

__device__ __forceinline__ int swzf64(int row) { return (((row >> 1) & 1) << 2) | ((row >> 2) & 3); }

// A [64][64] bf16 tile -> the swz<64> LDS image by LDS-DMA (global_load_lds_dwordx4).  Wave w of 4
// issues pieces 2w and 2w+1 (1 KiB = 8 rows each).  The image is lane-linear, so the XOR swizzle sits
// on the SOURCE address (cdna_hip_programming.md rule 21): lane L of piece i fetches row 8i + L/8,
// 16-B chunk (L % 8) ^ f(row).  Whole tiles only (S % 64 == 0: the launcher falls back to the
// register-staged kernels otherwise).  No staging registers and no ds_write pass: the tile lands in
// LDS while the wave computes, which is what lets the ring run two tiles ahead (the register-staged
// loop waited for each tile's global latency at its end: 48 % of the dK/dV kernel's wave time in
// s_waitcnt / barriers, profiles/r5_attn_pmc.md).  (buffer_load ... lds would range-check the tail,
// but hipcc then drains vmcnt before every later ds_read: LDS-DMA through the global path it does not.)
struct DmaTile64 {
  int o0, o1;  // this lane's source element offsets within the tile (pieces 2w, 2w+1)
  __device__ __forceinline__ void init(int wave, int lane, int64_t ld) {
    const int r0 = 16 * wave + (lane >> 3), r1 = r0 + 8;
    o0 = (int)((int64_t)r0 * ld + 8 * ((lane & 7) ^ swzf64(r0)));
    o1 = (int)((int64_t)r1 * ld + 8 * ((lane & 7) ^ swzf64(r1)));
  }
  __device__ __forceinline__ void issue(const uint16_t* base, int64_t ld, int row0, uint16_t* tile, int wave) const {
    const uint16_t* src = base + (int64_t)row0 * ld;
    char* t = reinterpret_cast<char*>(tile) + 2 * wave * 1024;
    glds16((const void*)(src + o0), (lds_void*)t);
    glds16((const void*)(src + o1), (lds_void*)(t + 1024));
  }
};

// 64 fp32 row statistics (LSE / delta of a query tile) -> LDS by one wave: one dword per lane
__device__ __forceinline__ void dma_stats(const float* arr, float* dst) {
  glds4((const void*)(arr + (threadIdx.x & 63)), (lds_void*)dst);
}

__device__ __forceinline__ void raw_barrier() {
  // an LDS-DMA is a pending LDS write on the VM counter: __syncthreads() would drain it (vmcnt(0))
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// dK / dV with D = 64 on a 3-stage LDS-DMA ring (Q, dO, LSE and delta of query tile it + 2 are in
// flight while tile it is computed).  Row constants as the initial accumulators, straight from LDS:
// the S accumulators start at +LSE against the -c prescaled K (acc = LSE - S', p = exp2(-acc)), the
// dP accumulators at +delta against a NEGATED V^T operand (a sign flip of the 8 loop-invariant V
// fragments in the prologue), so acc = delta - dP and dS = (-P) * acc, the negations free source
// modifiers -- neither row statistic costs VALU.
template <bool CAUSAL>
__global__ __launch_bounds__(kThreads) void attn_bwd_dkdv_dma_kernel(const MadnnAttnArgs a) {
  constexpr int D = 64, DS = D / 16, DB = D / 32;
  constexpr int kTileEl = kTile * D;
  // ONE LDS array (a second __shared__ object can make hipcc drain vmcnt before LDS reads:
  // cdna_hip_programming.md §5 'Projection GEMM' item 4a): Q[3] dO[3] tiles, LSE[3] delta[3], red
  __shared__ __attribute__((aligned(16))) uint16_t smem[6 * kTileEl + 6 * 2 * kTile + 8 * D * 2];
  uint16_t* const sQ = smem;
  uint16_t* const sO = smem + 3 * kTileEl;
  float* const sL = reinterpret_cast<float*>(smem + 6 * kTileEl);
  float* const sD = sL + 3 * kTile;
  float* const red = sD + 3 * kTile;  // [4][2 D]
  const int tid = threadIdx.x, lane = tid & 63, l32 = lane & 31, hh = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nkb = (a.S + kRowsWG - 1) / kRowsWG;
  int kblk, b, hk;
  map_block(nkb, a.Hkv, false, kblk, b, hk);
  const int G = a.H / a.Hkv;
  const int k0w = kblk * kRowsWG + wave * 32;
  const int krow = k0w + l32;
  const int kc = min(krow, a.S - 1);
  bf16x8 kf[DS], vf[DS];
  {
    const uint16_t* kp = a.k + b * a.k_sb + hk * a.k_sh + (int64_t)kc * a.k_ss;
    const uint16_t* vp = a.v + b * a.v_sb + hk * a.v_sh + (int64_t)kc * a.v_ss;
#pragma unroll
    for (int s = 0; s < DS; ++s) {
      kf[s] = scale_bf16x8(*reinterpret_cast<const bf16x8*>(kp + 16 * s + 8 * hh), -a.scale_log2);
      u32x4 v = *reinterpret_cast<const u32x4*>(vp + 16 * s + 8 * hh);
      v ^= u32x4{0x80008000u, 0x80008000u, 0x80008000u, 0x80008000u};  // -V (bf16 sign bits)
      vf[s] = __builtin_bit_cast(bf16x8, v);
    }
  }
  f32x16 dk[DB], dv[DB];
#pragma unroll
  for (int d = 0; d < DB; ++d) {
    dk[d] = zero16();
    dv[d] = zero16();
  }
  const int t0 = CAUSAL ? (kblk * kRowsWG) / kTile : 0;
  const int nt = (a.S + kTile - 1) / kTile - t0;
  const int total = G * nt;
  DmaTile64 gq, go;
  gq.init(wave, lane, a.q_ss);
  go.init(wave, lane, a.o_ss);
  // the issue cursor (query head offset, query tile) runs two tiles ahead of the compute cursor
  int iss_h = 0, iss_t = 0;
  auto issue = [&](int buf) {
    const int hq = hk * G + iss_h, q0 = (t0 + iss_t) * kTile;
    gq.issue(a.q + b * a.q_sb + hq * a.q_sh, a.q_ss, q0, sQ + buf * kTileEl, wave);
    go.issue(a.dout + b * a.o_sb + hq * a.o_sh, a.o_ss, q0, sO + buf * kTileEl, wave);
    if (wave < 2) {
      const int64_t so = ((int64_t)b * a.H + hq) * a.S + q0;
      dma_stats((wave == 0 ? a.lse : a.delta) + so, (wave == 0 ? sL : sD) + buf * kTile);
    }
    if (++iss_t == nt) {
      iss_t = 0;
      ++iss_h;
    }
  };
  // per-wave DMA instructions per tile (Q 2 + dO 2, + 1 statistics row on waves 0 / 1)
  auto wait_all_but_one_tile = [&]() {
    if (wave < 2) {
      asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    }
  };
  if (total > 0) issue(0);
  if (total > 1) {
    issue(1);
    wait_all_but_one_tile();
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  raw_barrier();
  int it = 0, cur_t = 0;
  auto tile = [&](auto curc) {
    constexpr int cur = decltype(curc)::value;
    if (it + 2 < total) issue((cur + 2) % 3);
    const int q0 = (t0 + cur_t) * kTile;
    if (++cur_t == nt) cur_t = 0;
    const uint16_t* tq = sQ + cur * kTileEl;
    const uint16_t* to = sO + cur * kTileEl;
    const float* tl = sL + cur * kTile;
    const float* td = sD + cur * kTile;
    if (!CAUSAL || q0 + kTile - 1 >= k0w) {
      f32x16 sc[2], dp[2];
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          sc[qb][r] = tl[qb * 32 + acc_row(r, hh)];
          dp[qb][r] = td[qb * 32 + acc_row(r, hh)];
        }
#pragma unroll
        for (int s = 0; s < DS; ++s) {
          sc[qb] = mfma(lds_row<D>(tq, qb * 32 + l32, 2 * s + hh), kf[s], sc[qb]);
          dp[qb] = mfma(lds_row<D>(to, qb * 32 + l32, 2 * s + hh), vf[s], dp[qb]);
        }
      }
      if (CAUSAL && q0 < k0w + 31) {  // diagonal tile: one compare per element against a per-lane limit
        const int lo = krow - q0 - 4 * hh;
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) {
#pragma unroll
          for (int r = 0; r < 16; ++r) sc[qb][r] = (qb * 32 + acc_row(r, 0) >= lo) ? sc[qb][r] : __builtin_inff();
        }
      }
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = ex2(-sc[qb][r]);
          sc[qb][r] = p;
          dp[qb][r] = (-p) * dp[qb][r];
        }
      }
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const bf16x8 pf = pack_acc(sc[qb], s);
          const bf16x8 sf = pack_acc(dp[qb], s);
#pragma unroll
          for (int d = 0; d < DB; ++d) {
            dv[d] = mfma(pf, lds_tr<D>(to, qb * 32 + 16 * s, d * 32, lane), dv[d]);
            dk[d] = mfma(sf, lds_tr<D>(tq, qb * 32 + 16 * s, d * 32, lane), dk[d]);
          }
        }
      }
    }
    // tile it + 1 has landed (tile it + 2 may stay in flight); every wave's reads of this tile
    // retire before the barrier, after which tile it + 3 may be issued into its stage
    if (it + 2 < total) {
      wait_all_but_one_tile();
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    raw_barrier();
    ++it;
  };
  while (it < total) {
    tile(std::integral_constant<int, 0>{});
    if (it < total) tile(std::integral_constant<int, 1>{});
    if (it < total) tile(std::integral_constant<int, 2>{});
  }
  // lane holds dK/dV[key = k0w + acc_row(r, hh)][d = 32*db + l32]
  uint16_t* kp = a.dk + b * a.dk_sb + hk * a.dk_sh;
  uint16_t* vp = a.dv + b * a.dv_sb + hk * a.dv_sh;
  float ck[DB], cv[DB];
#pragma unroll
  for (int d = 0; d < DB; ++d) ck[d] = cv[d] = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int key = k0w + acc_row(r, hh);
    if (key < a.S) {
#pragma unroll
      for (int d = 0; d < DB; ++d) {
        const unsigned short kb16 = f32_to_bf16(dk[d][r] * a.scale), vb16 = f32_to_bf16(dv[d][r]);
        kp[(int64_t)key * a.dk_ss + d * 32 + l32] = kb16;
        vp[(int64_t)key * a.dv_ss + d * 32 + l32] = vb16;
        ck[d] += bf16_to_f32(kb16);
        cv[d] += bf16_to_f32(vb16);
      }
    }
  }
  if (a.cpart != nullptr) {
#pragma unroll
    for (int d = 0; d < DB; ++d) {
      ck[d] += __shfl_xor(ck[d], 32);
      cv[d] += __shfl_xor(cv[d], 32);
      if (hh == 0) {
        red[wave * 2 * D + d * 32 + l32] = ck[d];
        red[wave * 2 * D + D + d * 32 + l32] = cv[d];
      }
    }
    __syncthreads();
    if (tid < 2 * D) {
      const float s = red[tid] + red[2 * D + tid] + red[4 * D + tid] + red[6 * D + tid];
      const int64_t C = (int64_t)(a.H + 2 * a.Hkv) * D;
      const int64_t col = (int64_t)a.H * D + (tid < D ? (int64_t)hk * D + tid : (int64_t)(a.Hkv + hk) * D + tid - D);
      a.cpart[((int64_t)b * nkb + kblk) * C + col] = s;
    }
  }
}

// The K / V key-tile ring of the D = 64 forward kernel (a dQ kernel on the same ring measured
// bitwise-equal and no faster, profiles/r5_attn_ab_fwd_dq_dma.json, and was dropped): tile t + 2 is issued into
// stage (t + 2) % 3 at the start of tile t (that stage last held tile t - 1, whose reads every wave
// retired before the barrier that ended it); at the end of tile t each wave waits until at most its
// own 4 DMA instructions of tile t + 2 are outstanding (tile t + 1 landed), then the barrier.
struct KVRing64 {
  static constexpr int kTileEl = kTile * 64;
  DmaTile64 gk, gv;
  const uint16_t *kb, *vb;
  int64_t kld, vld;
  uint16_t* sK;  // [3][kTileEl]
  uint16_t* sV;  // [3][kTileEl]
  int wave, ntiles;
  __device__ __forceinline__ void init(const uint16_t* kb_, int64_t kld_, const uint16_t* vb_, int64_t vld_,
                                       uint16_t* sK_, uint16_t* sV_, int wave_, int lane, int ntiles_) {
    kb = kb_, vb = vb_, kld = kld_, vld = vld_, sK = sK_, sV = sV_, wave = wave_, ntiles = ntiles_;
    gk.init(wave, lane, kld);
    gv.init(wave, lane, vld);
  }
  __device__ __forceinline__ void issue(int t, int buf) const {
    gk.issue(kb, kld, t * kTile, sK + buf * kTileEl, wave);
    gv.issue(vb, vld, t * kTile, sV + buf * kTileEl, wave);
  }
  __device__ __forceinline__ void prologue() const {
    if (ntiles > 0) issue(0, 0);
    if (ntiles > 1) {
      issue(1, 1);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    raw_barrier();
  }
  __device__ __forceinline__ void tile_start(int t, int cur) const {
    if (t + 2 < ntiles) issue(t + 2, (cur + 2) % 3);
  }
  __device__ __forceinline__ void tile_end(int t) const {
    if (t + 2 < ntiles) {
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    raw_barrier();
  }
};

// forward, D = 64, on the K / V LDS-DMA ring (numerics as attn_fwd_kernel<64, CAUSAL>)
template <bool CAUSAL>
__global__ __launch_bounds__(kThreads) void attn_fwd_dma_kernel(const MadnnAttnArgs a) {
  constexpr int D = 64, DS = D / 16, DB = D / 32;
  __shared__ __attribute__((aligned(16))) uint16_t smem[6 * kTile * D];
  const int tid = threadIdx.x, lane = tid & 63, l32 = lane & 31, hh = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nqb = (a.S + kRowsWG - 1) / kRowsWG;
  int qblk, b, h;
  map_block(nqb, a.H, CAUSAL, qblk, b, h);
  const int hk = h / (a.H / a.Hkv);
  const int q0w = qblk * kRowsWG + wave * 32;
  const int qrow = q0w + l32;
  bf16x8 qf[DS];
  {
    const uint16_t* qp = a.q + b * a.q_sb + h * a.q_sh + (int64_t)min(qrow, a.S - 1) * a.q_ss;
#pragma unroll
    for (int s = 0; s < DS; ++s) qf[s] = scale_bf16x8(*reinterpret_cast<const bf16x8*>(qp + 16 * s + 8 * hh), -a.scale_log2);
  }
  // retire the Q loads here: waited for lazily at first use, the compiler's counted wait would
  // land inside the key loop and (DMA being invisible to it) drain the ring every tile
#pragma unroll
  for (int s = 0; s < DS; ++s) asm volatile("" ::"v"(qf[s]));
  f32x16 o[DB];
#pragma unroll
  for (int d = 0; d < DB; ++d) o[d] = zero16();
  float m = kNegBig, mi = 0.f, l = 0.f;
  f32x16 mref = zero16();
  const int kv_end = CAUSAL ? min(a.S, qblk * kRowsWG + kRowsWG) : a.S;
  KVRing64 ring;
  ring.init(a.k + b * a.k_sb + hk * a.k_sh, a.k_ss, a.v + b * a.v_sb + hk * a.v_sh, a.v_ss, smem, smem + 3 * kTile * D,
            wave, lane, kv_end / kTile);
  ring.prologue();
  int t = 0;
  auto tile = [&](auto curc) {
    constexpr int cur = decltype(curc)::value;
    ring.tile_start(t, cur);
    const uint16_t* tk = ring.sK + cur * KVRing64::kTileEl;
    const uint16_t* tv = ring.sV + cur * KVRing64::kTileEl;
    const int k0 = t * kTile;
    if (!CAUSAL || k0 <= q0w + 31) {
      f32x16 sc[2];
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        sc[kb] = mref;
#pragma unroll
        for (int s = 0; s < DS; ++s) sc[kb] = mfma(lds_row<D>(tk, kb * 32 + l32, 2 * s + hh), qf[s], sc[kb]);
      }
      if (CAUSAL && k0 + kTile - 1 > q0w) {
        const int lim = qrow - k0 - 4 * hh;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
          for (int r = 0; r < 16; ++r) sc[kb][r] = kb * 32 + acc_row(r, 0) <= lim ? sc[kb][r] : __builtin_inff();
        }
      }
      softmax_tile<DB>(sc, o, m, mi, l, mref);
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const bf16x8 pf = pack_acc(sc[kb], s);
#pragma unroll
          for (int d = 0; d < DB; ++d) o[d] = mfma(lds_tr<D>(tv, kb * 32 + 16 * s, d * 32, lane), pf, o[d]);
        }
      }
    }
    ring.tile_end(t);
    ++t;
  };
  while (t < ring.ntiles) {
    tile(std::integral_constant<int, 0>{});
    if (t < ring.ntiles) tile(std::integral_constant<int, 1>{});
    if (t < ring.ntiles) tile(std::integral_constant<int, 2>{});
  }
  const float lt = l + __shfl_xor(l, 32);
  const float inv = lt > 0.f ? 1.f / lt : 0.f;
  if (qrow < a.S) {
    uint16_t* op = a.o + b * a.o_sb + h * a.o_sh + (int64_t)qrow * a.o_ss;
#pragma unroll
    for (int d = 0; d < DB; ++d) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        store4_bf16(op + d * 32 + 8 * g + 4 * hh, o[d][4 * g] * inv, o[d][4 * g + 1] * inv, o[d][4 * g + 2] * inv,
                    o[d][4 * g + 3] * inv);
      }
    }
    if (hh == 0) a.lse[((int64_t)b * a.H + h) * a.S + qrow] = m + log2f(lt);
  }
}

// --------------------------------------------------------------- backward: dK, dV
// Register-staged dK / dV (D = 128, or a sequence length that is not a multiple of the 64-row
// tile).  ACCD (D = 64): the tile's -delta rows are read from LDS straight into the dP accumulators
// before their MFMAs (dS = P * acc: no VALU for delta; -8 % at D = 128, profiles/
// r4_ab_attn_valu_trees.log).  The LSE stays a per-element subtraction here: started in the S
// accumulators as in the DMA kernel, the extra LDS reads made hipcc wait on the next tile's staging
// loads inside the MFMA chain (backward +40 %).  Two tiles per trip (compile-time LDS buffer index).
template <int D, bool CAUSAL>
__global__ __launch_bounds__(kThreads) void attn_bwd_dkdv_kernel(const MadnnAttnArgs a) {
  constexpr int DS = D / 16, DB = D / 32;
  constexpr bool ACCD = D == 64;
  __shared__ __attribute__((aligned(16))) uint16_t sQ[2][kTile * D];
  __shared__ __attribute__((aligned(16))) uint16_t sO[2][kTile * D];  // dO
  __shared__ float sL[2][kTile], sD[2][kTile];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, l32 = lane & 31, hh = lane >> 5;
  const int nkb = (a.S + kRowsWG - 1) / kRowsWG;
  int kblk, b, hk;
  map_block(nkb, a.Hkv, false, kblk, b, hk);  // causal: block 0 (longest) first already
  const int G = a.H / a.Hkv;
  const int k0w = kblk * kRowsWG + wave * 32;
  const int krow = k0w + l32;
  const int kc = min(krow, a.S - 1);
  // K^T / V^T as the B operand of S = Q.K^T / dP = dO.V^T: lane holds K[krow][16s + 8hh + j]
  bf16x8 kf[DS], vf[DS];
  {
    const uint16_t* kp = a.k + b * a.k_sb + hk * a.k_sh + (int64_t)kc * a.k_ss;
    const uint16_t* vp = a.v + b * a.v_sb + hk * a.v_sh + (int64_t)kc * a.v_ss;
#pragma unroll
    for (int s = 0; s < DS; ++s) {
      kf[s] = *reinterpret_cast<const bf16x8*>(kp + 16 * s + 8 * hh);
      vf[s] = *reinterpret_cast<const bf16x8*>(vp + 16 * s + 8 * hh);
    }
  }
  f32x16 dk[DB], dv[DB];
#pragma unroll
  for (int d = 0; d < DB; ++d) {
    dk[d] = zero16();
    dv[d] = zero16();
  }
  const int t0 = CAUSAL ? (kblk * kRowsWG) / kTile : 0;
  const int nt = (a.S + kTile - 1) / kTile - t0;
  const int total = G * nt;
  // tile `it` = (query head hk*G + it / nt, query tile t0 + it % nt); the loop walks it with two
  // counters instead of a per-tile integer division
  auto src = [&](int hq_i, int t_i, const uint16_t*& qp, const uint16_t*& dp, int& q0, int& hq) {
    hq = hk * G + hq_i;
    q0 = (t0 + t_i) * kTile;
    qp = a.q + b * a.q_sb + hq * a.q_sh;
    dp = a.dout + b * a.o_sb + hq * a.o_sh;
  };
  // the tile's LSE (threads 0..63) / delta (64..127) row statistics: fetched into a register
  // together with the tile's Q/dO loads and written to LDS with them, so their global-load
  // latency is covered by the tile's compute (a load stored right away exposes it every tile)
  // (one buffer load per lane of waves 0 / 1 through a descriptor that ends at row S: a row past the
  // end reads 0 for both -- harmless, since its Q and dO rows are zeros, so its P and dS terms
  // multiply zero operands)
  const int swave = __builtin_amdgcn_readfirstlane(wave);  // wave-uniform to the compiler
  auto fetch_stats = [&](int hq, int q0) -> float {
    float v = 0.f;
    if (swave < 2) {
      const float* arr = (swave == 0 ? a.lse : a.delta) + ((int64_t)b * a.H + hq) * a.S + q0;
      const __amdgpu_buffer_rsrc_t rsrc =
          __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(arr), 0, max(a.S - q0, 0) * 4, 0x00020000);
      v = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc, lane * 4, 0, 0));
      if (ACCD && swave == 1) v = -v;
    }
    return v;
  };
  auto put_stats = [&](float v, int buf) {
    if (tid < kTile) {
      sL[buf][tid] = v;
    } else if (tid < 2 * kTile) {
      sD[buf][tid - kTile] = v;
    }
  };
  TileStage<D, true> stq, sto;
  if (total > 0) {
    const uint16_t *qp, *dp;
    int q0, hq;
    src(0, 0, qp, dp, q0, hq);
    stq.load(qp, a.q_ss, q0, a.S, tid);
    sto.load(dp, a.o_ss, q0, a.S, tid);
    stq.store(sQ[0], tid);
    sto.store(sO[0], tid);
    put_stats(fetch_stats(hq, q0), 0);
  }
  __syncthreads();
  int cur_t = 0, nxt_h = 0, nxt_t = 0;  // this tile's query-tile index; the next tile's (head, tile)
  // two tiles per trip with the LDS buffer index a compile-time constant, so the buffer base folds
  // into the ds_read immediate offsets instead of costing a VALU op per read address
  int it = 0;
  auto tile = [&](auto curc) {
    constexpr int cur = decltype(curc)::value;
    const bool more = it + 1 < total;
    if (++nxt_t == nt) {
      nxt_t = 0;
      ++nxt_h;
    }
    float stat_next = 0.f;
    if (more) {
      const uint16_t *qp, *dp;
      int q0n, hqn;
      src(nxt_h, nxt_t, qp, dp, q0n, hqn);
      stq.load(qp, a.q_ss, q0n, a.S, tid);
      sto.load(dp, a.o_ss, q0n, a.S, tid);
      stat_next = fetch_stats(hqn, q0n);
    }
    const int q0 = (t0 + cur_t) * kTile;
    cur_t = nxt_t;
    if (!CAUSAL || q0 + kTile - 1 >= k0w) {
      f32x16 sc[2], dp[2];
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        sc[qb] = zero16();
        if constexpr (ACCD) {
#pragma unroll
          for (int r = 0; r < 16; ++r) dp[qb][r] = sD[cur][qb * 32 + acc_row(r, hh)];
        } else {
          dp[qb] = zero16();
        }
#pragma unroll
        for (int s = 0; s < DS; ++s) {
          sc[qb] = mfma(lds_row<D>(sQ[cur], qb * 32 + l32, 2 * s + hh), kf[s], sc[qb]);
          dp[qb] = mfma(lds_row<D>(sO[cur], qb * 32 + l32, 2 * s + hh), vf[s], dp[qb]);
        }
      }
      if (CAUSAL && q0 < k0w + 31) {  // diagonal tile: one wave-uniform masking block
        const int lo = krow - q0 - 4 * hh;  // query offset qb*32 + acc_row(r, 0) must reach it
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) {
#pragma unroll
          for (int r = 0; r < 16; ++r) sc[qb][r] = (qb * 32 + acc_row(r, 0) >= lo) ? sc[qb][r] : -__builtin_inff();
        }
      }
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int qi = qb * 32 + acc_row(r, hh);
          const float p = ex2(fmaf(sc[qb][r], a.scale_log2, -sL[cur][qi]));
          sc[qb][r] = p;
          dp[qb][r] = ACCD ? p * dp[qb][r] : p * (dp[qb][r] - sD[cur][qi]);
        }
      }
      // dV[key][d] += sum_q P[q][key] dO[q][d];  dK[key][d] += sum_q dS[q][key] Q[q][d]
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const bf16x8 pf = pack_acc(sc[qb], s);
          const bf16x8 sf = pack_acc(dp[qb], s);
#pragma unroll
          for (int d = 0; d < DB; ++d) {
            dv[d] = mfma(pf, lds_tr<D>(sO[cur], qb * 32 + 16 * s, d * 32, lane), dv[d]);
            dk[d] = mfma(sf, lds_tr<D>(sQ[cur], qb * 32 + 16 * s, d * 32, lane), dk[d]);
          }
        }
      }
    }
    if (more) {
      stq.store(sQ[cur ^ 1], tid);
      sto.store(sO[cur ^ 1], tid);
      put_stats(stat_next, cur ^ 1);
    }
    __syncthreads();
    ++it;
  };
  while (it + 1 < total) {
    tile(std::integral_constant<int, 0>{});
    tile(std::integral_constant<int, 1>{});
  }
  if (it < total) tile(std::integral_constant<int, 0>{});
  // lane holds dK/dV[key = k0w + acc_row(r, hh)][d = 32*db + l32]
  uint16_t* kp = a.dk + b * a.dk_sb + hk * a.dk_sh;
  uint16_t* vp = a.dv + b * a.dv_sb + hk * a.dv_sh;
  float ck[DB], cv[DB];  // this lane's column sums over its 16 keys (cpart)
#pragma unroll
  for (int d = 0; d < DB; ++d) ck[d] = cv[d] = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int key = k0w + acc_row(r, hh);
    if (key < a.S) {
#pragma unroll
      for (int d = 0; d < DB; ++d) {
        const unsigned short kb16 = f32_to_bf16(dk[d][r] * a.scale), vb16 = f32_to_bf16(dv[d][r]);
        kp[(int64_t)key * a.dk_ss + d * 32 + l32] = kb16;
        vp[(int64_t)key * a.dv_ss + d * 32 + l32] = vb16;
        ck[d] += bf16_to_f32(kb16);
        cv[d] += bf16_to_f32(vb16);
      }
    }
  }
  if (a.cpart != nullptr) {
    // + the partner half-wave (same columns, the other keys), then the 4 waves through LDS
    __shared__ float red[4][2 * D];
#pragma unroll
    for (int d = 0; d < DB; ++d) {
      ck[d] += __shfl_xor(ck[d], 32);
      cv[d] += __shfl_xor(cv[d], 32);
      if (hh == 0) {
        red[wave][d * 32 + l32] = ck[d];
        red[wave][D + d * 32 + l32] = cv[d];
      }
    }
    __syncthreads();
    if (tid < 2 * D) {
      const float s = red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid];
      const int64_t C = (int64_t)(a.H + 2 * a.Hkv) * D;
      const int64_t col = (int64_t)a.H * D + (tid < D ? (int64_t)hk * D + tid : (int64_t)(a.Hkv + hk) * D + tid - D);
      a.cpart[((int64_t)b * nkb + kblk) * C + col] = s;
    }
  }
}

// colsum[c] = sum_r cpart[r][c]: the dQKV column sums over all B * S rows
__global__ __launch_bounds__(1024) void attn_colsum_finalize_kernel(const float* __restrict__ cpart, int R, int C,
                                                                    void* __restrict__ out, int out_bf16) {
  __shared__ float red[32][33];
  const int c = threadIdx.x % 32, sl = threadIdx.x / 32;
  const int n = blockIdx.x * 32 + c;
  float acc = 0.f;
  if (n < C)
    for (int r = sl; r < R; r += 32) acc += cpart[(int64_t)r * C + n];
  red[sl][c] = acc;
  __syncthreads();
  if (sl == 0 && n < C) {
    float tot = 0.f;
    for (int q = 0; q < 32; ++q) tot += red[q][c];
    if (out_bf16) {
      static_cast<uint16_t*>(out)[n] = f32_to_bf16(tot);
    } else {
      static_cast<float*>(out)[n] = tot;
    }
  }
}

// madnn_attn_tune keys (A/B and the tests of the register-staged fallbacks, which serve sequence
// lengths that are not multiples of 64 and D = 128): 7 = D = 64 dK/dV on the 3-stage LDS-DMA ring,
// 8 = D = 64 forward on the K / V LDS-DMA ring (0: the register-staged kernels)
int g_attn_dkdv_dma = 1;
int g_attn_fwd_dma = 1;

template <int D, bool CAUSAL>
hipError_t launch_fwd(const MadnnAttnArgs& a, hipStream_t st) {
  const int nqb = (a.S + kRowsWG - 1) / kRowsWG;
  if (D == 64 && g_attn_fwd_dma && a.S % kTile == 0) {
    hipLaunchKernelGGL((attn_fwd_dma_kernel<CAUSAL>), dim3(nqb * a.B * a.H), dim3(kThreads), 0, st, a);
  } else {
    hipLaunchKernelGGL((attn_fwd_kernel<D, CAUSAL>), dim3(nqb * a.B * a.H), dim3(kThreads), 0, st, a);
  }
  return hipGetLastError();
}

template <int D, bool CAUSAL>
hipError_t launch_bwd(const MadnnAttnArgs& a, hipStream_t st) {
  const int nb = (a.S + kRowsWG - 1) / kRowsWG;
  hipLaunchKernelGGL((attn_bwd_dq_kernel<D, CAUSAL>), dim3(nb * a.B * a.H), dim3(kThreads), 0, st, a);
  MADNN_HIP_CHECK(hipGetLastError());
  if (D == 64 && g_attn_dkdv_dma && a.S % kTile == 0) {
    hipLaunchKernelGGL((attn_bwd_dkdv_dma_kernel<CAUSAL>), dim3(nb * a.B * a.Hkv), dim3(kThreads), 0, st, a);
  } else {
    hipLaunchKernelGGL((attn_bwd_dkdv_kernel<D, CAUSAL>), dim3(nb * a.B * a.Hkv), dim3(kThreads), 0, st, a);
  }
  return hipGetLastError();
}

}  // namespace attn
}  // namespace madnn

using namespace madnn::attn;

extern "C" {

int madnn_attn_supported(int D) { return D == 64 || D == 128; }

// knob keys 7 / 8 (see g_attn_dkdv_dma); returns the previous value, -1 for an unknown key
int madnn_attn_tune(int key, int value) {
  int* slot = key == 7 ? &g_attn_dkdv_dma : key == 8 ? &g_attn_fwd_dma : nullptr;
  if (slot == nullptr) return -1;
  const int old = *slot;
  *slot = value ? 1 : 0;
  return old;
}

hipError_t madnn_attn_fwd(const MadnnAttnArgs* a, int D, int causal, hipStream_t st) {
  if (a->S <= 0 || a->B <= 0) return hipSuccess;
  if (D == 64) return causal ? launch_fwd<64, true>(*a, st) : launch_fwd<64, false>(*a, st);
  if (D == 128) return causal ? launch_fwd<128, true>(*a, st) : launch_fwd<128, false>(*a, st);
  return hipErrorInvalidValue;
}

// rows of MadnnAttnArgs::cpart: one per (batch, 128-row sequence block)
int64_t madnn_attn_colsum_rows(int B, int S) { return (int64_t)B * ((S + kRowsWG - 1) / kRowsWG); }

hipError_t madnn_attn_colsum_finalize(const float* cpart, int64_t R, int64_t C, void* out, int out_bf16,
                                      hipStream_t st) {
  if (R <= 0 || C <= 0) return hipSuccess;
  hipLaunchKernelGGL(attn_colsum_finalize_kernel, dim3((unsigned)((C + 31) / 32)), dim3(1024), 0, st, cpart, (int)R,
                     (int)C, out, out_bf16);
  return hipGetLastError();
}

hipError_t madnn_attn_bwd(const MadnnAttnArgs* a, int D, int causal, hipStream_t st) {
  if (a->S <= 0 || a->B <= 0) return hipSuccess;
  if (D == 64) return causal ? launch_bwd<64, true>(*a, st) : launch_bwd<64, false>(*a, st);
  if (D == 128) return causal ? launch_bwd<128, true>(*a, st) : launch_bwd<128, false>(*a, st);
  return hipErrorInvalidValue;
}

}  // extern "C"
