// K12 — bf16 MFMA GEMM for gfx950 with fused epilogues: the Linear layers of the transformer
// models (forward with bias / tanh-GELU / residual, data gradient with in-place accumulation).
//
// Why: the GPT-2 medium step is ~2/3 hipBLASLt GEMMs (profiles/r2_bench_all_rehearsal1.md),
// which run at ~1.15 PF/s on MI355X (madnn/tuning/hw_mi355x.json, 8192^3), and hipBLASLt
// refuses its GELU/bias epilogues at GPT-2's 65536-row shapes ("no algorithm"), so the GELU
// is a separate HBM pass (K11 gelu_fwd).  This kernel follows the CDNA4 structure that
// reaches ~1.3-1.5 PF/s in plain HIP (cdna_hip_programming.md §5 "The 256^2 8-phase
// template"): a 256x256 output tile per 512-thread workgroup, LDS-DMA staging with counted
// vmcnt waits that never drain in the main loop, and two wave groups one barrier apart so
// that one group's LDS reads and DMA issue overlap the other group's MFMAs on the same SIMD.
//
// Problem: Out[j][i] = sum_k A(i, k) B(k, j)   (bf16 in, fp32 accumulate, bf16 out)
//   * "row" operand memory: X[x][k], k contiguous (ds_read_b128 fragments);
//   * "col" operand memory: X[k][x], x contiguous (ds_read_b64_tr_b16 fragments).
//   linear forward : i = out feature (A = W[n][k], row), j = token (B = X[m][k], row)
//   linear dgrad   : i = in feature  (A = W[n][k] read as [k=n][i], col), j = token (B = dY, row)
//   linear wgrad   : i = in feature  (A = X[m][k], col), j = out feature (B = dY[m][n], col); the
//                    reduction runs over the TOKENS (65536 for GPT-2 at 64 x 1024), the output is
//                    small (a few 256^2 tiles), so the reduction is split over `splits` workgroups
//                    per tile: fp32 partial slabs + one streaming reduce (wgrad_reduce_kernel).
// i sits on the accumulator rows, j on the MFMA lane, so a lane owns 4 consecutive i of one
// output row (the same orientation as K9, conv.hip).
//
// Geometry: 8 waves = 2 groups (wr: i half of the tile) x 4 (wc: 64-column j quarter);
// each wave owns a 128 x 64 block of D = 8 x 4 v_mfma_f32_16x16x32_bf16 accumulators
// (128 VGPRs).  K steps of 64.  LDS = 2 stages x 4 half-tiles (A i-half 0/1, B j-half 0/1)
// of 128 x 64 bf16 = 128 KiB, one workgroup per CU.
//
// Schedule (per K tile: 4 phases, one per 64x32 quadrant of the wave block):
//   phase q: LOAD  = ds_read this quadrant's new fragments + issue one half-tile of DMA
//            s_barrier
//            MFMA  = 16 MFMAs (setprio 1)
//            s_barrier
//   Q0 reads A(i 0..63) + B(j 0..31), Q1 B(j 32..63), Q2 A(i 64..127), Q3 nothing.
//   Group 1 issues one extra barrier first, so its LOAD segments coincide with group 0's MFMA
//   segments and vice versa.
//   DMA: half-tile H = 4u + p of K tile u, parts in the order B0, B1, A0, A1, is issued in
//   global phase H-6; the Q3 LOAD of K tile t waits vmcnt(4) (the two B half-tiles of K tile
//   t+2 issued in Q2/Q3 stay in flight), so K tile t+1 has landed before barrier 8(t+1) and
//   is read after it by both groups; each half-tile gets >= 2 phases of latency cover.
//   WAR: B half-tiles are last read in Q1, A half-tiles in Q2; both LOADs end with
//   lgkmcnt(0) before their barrier, so every wave's reads of a half-tile retire before the
//   barrier that precedes the first DMA into it (B: phase 4u-6, A: phase 4u-4 for K tile u).
//   Derivation in docs/ARCHITECTURE.md (K12).
// LDS images are lane-linear (DMA writes base + 16*lane); the XOR swizzles of mfma.h are
// applied to the per-lane SOURCE address and to the read address (cdna_hip_programming.md
// rule 21), so both fragment kinds read conflict-free.
//
// Epilogue: bias added in fp32, rounded to bf16 once, the tile staged through LDS as bf16
// [256 j][256 i] (XOR-swizzled 16-B chunks) and stored as full 512-B rows; in that row pass:
// aux = pre-activation store, tanh-GELU, residual add (fp32 add of two bf16, one rounding:
// the same two roundings as the unfused PyTorch graph).
#include <type_traits>
#include <utility>

#include "k12.h"

namespace madnn {
namespace gemm {

using namespace mf;
using namespace k12;

struct Args {
  const uint16_t* a;
  const uint16_t* b;
  uint16_t* out;
  const uint16_t* res;  // epilogue: out = y + res (same [j][i] layout, row stride ldr), or null
  const void* bias;     // [I] fp32 (bias_f32) or bf16, or null
  uint16_t* aux;        // pre-activation store (row stride ldx), or null
  int64_t lda, ldb, ldo, ldr, ldx;
  int64_t I, J, K;
  int i_tiles, j_tiles;
  int bias_f32, act;    // act: 0 none, 1 tanh-GELU, 2 erf-GELU
  float* ws;            // split-K: fp32 partial slabs [splits][J][I] (null: bf16 epilogue)
  int splits;           // workgroups per output tile along the reduction
  int64_t kper;         // reduction elements per split (multiple of kBK)
};

template <bool A_COL, bool B_COL>
__global__ __launch_bounds__(kThreads) void gemm_kernel(const Args p) {
  __shared__ __attribute__((aligned(16))) uint16_t smem[kLds];
  const int tid = threadIdx.x, lane = tid & 63, hh = lane >> 5, l32 = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;

  // XCD-grouped logical id (bijective remap), i tile fastest
  int wid = blockIdx.x;
  {
    const int n = gridDim.x, x = wid % 8, q8 = n / 8, r8 = n % 8;
    wid = (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + wid / 8;
  }
  const int ntile = p.i_tiles * p.j_tiles;
  const int split = wid / ntile;
  wid -= split * ntile;
  const int it = wid % p.i_tiles, jt = wid / p.i_tiles;
  const int64_t i0 = (int64_t)it * kT, j0 = (int64_t)jt * kT;
  const int64_t kbeg = (int64_t)split * p.kper;
  const int64_t klen = p.K - kbeg < p.kper ? p.K - kbeg : p.kper;
  const int nk = (int)(klen / kBK);
  const int total = 4 * nk;  // half-tiles

  // per-lane DMA offsets: part (0,1: A halves; 2,3: B halves) x 2 instructions per wave
  int64_t off[4][2];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int inst = 2 * wave + e;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      off[h][e] = dma_offset<A_COL>(inst, lane, p.lda, i0 + 128 * h, p.I);
      off[2 + h][e] = dma_offset<B_COL>(inst, lane, p.ldb, j0 + 128 * h, p.J);
    }
  }
  // issue half-tile H: 2 DMA instructions per lane into stage (H/4)&1; H%4 = 0,1: B halves,
  // 2,3: A halves (the B halves are consumed first, so they are restaged first)
  auto stage = [&](int H) {
    const int u = H >> 2, part = (H + 2) & 3;
    const int64_t k0 = kbeg + (int64_t)u * kBK;
    const uint16_t* base;
    if (part < 2) {
      const int64_t x0 = i0 + 128 * part;
      base = A_COL ? p.a + k0 * p.lda + x0 : p.a + x0 * p.lda + k0;
    } else {
      const int64_t x0 = j0 + 128 * (part - 2);
      base = B_COL ? p.b + k0 * p.ldb + x0 : p.b + x0 * p.ldb + k0;
    }
    uint16_t* dst = smem + (u & 1) * kStage + part * kHalf + (2 * wave) * 512;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      int64_t o;
      // static index into off[][] (rule 20: no runtime-indexed register arrays)
      if (part == 0) o = off[0][e];
      else if (part == 1) o = off[1][e];
      else if (part == 2) o = off[2][e];
      else o = off[3][e];
      glds16((const void*)(base + o), (lds_void*)(dst + e * 512));
    }
  };

  // accumulators: ac4[8 i-blocks of 16][4 j-blocks of 16] of v_mfma_f32_16x16x32_bf16 (128 VGPRs)
  // (a 32x32x16 variant with the same schedule measured 6-12 % slower at every GPT-2 / square shape,
  // profiles/r5_gemm_ab_b128_asm_dma.json "k12m32", and was removed)
  f32x4 ac4[8][4];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) ac4[a][b] = zero4();

  // prologue: half-tiles 0..5 (K tile 0 + the B halves of K tile 1)
#pragma unroll
  for (int H = 0; H < 6; ++H)
    if (H < total) stage(H);
  if (total > 4) {
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  barrier();
  if (wr == 1) barrier();  // group 1 runs one barrier behind

  bf16x8 af[2][4], bf0[4], bf1[4];
  const int bcol = (wc & 1) * 64;
  {
    // 4-phase schedule, 16 MFMAs per phase: af[a][s] = i-block a (of 4) x k-step s (of 2),
    // bf0 / bf1 [c][s] = j-blocks 0,1 / 2,3 of the wave's 64 columns
    for (int t = 0; t < nk; ++t) {
      const uint16_t* sa = smem + (t & 1) * kStage + wr * kHalf;
      const uint16_t* sb = smem + (t & 1) * kStage + (2 + (wc >> 1)) * kHalf;
      const int P = 4 * t;
      // ---- Q0: A rows 0..63, B cols 0..31
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
        for (int c = 0; c < 2; ++c) bf0[2 * c + s2] = frag16<B_COL>(sb, s2, bcol + 16 * c, lane);
#pragma unroll
        for (int a = 0; a < 4; ++a) af[a >> 1][2 * (a & 1) + s2] = frag16<A_COL>(sa, s2, 16 * a, lane);
      }
      if (P + 6 < total) stage(P + 6);
      barrier();
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int c = 0; c < 2; ++c)
            ac4[a][c] = mfma16(af[a >> 1][2 * (a & 1) + s2], bf0[2 * c + s2], ac4[a][c]);
      __builtin_amdgcn_s_setprio(0);
      barrier();
      // ---- Q1: B cols 32..63
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int c = 0; c < 2; ++c) bf1[2 * c + s2] = frag16<B_COL>(sb, s2, bcol + 32 + 16 * c, lane);
      if (P + 7 < total) stage(P + 7);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the B half-tiles' last reads
      barrier();
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int c = 0; c < 2; ++c)
            ac4[a][2 + c] = mfma16(af[a >> 1][2 * (a & 1) + s2], bf1[2 * c + s2], ac4[a][2 + c]);
      __builtin_amdgcn_s_setprio(0);
      barrier();
      // ---- Q2: A rows 64..127 (the stage's last reads: retire them before the barrier)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int a = 0; a < 4; ++a) af[a >> 1][2 * (a & 1) + s2] = frag16<A_COL>(sa, s2, 64 + 16 * a, lane);
      if (P + 8 < total) stage(P + 8);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the A half-tiles' last reads
      barrier();
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int c = 0; c < 2; ++c)
            ac4[4 + a][2 + c] = mfma16(af[a >> 1][2 * (a & 1) + s2], bf1[2 * c + s2], ac4[4 + a][2 + c]);
      __builtin_amdgcn_s_setprio(0);
      barrier();
      // ---- Q3: no reads; retire K tile t+1's DMA (the B halves of K tile t+2 stay in flight)
      if (P + 9 < total) {
        stage(P + 9);
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      } else if (P + 8 < total) {
        asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      barrier();
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int c = 0; c < 2; ++c)
            ac4[4 + a][c] = mfma16(af[a >> 1][2 * (a & 1) + s2], bf0[2 * c + s2], ac4[4 + a][c]);
      __builtin_amdgcn_s_setprio(0);
      barrier();
    }
  }
  if (wr == 0) barrier();  // balance the stagger: every wave has now passed the same barriers

  // every lane owns groups of 4 consecutive i of one j: visit them as (il, jl, v[4])
  auto for_each_group = [&](auto&& fn) {
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) fn(wr * 128 + a * 16 + 4 * (lane >> 4), wc * 64 + b * 16 + (lane & 15), ac4[a][b]);
  };

  if (p.ws != nullptr) {
    // split-K partial: fp32 straight from the accumulators, 4 consecutive i (16 B) per lane
    float* slab = p.ws + (int64_t)split * p.J * p.I;
    for_each_group([&](int il, int jl, const f32x4& v) {
      const int64_t ig = i0 + il, jg = j0 + jl;
      if (ig < p.I && jg < p.J) *reinterpret_cast<f32x4*>(slab + jg * p.I + ig) = v;
    });
    return;
  }

  // ---- epilogue: (acc + bias) -> bf16 -> LDS [256 j][256 i] -> rows
  char* ot = reinterpret_cast<char*>(smem);
  for_each_group([&](int il, int jl, const f32x4& v) {  // il: first of this lane's 4 i
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if (p.bias != nullptr) {
      const int64_t ig = i0 + il;
      if (ig < p.I) {
        if (p.bias_f32) {
          const f32x4 w = *reinterpret_cast<const f32x4*>(static_cast<const float*>(p.bias) + ig);
          bv[0] = w[0]; bv[1] = w[1]; bv[2] = w[2]; bv[3] = w[3];
        } else {
          const u32x2 w = *reinterpret_cast<const u32x2*>(static_cast<const uint16_t*>(p.bias) + ig);
          bv[0] = bf16_to_f32((unsigned short)(w[0] & 0xffffu));
          bv[1] = bf16_to_f32((unsigned short)(w[0] >> 16));
          bv[2] = bf16_to_f32((unsigned short)(w[1] & 0xffffu));
          bv[3] = bf16_to_f32((unsigned short)(w[1] >> 16));
        }
      }
    }
    const unsigned lo = (unsigned)f32_to_bf16(v[0] + bv[0]) | ((unsigned)f32_to_bf16(v[1] + bv[1]) << 16);
    const unsigned hi = (unsigned)f32_to_bf16(v[2] + bv[2]) | ((unsigned)f32_to_bf16(v[3] + bv[3]) << 16);
    *reinterpret_cast<u32x2*>(ot + jl * 512 + 16 * ((il >> 3) ^ (jl & 31)) + 8 * ((il >> 2) & 1)) = u32x2{lo, hi};
  });
  __syncthreads();
  const int c = tid & 31;
  const int64_t ig = i0 + 8 * c;
  if (ig < p.I) {
#pragma unroll 4
    for (int r = tid >> 5; r < kT; r += kThreads / 32) {
      const int64_t jg = j0 + r;
      if (jg >= p.J) break;
      u32x4 v = *reinterpret_cast<const u32x4*>(ot + r * 512 + 16 * (c ^ (r & 31)));
      if (p.aux != nullptr) *reinterpret_cast<u32x4*>(p.aux + jg * p.ldx + ig) = v;
      if (p.act != 0 || p.res != nullptr) {
        u32x4 rv = u32x4{0u, 0u, 0u, 0u};
        if (p.res != nullptr) rv = *reinterpret_cast<const u32x4*>(p.res + jg * p.ldr + ig);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float x0 = bf16_to_f32((unsigned short)(v[e] & 0xffffu));
          float x1 = bf16_to_f32((unsigned short)(v[e] >> 16));
          if (p.act == kGeluErf) {
            x0 = round_bf16(gelu_erf(x0));
            x1 = round_bf16(gelu_erf(x1));
          } else if (p.act == kGeluTanh) {
            x0 = round_bf16(gelu_tanh(x0));
            x1 = round_bf16(gelu_tanh(x1));
          }
          if (p.res != nullptr) {
            x0 += bf16_to_f32((unsigned short)(rv[e] & 0xffffu));
            x1 += bf16_to_f32((unsigned short)(rv[e] >> 16));
          }
          v[e] = (unsigned)f32_to_bf16(x0) | ((unsigned)f32_to_bf16(x1) << 16);
        }
      }
      *reinterpret_cast<u32x4*>(p.out + jg * p.ldo + ig) = v;
    }
  }
}

// out[e] = bf16(sum_s ws[s][e] (+ out[e])), 8 elements per lane, 16-B accesses
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ ws, uint16_t* out, int splits,
                                                           int64_t n, int accumulate) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * 8;
  for (int64_t e = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8; e < n; e += stride) {
    f32x4 lo = *reinterpret_cast<const f32x4*>(ws + e), hi = *reinterpret_cast<const f32x4*>(ws + e + 4);
    for (int q = 1; q < splits; ++q) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(ws + (int64_t)q * n + e);
      const f32x4 b = *reinterpret_cast<const f32x4*>(ws + (int64_t)q * n + e + 4);
      lo += a;
      hi += b;
    }
    if (accumulate) {
      const u32x4 o = *reinterpret_cast<const u32x4*>(out + e);
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        lo[2 * k] += bf16_to_f32((unsigned short)(o[k] & 0xffffu));
        lo[2 * k + 1] += bf16_to_f32((unsigned short)(o[k] >> 16));
        hi[2 * k] += bf16_to_f32((unsigned short)(o[2 + k] & 0xffffu));
        hi[2 * k + 1] += bf16_to_f32((unsigned short)(o[2 + k] >> 16));
      }
    }
    u32x4 v;
    v[0] = (unsigned)f32_to_bf16(lo[0]) | ((unsigned)f32_to_bf16(lo[1]) << 16);
    v[1] = (unsigned)f32_to_bf16(lo[2]) | ((unsigned)f32_to_bf16(lo[3]) << 16);
    v[2] = (unsigned)f32_to_bf16(hi[0]) | ((unsigned)f32_to_bf16(hi[1]) << 16);
    v[3] = (unsigned)f32_to_bf16(hi[2]) | ((unsigned)f32_to_bf16(hi[3]) << 16);
    *reinterpret_cast<u32x4*>(out + e) = v;
  }
}

// ---------------------------------------------------------------------------------------------
// K12W: the weight-gradient GEMM (both operands k-major: "col" images) at ONE wave per SIMD.
//
// Why (profiles/r5_gemm_pmc.md): K12's 8 waves own 128 x 64 blocks, so every bf16 fragment read
// from LDS feeds 4 (A) or 8 (B) MFMAs and each phase's reads must land inside the partner group's
// 256-cycle MFMA segment; the matrix cores idle ~12 points in its main loop.  Here 4 waves each own
// a 128 x 128 block -- 4 x 4 v_mfma_f32_32x32x16_bf16 accumulators, 256 registers: the
// accumulation registers of a lone wave -- every fragment feeds 4 MFMAs of 32 cycles, and a wave
// issues the NEXT phase's fragment reads between its own MFMAs (software pipelining inside the wave
// instead of across two wave groups).
//
// K tile (64 deep) = 4 phases, one per 16-deep k step ks: 4 A + 4 B fragments, 16 MFMAs; the
// fragments of phase ks + 1 are read during phase ks.
// LDS: the [64 k][128 x] swz<128> half-tile images of K12, laid out half-tile-major
// [A0 s0, A0 s1, A1 s0, A1 s1, B0 s0, ...] so that a wave's two stages of one operand sit within the
// 16-bit ds_read immediate of one address: every fragment read is one of 8 per-lane address
// registers per operand (4 x blocks x 2 row quads: the XOR swizzle is per lane) + an immediate.
// Each half-tile is split by k half (rows 0..31 = part K0: k steps 0, 1; rows 32..63 = part K1:
// k steps 2, 3; 8 of its 16 1-KiB DMA pieces each); wave w streams half-tile w (A0, A1, B0, B1).
//   reads: P3(t-1) -> ks 0 of tile t (K0); P0(t) -> ks 1 (K0); P1(t) -> ks 2 (K1); P2(t) -> ks 3 (K1).
//   P1(t): RAW for K1(t) + WAR for K0(t) (last read in P0): counted vmcnt + lgkmcnt(0) + barrier,
//          then K0(t + 2) is issued into the same stage (pieces 0..3 in P1, 4..7 in P2).
//   P3(t): RAW for K0(t + 1) + WAR for K1(t) (last read in P2), then K1(t + 2) (pieces 0..3 in P3,
//          4..7 in P0(t + 1)).
//   vmcnt(16) at both: a wave's pieces retire in issue order and two whole parts (16 pieces) were
//   issued after the one waited for by then.  Latency cover: >= 5 phases per piece.
//
// Issue schedule (one wave per SIMD: every non-MFMA instruction between two MFMAs is issue time of the
// only wave on the SIMD; MI355X_MICROARCH.md: <= 5 single-issue instructions hide per
// v_mfma_f32_32x32x16_bf16 gap, <= 3 ds_read_b64_tr_b16): the 16 MFMAs of a phase are pinned one per
// gap (sched_barrier) with
//   plain phase (P0, P2):   the next phase's 8 fragments (2 reads each) in gaps 0..7, DMA pieces 4..7
//                           in gaps 8, 10, 12, 14;
//   barrier phase (P1, P3): MFMAs 0..2 from registers, then vmcnt(16) + lgkmcnt(0) + barrier (the
//                           in-flight MFMA covers the wait), DMA pieces 0..3 in gaps 3, 5, 7, 9 and
//                           the 8 fragments in gaps 4, 6, 8, 10..14.
// A DMA piece is one 5-instruction statement (glds16_one: the saddr form, a wave-uniform SGPR base +
// a per-lane 32-bit offset, no 64-bit address VALU; M0 from the wave's LDS base + an immediate).
// Measured against the burst schedule it replaced (16 reads after the 4th MFMA, 8 seven-instruction
// DMA pieces after the barrier): GPT-2 c_fc weight gradient 937 -> 777-786 us (1.40 PF/s), LM head
// 12.2 -> 10.2-10.5 ms; the pinned schedule with two-piece statements in between
// (profiles/r6_k12w_spread_ab.json).  PMC (profiles/r6_k12w_pmc.md): MFMA busy 53 % (K12) / 76 %
// (pinned, two-piece) of the cycles at the 1.65-1.68 GHz the chip holds under this load.

// one LDS-DMA piece: 16 B per lane from a wave-uniform 64-bit base (SGPR pair) + a per-lane 32-bit
// byte offset to LDS bytes lds + O + 16 * lane (M0 written and restored inside the statement:
// common.h glds16)
template <unsigned O>
__device__ __forceinline__ void glds16_one(const void* sbase, unsigned lds, unsigned v) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_add_u32 m0, %2, %4\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %3, %1\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "s"(sbase), "s"(lds), "v"(v), "i"(O)
      : "memory", "scc");
}

template <bool A_COL, bool B_COL>
__global__ __launch_bounds__(256, 1) void gemm4_kernel(const Args p) {
  static_assert(A_COL && B_COL, "K12W: weight gradient (both operands k-major)");
  __shared__ __attribute__((aligned(16))) uint16_t smem[kLds];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;

  int wid = blockIdx.x;
  {
    const int n = gridDim.x, x = wid % 8, q8 = n / 8, r8 = n % 8;
    wid = (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + wid / 8;
  }
  const int ntile = p.i_tiles * p.j_tiles;
  const int split = wid / ntile;
  wid -= split * ntile;
  const int it = wid % p.i_tiles, jt = wid / p.i_tiles;
  const int64_t i0 = (int64_t)it * kT, j0 = (int64_t)jt * kT;
  const int64_t kbeg = (int64_t)split * p.kper;
  const int64_t klen = p.K - kbeg < p.kper ? p.K - kbeg : p.kper;
  const int nk = (int)(klen / kBK);

  // this wave's DMA half-tile (0, 1: A halves; 2, 3: B halves): 8 per-lane byte offsets (rows
  // 4e .. 4e + 3 of a 32-row part, relative to the part's first row, column 0: the clamped columns of a
  // ragged edge tile lie left of x0, and the saddr offset is unsigned) and the uniform part bases
  const bool isA = wave < 2;
  const uint16_t* const op = isA ? p.a : p.b;
  const int64_t ld = isA ? p.lda : p.ldb;
  const int64_t x0 = isA ? i0 + 128 * wave : j0 + 128 * (wave - 2);
  unsigned voff[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) voff[e] = (unsigned)(2 * (x0 + dma_offset<true>(e, lane, ld, x0, isA ? p.I : p.J)));
  const char* const gbase = reinterpret_cast<const char*>(op + kbeg * ld);
  const int64_t tbytes = (int64_t)kBK * ld * 2, pbytes = (int64_t)32 * ld * 2;
  const unsigned ldsw = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(smem + 2 * wave * kHalf));
  // piece e of part `part` of the K tile at tb (= gbase + t * tbytes) into stage ST: LDS bytes
  // (2w + ST) * 16 KiB + part * 8 KiB + e * 1 KiB
  auto dma1 = [&](const char* tb, auto st_c, auto part_c, auto e_c) {
    constexpr unsigned o = decltype(st_c)::value * kHalf * 2 + decltype(part_c)::value * 8192 + decltype(e_c)::value * 1024;
    glds16_one<o>(tb + decltype(part_c)::value * pbytes, ldsw, voff[decltype(e_c)::value]);
  };
  using C0 = std::integral_constant<int, 0>;
  using C1 = std::integral_constant<int, 1>;
  using C2 = std::integral_constant<int, 2>;
  using C3 = std::integral_constant<int, 3>;
  using C4 = std::integral_constant<int, 4>;
  using C5 = std::integral_constant<int, 5>;
  using C6 = std::integral_constant<int, 6>;
  using C7 = std::integral_constant<int, 7>;
  auto dma_half = [&](const char* tb, auto st_c, auto part_c, auto e0_c) {   // pieces e0 .. e0 + 3
    constexpr int e0 = decltype(e0_c)::value;
    dma1(tb, st_c, part_c, std::integral_constant<int, e0>{});
    dma1(tb, st_c, part_c, std::integral_constant<int, e0 + 1>{});
    dma1(tb, st_c, part_c, std::integral_constant<int, e0 + 2>{});
    dma1(tb, st_c, part_c, std::integral_constant<int, e0 + 3>{});
  };

  f32x16 ac[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) ac[a][b] = zero16();

  // per-lane LDS byte addresses of the 32x32x16 operand reads (mf::lds_col<128>: two
  // ds_read_b64_tr_b16, row quads hq = 0 / 1) of x block xb (32 columns):
  //   byte(st, ks, xb, hq) = st * 16 KiB + ks * 4 KiB + lanepart(hq) + 64 * (xb ^ (f(hq) >> 2))
  const int g = lane >> 4, i = lane & 15;
  unsigned adA[4][2], adB[4][2];
  {
    const unsigned baseA = (unsigned)(size_t)(smem + 2 * wr * kHalf);
    const unsigned baseB = (unsigned)(size_t)(smem + 2 * (2 + wc) * kHalf);
#pragma unroll
    for (int hq = 0; hq < 2; ++hq) {
      const int row = 8 * (g >> 1) + (i >> 2) + 4 * hq;
      const int f = ((row & 3) << 2) | ((row >> 2) & 3);
      const int cl = 2 * (g & 1) + ((i & 3) >> 1);
      const unsigned lanepart = (unsigned)(row * 256 + 16 * (cl ^ (f & 3)) + 8 * (i & 1));
#pragma unroll
      for (int xb = 0; xb < 4; ++xb) {
        const unsigned o = lanepart + 64u * (unsigned)(xb ^ (f >> 2));
        adA[xb][hq] = baseA + o;
        adB[xb][hq] = baseB + o;
      }
    }
  }
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  auto frag = [&](const unsigned (&ad)[2], auto st_c, auto ks_c) {
    constexpr int imm = decltype(st_c)::value * kHalf * 2 + decltype(ks_c)::value * 4096;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(size_t)(ad[0] + imm));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(size_t)(ad[1] + imm));
    const s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, r);
  };
  // fragment f of the next phase, in the order its first MFMAs consume them: A0, B0..B3, A1..A3
  auto rdf = [&](bf16x8 (&fa)[4], bf16x8 (&fb)[4], auto st_c, auto ks_c, int f) {
    if (f == 0) fa[0] = frag(adA[0], st_c, ks_c);
    else if (f < 5) {
      if (f == 1) fb[0] = frag(adB[0], st_c, ks_c);
      else if (f == 2) fb[1] = frag(adB[1], st_c, ks_c);
      else if (f == 3) fb[2] = frag(adB[2], st_c, ks_c);
      else fb[3] = frag(adB[3], st_c, ks_c);
    } else if (f == 5) fa[1] = frag(adA[1], st_c, ks_c);
    else if (f == 6) fa[2] = frag(adA[2], st_c, ks_c);
    else fa[3] = frag(adA[3], st_c, ks_c);
  };
  bf16x8 fa0[4], fb0[4], fa1[4], fb1[4];

  if (nk > 0) {
  // tiles 0 and 1, except pieces 4..7 of K1(1): those go out in P0 of tile 0, as every K1's second half
  const char* tbp = gbase + (int64_t)(nk > 1 ? 1 : 0) * tbytes;
  dma_half(gbase, C0{}, C0{}, C0{});
  dma_half(gbase, C0{}, C0{}, C4{});
  dma_half(gbase, C0{}, C1{}, C0{});
  dma_half(gbase, C0{}, C1{}, C4{});
  dma_half(tbp, C1{}, C0{}, C0{});
  dma_half(tbp, C1{}, C0{}, C4{});
  dma_half(tbp, C1{}, C1{}, C0{});
  asm volatile("s_waitcnt vmcnt(20)" ::: "memory");   // K0(0)
  barrier();
#pragma unroll
  for (int f = 0; f < 8; ++f) rdf(fa0, fb0, C0{}, C0{}, f);

  // plain phase: MFMAs on (fc, gc), the next fragments (stage NS, k step NK) into (fn, gn), pieces
  // 4..7 of part `part` of the K tile at tb into stage ST
  auto plain = [&](const bf16x8 (&fc)[4], const bf16x8 (&gc)[4], bf16x8 (&fn)[4], bf16x8 (&gn)[4], auto ns_c,
                   auto nk_c, const char* tb, auto st_c, auto part_c) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      ac[q >> 2][q & 3] = mf::mfma(fc[q >> 2], gc[q & 3], ac[q >> 2][q & 3]);
      if (q < 8) rdf(fn, gn, ns_c, nk_c, q);
      else if (q == 8) dma1(tb, st_c, part_c, C4{});
      else if (q == 10) dma1(tb, st_c, part_c, C5{});
      else if (q == 12) dma1(tb, st_c, part_c, C6{});
      else if (q == 14) dma1(tb, st_c, part_c, C7{});
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // barrier phase: the wait + barrier after MFMA 2, pieces 0..3 of part `part` of the K tile at tb
  // into stage ST in gaps 3, 5, 7, 9, the next fragments in the other gaps
  auto barred = [&](const bf16x8 (&fc)[4], const bf16x8 (&gc)[4], bf16x8 (&fn)[4], bf16x8 (&gn)[4], auto ns_c,
                    auto nk_c, const char* tb, auto st_c, auto part_c) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      ac[q >> 2][q & 3] = mf::mfma(fc[q >> 2], gc[q & 3], ac[q >> 2][q & 3]);
      if (q == 2) {
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        barrier();
      } else if (q == 3) dma1(tb, st_c, part_c, C0{});
      else if (q == 5) dma1(tb, st_c, part_c, C1{});
      else if (q == 7) dma1(tb, st_c, part_c, C2{});
      else if (q == 9) dma1(tb, st_c, part_c, C3{});
      else if (q == 4) rdf(fn, gn, ns_c, nk_c, 0);
      else if (q == 6) rdf(fn, gn, ns_c, nk_c, 1);
      else if (q == 8) rdf(fn, gn, ns_c, nk_c, 2);
      else if (q >= 10 && q <= 14) rdf(fn, gn, ns_c, nk_c, q - 7);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  auto ktile = [&](int t, auto st_c) {
    using ST = decltype(st_c);
    using NST = std::integral_constant<int, 1 - ST::value>;
    // the DMA base of K tile t + 2 (clamped), computed in the filler-free last gap of the previous phase
    const int t2 = t + 2 < nk ? t + 2 : nk - 1;
    const char* tb = gbase + (int64_t)t2 * tbytes;
    __builtin_amdgcn_sched_barrier(0);
    // P0 finishes K1 of the previous tile's t2 (tbp), P2 finishes K0(t + 2)
    plain(fa0, fb0, fa1, fb1, ST{}, C1{}, tbp, NST{}, C1{});  // P0: ks 0, reads ks 1 (K0)
    barred(fa1, fb1, fa0, fb0, ST{}, C2{}, tb, ST{}, C0{});   // P1: RAW K1(t), WAR K0(t) -> K0(t + 2)
    plain(fa0, fb0, fa1, fb1, ST{}, C3{}, tb, ST{}, C0{});    // P2: ks 2, reads ks 3 (K1)
    barred(fa1, fb1, fa0, fb0, NST{}, C0{}, tb, ST{}, C1{});  // P3: RAW K0(t + 1), WAR K1(t) -> K1(t + 2)
    tbp = tb;
  };
  int t = 0;
  for (; t + 1 < nk; t += 2) {
    ktile(t, C0{});
    ktile(t + 1, C1{});
  }
  if (t < nk) ktile(t, C0{});
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the clamped reloads
  }

  const int h = lane >> 5, l32 = lane & 31;
  auto for_each_group = [&](auto&& fn) {
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int m = 0; m < 4; ++m)
          fn(wr * 128 + 32 * a + 8 * m + 4 * h, wc * 128 + 32 * b + l32,
             f32x4{ac[a][b][4 * m], ac[a][b][4 * m + 1], ac[a][b][4 * m + 2], ac[a][b][4 * m + 3]});
  };
  if (p.ws != nullptr) {
    float* slab = p.ws + (int64_t)split * p.J * p.I;
    for_each_group([&](int il, int jl, const f32x4& v) {
      const int64_t ig = i0 + il, jg = j0 + jl;
      if (ig < p.I && jg < p.J) *reinterpret_cast<f32x4*>(slab + jg * p.I + ig) = v;
    });
    return;
  }
  for_each_group([&](int il, int jl, const f32x4& v) {
    const int64_t ig = i0 + il, jg = j0 + jl;
    if (ig < p.I && jg < p.J) {
      float w[4] = {v[0], v[1], v[2], v[3]};
      if (p.res != nullptr) {
        const u32x2 r = *reinterpret_cast<const u32x2*>(p.res + jg * p.ldr + ig);
        w[0] += bf16_to_f32((unsigned short)(r[0] & 0xffffu));
        w[1] += bf16_to_f32((unsigned short)(r[0] >> 16));
        w[2] += bf16_to_f32((unsigned short)(r[1] & 0xffffu));
        w[3] += bf16_to_f32((unsigned short)(r[1] >> 16));
      }
      const unsigned lo = (unsigned)f32_to_bf16(w[0]) | ((unsigned)f32_to_bf16(w[1]) << 16);
      const unsigned hi = (unsigned)f32_to_bf16(w[2]) | ((unsigned)f32_to_bf16(w[3]) << 16);
      *reinterpret_cast<u32x2*>(p.out + jg * p.ldo + ig) = u32x2{lo, hi};
    }
  });
}

// f(integral_constant<int, 0>) .. f(integral_constant<int, N - 1>): a compile-time loop (a 64-step
// `#pragma unroll` body this large stays a runtime loop, and its register arrays go to scratch)
template <class F, int... Q>
__device__ __forceinline__ void seq_impl(F&& f, std::integer_sequence<int, Q...>) {
  (f(std::integral_constant<int, Q>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void for_seq(F&& f) {
  seq_impl(f, std::make_integer_sequence<int, N>{});
}

// K12W on v_mfma_f32_16x16x32_bf16 (K12W16, madnn_linear_wgrad4h): the same 256x256 tile, one wave
// per SIMD owning 128 x 128 as 8 x 8 blocks of 16 x 16 (64 f32x4 accumulators, 256 AGPRs), the same
// LDS images / DMA pieces / counted waits; a K tile is 2 phases of one 32-deep k step each (64 MFMAs of
// 16 cycles), both behind a barrier (RAW for the part read during the phase, WAR for the part the
// phase's DMA refills).  Why: on random data the chip holds a higher clock on this shape at equal cycles
// per FLOP (MI355X_MICROARCH.md, DVFS give-back 7).
//   gap q of a phase: q == 2 wait + barrier; q = 3, 7, .., 31 one DMA piece; q = 4, 6, .., 34 the
//   next phase's fragment 0..15 (A0, B0..B7, A1..A7: the order its MFMAs consume them).
// v_mfma_f32_16x16x32_bf16 with the accumulator pinned to AGPRs: hipcc spreads 64 f32x4 accumulator
// tuples over both register files and shuffles them every iteration (v_accvgpr_read / write around the
// MFMAs); as an asm operand ("+a") every tuple stays in its AGPRs.  hipcc sees no MFMA here, so its
// result is read only after mfma_drain() (wait states for the last MFMAs' writes).
__device__ __forceinline__ void mfma16a(f32x4& c, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma_drain() {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
}

template <bool A_COL, bool B_COL>
__global__ __launch_bounds__(256, 1) void gemm4h_kernel(const Args p) {
  static_assert(A_COL && B_COL, "K12W: weight gradient (both operands k-major)");
  __shared__ __attribute__((aligned(16))) uint16_t smem[kLds];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;

  int wid = blockIdx.x;
  {
    const int n = gridDim.x, x = wid % 8, q8 = n / 8, r8 = n % 8;
    wid = (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + wid / 8;
  }
  const int ntile = p.i_tiles * p.j_tiles;
  const int split = wid / ntile;
  wid -= split * ntile;
  const int it = wid % p.i_tiles, jt = wid / p.i_tiles;
  const int64_t i0 = (int64_t)it * kT, j0 = (int64_t)jt * kT;
  const int64_t kbeg = (int64_t)split * p.kper;
  const int64_t klen = p.K - kbeg < p.kper ? p.K - kbeg : p.kper;
  const int nk = (int)(klen / kBK);

  const bool isA = wave < 2;
  const uint16_t* const op = isA ? p.a : p.b;
  const int64_t ld = isA ? p.lda : p.ldb;
  const int64_t x0 = isA ? i0 + 128 * wave : j0 + 128 * (wave - 2);
  unsigned voff[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) voff[e] = (unsigned)(2 * (x0 + dma_offset<true>(e, lane, ld, x0, isA ? p.I : p.J)));
  const char* const gbase = reinterpret_cast<const char*>(op + kbeg * ld);
  const int64_t tbytes = (int64_t)kBK * ld * 2, pbytes = (int64_t)32 * ld * 2;
  const unsigned ldsw = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(smem + 2 * wave * kHalf));
  auto dma1 = [&](const char* tb, auto st_c, auto part_c, auto e_c) {
    constexpr unsigned o = decltype(st_c)::value * kHalf * 2 + decltype(part_c)::value * 8192 + decltype(e_c)::value * 1024;
    glds16_one<o>(tb + decltype(part_c)::value * pbytes, ldsw, voff[decltype(e_c)::value]);
  };
  using C0 = std::integral_constant<int, 0>;
  using C1 = std::integral_constant<int, 1>;
  auto dma_part = [&](const char* tb, auto st_c, auto part_c) {
    dma1(tb, st_c, part_c, std::integral_constant<int, 0>{});
    dma1(tb, st_c, part_c, std::integral_constant<int, 1>{});
    dma1(tb, st_c, part_c, std::integral_constant<int, 2>{});
    dma1(tb, st_c, part_c, std::integral_constant<int, 3>{});
    dma1(tb, st_c, part_c, std::integral_constant<int, 4>{});
    dma1(tb, st_c, part_c, std::integral_constant<int, 5>{});
    dma1(tb, st_c, part_c, std::integral_constant<int, 6>{});
    dma1(tb, st_c, part_c, std::integral_constant<int, 7>{});
  };

  f32x4 ac[8][8];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) ac[a][b] = zero4();

  // per-lane LDS byte addresses of k12::frag16<true> reads of 16-column block x (of 8) of this wave's
  // A / B half-tile, row quad hq (lo / hi): byte(st, s, x, hq) = st * 16 KiB + s * 8 KiB + ad[x][hq]
  const int g = lane >> 4, i = lane & 15;
  unsigned adA[8][2], adB[8][2];
  {
    const unsigned baseA = (unsigned)(size_t)(smem + 2 * wr * kHalf);
    const unsigned baseB = (unsigned)(size_t)(smem + 2 * (2 + wc) * kHalf);
#pragma unroll
    for (int hq = 0; hq < 2; ++hq) {
      const int row = 8 * g + (i >> 2) + 4 * hq;
      const int f = ((row & 3) << 2) | ((row >> 2) & 3);
#pragma unroll
      for (int xb = 0; xb < 8; ++xb) {
        const int ch = 2 * xb + ((i & 3) >> 1);
        const unsigned o = (unsigned)(row * 256 + 16 * (ch ^ f) + 8 * (i & 1));
        adA[xb][hq] = baseA + o;
        adB[xb][hq] = baseB + o;
      }
    }
  }
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  auto frag = [&](const unsigned (&ad)[2], auto st_c, auto s_c) {
    constexpr int imm = decltype(st_c)::value * kHalf * 2 + decltype(s_c)::value * 8192;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(size_t)(ad[0] + imm));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(size_t)(ad[1] + imm));
    const s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, r);
  };
  bf16x8 fa0[8], fb0[8], fa1[8], fb1[8];

  if (nk > 0) {
  const char* const tb1 = gbase + (int64_t)(nk > 1 ? 1 : 0) * tbytes;
  dma_part(gbase, C0{}, C0{});
  dma_part(gbase, C0{}, C1{});
  dma_part(tb1, C1{}, C0{});
  dma_part(tb1, C1{}, C1{});
  asm volatile("s_waitcnt vmcnt(24)" ::: "memory");   // K0(0)
  barrier();
#pragma unroll
  for (int x = 0; x < 8; ++x) {
    fa0[x] = frag(adA[x], C0{}, C0{});
    fb0[x] = frag(adB[x], C0{}, C0{});
  }

  // one phase: 64 MFMAs on (fc, gc) in A-block-major order (all 16 fragments read in the previous
  // phase: the DMA of this phase refills the part they came from); after MFMA 2 the wait + barrier;
  // part `part` of the K tile at tb into stage ST; the next phase's fragments (stage NS, k step NSS)
  // into (fn, gn): A0, B0..B7, A1..A7, the order its MFMAs consume them
  auto phase = [&](const bf16x8 (&fc)[8], const bf16x8 (&gc)[8], bf16x8 (&fn)[8], bf16x8 (&gn)[8], auto ns_c,
                   auto nss_c, const char* tb, auto st_c, auto part_c) {
    for_seq<64>([&](auto q_c) {
      constexpr int q = decltype(q_c)::value;
      mfma16a(ac[q >> 3][q & 7], fc[q >> 3], gc[q & 7]);
      if constexpr (q == 2) {
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        barrier();
      }
      if constexpr (q >= 3 && q <= 31 && (q - 3) % 4 == 0)
        dma1(tb, st_c, part_c, std::integral_constant<int, (q - 3) / 4>{});
      if constexpr (q >= 4 && q <= 34 && (q & 1) == 0) {
        constexpr int f = (q - 4) >> 1;
        if constexpr (f == 0) fn[0] = frag(adA[0], ns_c, nss_c);
        else if constexpr (f <= 8) gn[f - 1] = frag(adB[f - 1], ns_c, nss_c);
        else fn[f - 8] = frag(adA[f - 8], ns_c, nss_c);
      }
      __builtin_amdgcn_sched_barrier(0);
    });
  };
  auto ktile = [&](int t, auto st_c) {
    using ST = decltype(st_c);
    using NST = std::integral_constant<int, 1 - ST::value>;
    const int t2 = t + 2 < nk ? t + 2 : nk - 1;
    const char* tb = gbase + (int64_t)t2 * tbytes;
    __builtin_amdgcn_sched_barrier(0);
    phase(fa0, fb0, fa1, fb1, ST{}, C1{}, tb, ST{}, C0{});    // P0: k step 0 (K0(t)); RAW K1(t), refill K0(t + 2)
    phase(fa1, fb1, fa0, fb0, NST{}, C0{}, tb, ST{}, C1{});   // P1: k step 1 (K1(t)); RAW K0(t + 1), refill K1(t + 2)
  };
  // nk is even (the host gives every split an even number of K tiles): no odd tail block, around
  // which hipcc would copy accumulators out of the AGPRs while the asm MFMAs are still writing them
  for (int t = 0; t < nk; t += 2) {
    ktile(t, C0{});
    ktile(t + 1, C1{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the clamped reloads
  mfma_drain();   // inside the branch: the join block after it may already copy accumulators
  }

  // accumulator (a, b) register r: i row wr*128 + 16a + 4(lane >> 4) + r, j col wc*128 + 16b + (lane & 15)
  const int ig4 = 4 * (lane >> 4), l16 = lane & 15;
  if (p.ws != nullptr) {
    float* slab = p.ws + (int64_t)split * p.J * p.I;
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        const int64_t ig = i0 + wr * 128 + 16 * a + ig4, jg = j0 + wc * 128 + 16 * b + l16;
        if (ig < p.I && jg < p.J) *reinterpret_cast<f32x4*>(slab + jg * p.I + ig) = ac[a][b];
      }
    return;
  }
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const int64_t ig = i0 + wr * 128 + 16 * a + ig4, jg = j0 + wc * 128 + 16 * b + l16;
      if (ig < p.I && jg < p.J) {
        const f32x4 v = ac[a][b];
        float w[4] = {v[0], v[1], v[2], v[3]};
        if (p.res != nullptr) {
          const u32x2 r = *reinterpret_cast<const u32x2*>(p.res + jg * p.ldr + ig);
          w[0] += bf16_to_f32((unsigned short)(r[0] & 0xffffu));
          w[1] += bf16_to_f32((unsigned short)(r[0] >> 16));
          w[2] += bf16_to_f32((unsigned short)(r[1] & 0xffffu));
          w[3] += bf16_to_f32((unsigned short)(r[1] >> 16));
        }
        const unsigned lo = (unsigned)f32_to_bf16(w[0]) | ((unsigned)f32_to_bf16(w[1]) << 16);
        const unsigned hi = (unsigned)f32_to_bf16(w[2]) | ((unsigned)f32_to_bf16(w[3]) << 16);
        *reinterpret_cast<u32x2*>(p.out + jg * p.ldo + ig) = u32x2{lo, hi};
      }
    }
}

template <bool A_COL, bool B_COL>
hipError_t launch(Args& p, hipStream_t s) {
  p.i_tiles = (int)((p.I + kT - 1) / kT);
  p.j_tiles = (int)((p.J + kT - 1) / kT);
  if (p.splits < 1) p.splits = 1;
  if (p.kper <= 0) p.kper = p.K;
  const int64_t grid = (int64_t)p.i_tiles * p.j_tiles * p.splits;
  if (grid > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL((gemm_kernel<A_COL, B_COL>), dim3((unsigned)grid), dim3(kThreads), 0, s, p);
  return hipGetLastError();
}

}  // namespace gemm
}  // namespace madnn

using namespace madnn::gemm;

extern "C" {

// Shapes K12 takes: reduction % 64 == 0, output features % 8 == 0, 16-B aligned rows, and
// 32-bit-safe per-lane DMA offsets.
int madnn_gemm_supported(int64_t I, int64_t J, int64_t K, int64_t lda, int64_t ldb) {
  if (I <= 0 || J <= 0 || K <= 0) return 0;
  if (K % kBK || I % 8 || lda % 8 || ldb % 8) return 0;
  return 1;
}

// Y[m][n] = X[m][k] W[n][k] (+ bias[n]) (-> gelu) (+ res[m][n]); aux (if given) = pre-activation
hipError_t madnn_linear_fwd(const void* x, const void* w, const void* bias, int bias_f32, const void* res,
                            void* y, void* aux, int act, int64_t M, int64_t N, int64_t K, hipStream_t s) {
  if (!madnn_gemm_supported(N, M, K, K, K)) return hipErrorInvalidValue;
  Args p{};
  p.a = static_cast<const uint16_t*>(w);
  p.lda = K;
  p.b = static_cast<const uint16_t*>(x);
  p.ldb = K;
  p.out = static_cast<uint16_t*>(y);
  p.ldo = N;
  p.res = static_cast<const uint16_t*>(res);
  p.ldr = N;
  p.bias = bias;
  p.bias_f32 = bias_f32;
  p.aux = static_cast<uint16_t*>(aux);
  p.ldx = N;
  p.act = act;
  p.I = N;
  p.J = M;
  p.K = K;
  return launch<false, false>(p, s);
}

// dX[m][k] = dY[m][n] W[n][k] (+ res[m][k]; res may alias dX for in-place accumulation)
hipError_t madnn_linear_dgrad(const void* dy, const void* w, const void* res, void* dx, int64_t M, int64_t N,
                              int64_t K, hipStream_t s) {
  if (!madnn_gemm_supported(K, M, N, K, N)) return hipErrorInvalidValue;
  Args p{};
  p.a = static_cast<const uint16_t*>(w);  // A[i = k][kk = n] = W[n][k]: column memory
  p.lda = K;
  p.b = static_cast<const uint16_t*>(dy);  // B[kk = n][j = m] = dY[m][n]: row memory
  p.ldb = N;
  p.out = static_cast<uint16_t*>(dx);
  p.ldo = K;
  p.res = static_cast<const uint16_t*>(res);
  p.ldr = K;
  p.I = K;
  p.J = M;
  p.K = N;
  return launch<true, false>(p, s);
}

// Workgroups per output tile for a weight gradient: 256 CUs, one 128-KiB-LDS workgroup per CU.
// Model: rounds of 256 workgroups x k-steps per split (~1.8 us per 256^2 x 64 step at ~1.2 PF/s)
// + the fp32 slab round trip (splits x I x J x 8 B at ~5 TB/s); splits keep >= 8 k-steps each.
int madnn_wgrad_splits(int64_t M, int64_t N, int64_t K) {
  const int64_t tiles = ((K + kT - 1) / kT) * ((N + kT - 1) / kT);
  const int64_t nk = M / kBK;
  int best = 1;
  double best_t = 1e30;
  for (int sp = 1; sp <= 256; ++sp) {  // ResNet's 1x1 convs: 4-16 tiles over 10^5-10^6 pixels
    if (nk / sp < 8) break;
    const int64_t kper_steps = (nk + sp - 1) / sp;
    const int64_t rounds = (tiles * sp + 255) / 256;
    const double t = rounds * kper_steps * 1.8 + (sp > 1 ? sp * (double)N * K * 8.0 / 5.0e6 : 0.0);
    if (t < best_t * 0.98) {
      best_t = t;
      best = sp;
    }
  }
  return best;
}

// dW[n][k] (+)= sum_m dY[m][n] X[m][k] (bf16 out; with accumulate the existing dW is added).
// ws: splits x N x K fp32 workspace when splits > 1 (madnn_wgrad_splits), else unused.
hipError_t madnn_linear_wgrad(const void* dy, const void* x, void* dw, float* ws, int splits, int accumulate,
                              int64_t M, int64_t N, int64_t K, hipStream_t s) {
  if (M % kBK || !madnn_gemm_supported(K, N, M, K, N)) return hipErrorInvalidValue;
  if (splits > 1 && ws == nullptr) return hipErrorInvalidValue;
  Args p{};
  p.a = static_cast<const uint16_t*>(x);   // A[i = k][kk = m] = X[m][k]: column memory
  p.lda = K;
  p.b = static_cast<const uint16_t*>(dy);  // B[kk = m][j = n] = dY[m][n]: column memory
  p.ldb = N;
  p.out = static_cast<uint16_t*>(dw);
  p.ldo = K;
  p.res = accumulate && splits <= 1 ? static_cast<const uint16_t*>(dw) : nullptr;
  p.ldr = K;
  p.I = K;
  p.J = N;
  p.K = M;
  p.splits = splits > 1 ? splits : 1;
  const int64_t nk = M / kBK;
  p.kper = ((nk + p.splits - 1) / p.splits) * kBK;
  p.ws = p.splits > 1 ? ws : nullptr;
  hipError_t e = launch<true, true>(p, s);
  if (e != hipSuccess || p.splits == 1) return e;
  const int64_t n = N * K;
  int64_t blocks = (n / 8 + 255) / 256;
  blocks = blocks < 1 ? 1 : (blocks > 2048 ? 2048 : blocks);
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, s, ws, static_cast<uint16_t*>(dw),
                     p.splits, n, accumulate);
  return hipGetLastError();
}

// K12W weight gradient (same contract as madnn_linear_wgrad; the split count from madnn_wgrad_splits).
// mfma16: the v_mfma_f32_16x16x32_bf16 form (gemm4h_kernel), which needs an even number of K tiles per
// split (M a multiple of 128; every split gets an even share).
static hipError_t linear_wgrad4_launch(const void* dy, const void* x, void* dw, float* ws, int splits, int accumulate,
                                       int64_t M, int64_t N, int64_t K, hipStream_t s, bool mfma16) {
  if (M % kBK || !madnn_gemm_supported(K, N, M, K, N)) return hipErrorInvalidValue;
  if (mfma16 && M % (2 * kBK)) return hipErrorInvalidValue;
  if (splits > 1 && ws == nullptr) return hipErrorInvalidValue;
  Args p{};
  p.a = static_cast<const uint16_t*>(x);
  p.lda = K;
  p.b = static_cast<const uint16_t*>(dy);
  p.ldb = N;
  p.out = static_cast<uint16_t*>(dw);
  p.ldo = K;
  p.res = accumulate && splits <= 1 ? static_cast<const uint16_t*>(dw) : nullptr;
  p.ldr = K;
  p.I = K;
  p.J = N;
  p.K = M;
  p.splits = splits > 1 ? splits : 1;
  if (mfma16) {
    const int64_t pairs = M / (2 * kBK);
    p.kper = ((pairs + p.splits - 1) / p.splits) * 2 * kBK;
  } else {
    const int64_t nk = M / kBK;
    p.kper = ((nk + p.splits - 1) / p.splits) * kBK;
  }
  p.ws = p.splits > 1 ? ws : nullptr;
  p.i_tiles = (int)((p.I + kT - 1) / kT);
  p.j_tiles = (int)((p.J + kT - 1) / kT);
  const int64_t grid = (int64_t)p.i_tiles * p.j_tiles * p.splits;
  if (grid > 0x7fffffff) return hipErrorInvalidValue;
  // saddr DMA: per-lane 32-bit byte offsets (31 rows + a column) within a 32-row part
  if ((p.lda > p.ldb ? p.lda : p.ldb) >= ((int64_t)1 << 25) || p.I > p.lda || p.J > p.ldb) return hipErrorInvalidValue;
  if (mfma16)
    hipLaunchKernelGGL((gemm4h_kernel<true, true>), dim3((unsigned)grid), dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL((gemm4_kernel<true, true>), dim3((unsigned)grid), dim3(256), 0, s, p);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || p.splits == 1) return e;
  const int64_t n = N * K;
  int64_t blocks = (n / 8 + 255) / 256;
  blocks = blocks < 1 ? 1 : (blocks > 2048 ? 2048 : blocks);
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, s, ws, static_cast<uint16_t*>(dw),
                     p.splits, n, accumulate);
  return hipGetLastError();
}

hipError_t madnn_linear_wgrad4(const void* dy, const void* x, void* dw, float* ws, int splits, int accumulate,
                               int64_t M, int64_t N, int64_t K, hipStream_t s) {
  return linear_wgrad4_launch(dy, x, dw, ws, splits, accumulate, M, N, K, s, false);
}

hipError_t madnn_linear_wgrad4h(const void* dy, const void* x, void* dw, float* ws, int splits, int accumulate,
                                int64_t M, int64_t N, int64_t K, hipStream_t s) {
  return linear_wgrad4_launch(dy, x, dw, ws, splits, accumulate, M, N, K, s, true);
}

}  // extern "C"

