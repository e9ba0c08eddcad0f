// K12P — persistent K12: the transformer Linear forward / data-gradient GEMMs with their
// element-wise neighbours fused into an epilogue that overlaps the next tile's loads.
//
// Why (profiles/r5_gemm_pmc.md): on GPT-2's K = 1024 shapes hipBLASLt keeps the matrix cores busy
// 66 % of the time and one-tile-per-workgroup K12 54 %, against 87 % / 75 % at 8192^3 -- both lose
// ~21 points to the per-tile prologue fill + epilogue, during which a 1-workgroup-per-CU kernel
// has nothing else to run.  And the GELU after c_fc (gelu_fwd_kernel) and the dGELU + bias column
// sum after c_proj's data gradient (bias_grad_kernel) are standalone HBM passes (6.9 % of the
// GPT-2 medium step, profiles/r4_gpt2m_b128_steady_steps_attn_valu.md).
//
// Structure: one workgroup per CU (grid = min(tiles, CUs)), each walking a list of 256x256 output
// tiles (XCD-grouped: the tiles of one XCD's workgroups are contiguous, i fastest, so neighbours
// share operand panels in that XCD's L2).  The K tiles of all of a workgroup's output tiles form
// ONE continuous LDS-DMA stream: the 4-phase K12 schedule (gemm.hip header: two wave groups one
// barrier apart, counted vmcnt, never drained in the loop) runs straight across tile boundaries,
// so the next tile's first K tiles are already in LDS when an epilogue ends.  The epilogue works
// from the accumulators (no LDS round trip, the LDS holds the next tile's operands):
//   * v_permlane16_swap pairs two 16x16 accumulator blocks so each lane owns 8 consecutive
//     outputs of one row: one 16-B store per pair (a wave instruction writes 16 rows x 64 B);
//   * kPlain: (acc + bias) -> bf16;  kGelu: h = bf16(acc + bias) stored as the pre-activation,
//     out = bf16(gelu(h));  kDGelu: dh = bf16(bf16(acc) * gelu'(pre)), plus fp32 column sums of
//     dh (the c_fc bias gradient) as per-wave partial rows [j_tiles * 4][I] for a finalize pass.
//   The formulas and roundings are the unfused passes' own (gelu.h): fused == unfused.
// vmcnt across an epilogue: loads, stores and LDS-DMA retire in issue order on one counter, so the
// epilogue first issues the DMA that the next K tile's Q0/Q1 would have issued (the A halves of
// the K tile after it: their LDS stage was last read two phases earlier), then its S stores; the
// first K tile after it waits vmcnt(S + 4) instead of vmcnt(4) -- the S stores and the two B
// half-tiles issued since stay in flight, everything the next K tile reads has landed.  S is the
// exact per-wave count of VMEM stores of the epilogue (a compile-time constant per variant), and
// the kernel must have no scratch traffic (checked in the ISA by tests/test_gemm_gpu.py's build).
#include <type_traits>

#include "k12.h"

namespace madnn {
namespace gemmp {

using namespace mf;
using namespace k12;

enum Epi : int { kPlain = 0, kGelu = 1, kDGelu = 2 };

constexpr int kBiasMax = 8192;  // fp32 bias entries staged in LDS beside the 128 KiB of stages

// VMEM stores per wave per epilogue: 16 output pairs (+16 pre-activation / +4 column-sum dwords)
template <int EPI>
constexpr int store_count() {
  return EPI == kGelu ? 32 : EPI == kDGelu ? 20 : 16;
}

struct PArgs {
  const uint16_t* a;
  const uint16_t* b;
  uint16_t* out;         // [J][I], row stride ldo
  uint16_t* aux;         // kGelu: pre-activation store, same layout
  const uint16_t* pre;   // kDGelu: pre-activation read, same layout
  const void* bias;      // kPlain / kGelu: [I] fp32 (bias_f32) or bf16, or null
  float* colsum;         // kDGelu: [j_tiles * 4][I] fp32 partial column sums
  int64_t lda, ldb, ldo;
  int64_t I, J, K;
  int i_tiles, j_tiles, nk, ntile;
  int bias_f32;
};

__device__ __forceinline__ unsigned pack2(float a, float b) {
  return (unsigned)f32_to_bf16(a) | ((unsigned)f32_to_bf16(b) << 16);
}
__device__ __forceinline__ float lo16(unsigned v) { return bf16_to_f32((unsigned short)(v & 0xffffu)); }
__device__ __forceinline__ float hi16(unsigned v) { return bf16_to_f32((unsigned short)(v >> 16)); }

// two accumulator blocks X, Y (4 rows each per lane: rows 4g..4g+3 of a 16-row block, g = lane >> 4)
// as packed bf16 pairs -> this lane's 8 consecutive rows: X rows 8(g>>1).. for even g, Y's for odd g
__device__ __forceinline__ u32x4 swap_pairs(unsigned x0, unsigned x1, unsigned y0, unsigned y1) {
  const auto d0 = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
  const auto d1 = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
  return u32x4{d0[0], d1[0], d0[1], d1[1]};
}

template <bool A_COL, bool B_COL, int EPI, int GK = kGeluTanh>
__global__ __launch_bounds__(kThreads) void gemmp_kernel(const PArgs p) {
  // ONE LDS array (cdna_hip_programming.md §5 'Projection GEMM' item 4a): stages + fp32 bias
  __shared__ __attribute__((aligned(16))) uint16_t smem[kLds + 2 * kBiasMax];
  float* sbias = reinterpret_cast<float*>(smem + kLds);
  const int tid = threadIdx.x, lane = tid & 63, g4 = lane >> 4, l16 = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;

  // ---- this workgroup's tiles: XCD label x (dispatch is round-robin over the 8 XCDs) owns the
  // contiguous tile range [t_lo, t_hi); its gx workgroups take every gx-th tile of it
  const int G = gridDim.x, w = blockIdx.x;
  const int X = G < 8 ? G : 8;
  const int x = w % X, slot = w / X;
  const int gx = G / X + (x < G % X ? 1 : 0);
  const int t_lo = (int)((int64_t)p.ntile * x / X), t_hi = (int)((int64_t)p.ntile * (x + 1) / X);
  const int ntiles = slot < t_hi - t_lo ? (t_hi - t_lo - slot + gx - 1) / gx : 0;
  const int nk = p.nk;
  const int total = 4 * ntiles * nk;  // half-tiles in this workgroup's DMA stream

  const bool has_bias = EPI != kDGelu && p.bias != nullptr;
  if (has_bias) {  // before any DMA: ordinary loads + one plain barrier
    for (int i = tid; i < p.I; i += kThreads)
      sbias[i] = p.bias_f32 ? static_cast<const float*>(p.bias)[i]
                            : bf16_to_f32(static_cast<const uint16_t*>(p.bias)[i]);
    __syncthreads();
  }

  // per-lane DMA offsets: tiles never clamp here (I, J multiples of 256), so they are tile-free;
  // 32-bit (madnn_gemmp_supported bounds them): 8 VGPRs instead of 16
  // named scalars, selected with ?: (an indexed register array goes to scratch: guide rule 20)
  const int o00 = (int)dma_offset<A_COL>(2 * wave, lane, p.lda, 0, (int64_t)1 << 40);
  const int o01 = (int)dma_offset<A_COL>(2 * wave + 1, lane, p.lda, 0, (int64_t)1 << 40);
  const int o10 = (int)dma_offset<A_COL>(2 * wave, lane, p.lda, 128, (int64_t)1 << 40);
  const int o11 = (int)dma_offset<A_COL>(2 * wave + 1, lane, p.lda, 128, (int64_t)1 << 40);
  const int o20 = (int)dma_offset<B_COL>(2 * wave, lane, p.ldb, 0, (int64_t)1 << 40);
  const int o21 = (int)dma_offset<B_COL>(2 * wave + 1, lane, p.ldb, 0, (int64_t)1 << 40);
  const int o30 = (int)dma_offset<B_COL>(2 * wave, lane, p.ldb, 128, (int64_t)1 << 40);
  const int o31 = (int)dma_offset<B_COL>(2 * wave + 1, lane, p.ldb, 128, (int64_t)1 << 40);

  // kernel-argument fields as scalars: lambdas capturing the argument struct by reference make
  // hipcc spill it to scratch
  const uint16_t* const pa = p.a;
  const uint16_t* const pb = p.b;
  const int64_t lda = p.lda, ldb = p.ldb;
  const int itiles = p.i_tiles;
  auto tile_origin = [&](int q, int64_t& i0, int64_t& j0) {
    const int tile = t_lo + slot + q * gx;
    const int it = tile % itiles, jt = tile / itiles;
    i0 = (int64_t)it * kT;
    j0 = (int64_t)jt * kT;
  };

  // DMA cursor: the next half-tile H of the stream (H = 4u + h: h 0,1 = B halves, 2,3 = A halves
  // of global K tile u, stage u & 1) and the (tile, k) position of its K tile
  int cur_H = 0, cur_t = 0, cur_q = 0;
  int64_t ci0 = 0, cj0 = 0;
  if (ntiles > 0) tile_origin(0, ci0, cj0);
  // every call site knows which part it issues (H % 4 is fixed by the schedule), so the part --
  // and with it the offset pair and the operand -- is a compile-time constant: no selects
  auto stage_next = [&](auto part_c) {
    constexpr int part = decltype(part_c)::value;
    const int64_t k0 = (int64_t)cur_t * kBK;
    const uint16_t* base;
    int oe0, oe1;
    if constexpr (part < 2) {
      const int64_t x0 = ci0 + 128 * part;
      base = A_COL ? pa + k0 * lda + x0 : pa + x0 * lda + k0;
      oe0 = part == 0 ? o00 : o10;
      oe1 = part == 0 ? o01 : o11;
    } else {
      const int64_t x0 = cj0 + 128 * (part - 2);
      base = B_COL ? pb + k0 * ldb + x0 : pb + x0 * ldb + k0;
      oe0 = part == 2 ? o20 : o30;
      oe1 = part == 2 ? o21 : o31;
    }
    uint16_t* dst = smem + ((cur_H >> 2) & 1) * kStage + part * kHalf + (2 * wave) * 512;
    glds16((const void*)(base + oe0), (lds_void*)dst);
    glds16((const void*)(base + oe1), (lds_void*)(dst + 512));
    cur_H += 1;
    if ((cur_H & 3) == 0 && ++cur_t == nk) {
      cur_t = 0;
      if (++cur_q < ntiles) tile_origin(cur_q, ci0, cj0);
    }
  };
  using P0 = std::integral_constant<int, 0>;
  using P1 = std::integral_constant<int, 1>;
  using P2 = std::integral_constant<int, 2>;
  using P3 = std::integral_constant<int, 3>;

  f32x4 ac4[8][4];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) ac4[a][b] = zero4();

  // prologue: half-tiles 0..5 (K tile 0 + the B halves of K tile 1)
  // (parts in stream order: B0 B1 A0 A1 of K tile 0, then B0 B1 of K tile 1)
  if (total > 0) {
    stage_next(P2{});
    stage_next(P3{});
    stage_next(P0{});
    stage_next(P1{});
  }
  if (total > 4) {
    stage_next(P2{});
    stage_next(P3{});
  }
  if (total > 4) {
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  barrier();
  if (wr == 1) barrier();  // group 1 runs one barrier behind, across every tile

  bf16x8 af[2][4], bf0[4], bf1[4];
  const int bcol = (wc & 1) * 64;
  constexpr int S = store_count<EPI>();
  int u = 0;  // global K tile
  for (int q = 0; q < ntiles; ++q) {
    int64_t i0, j0;
    tile_origin(q, i0, j0);
    for (int t = 0; t < nk; ++t, ++u) {
      const uint16_t* sa = smem + (u & 1) * kStage + wr * kHalf;
      const uint16_t* sb = smem + (u & 1) * kStage + (2 + (wc >> 1)) * kHalf;
      const int P = 4 * u;
      const bool first = q > 0 && t == 0;  // the epilogue issued this K tile's Q0 / Q1 DMA
      // ---- Q0: A rows 0..63, B cols 0..31
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
        for (int c = 0; c < 2; ++c) bf0[2 * c + s2] = frag16<B_COL>(sb, s2, bcol + 16 * c, lane);
#pragma unroll
        for (int a = 0; a < 4; ++a) af[a >> 1][2 * (a & 1) + s2] = frag16<A_COL>(sa, s2, 16 * a, lane);
      }
      if (!first && cur_H < total) stage_next(P0{});
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
      if (!first && cur_H < total) stage_next(P1{});
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
      if (cur_H < total) stage_next(P2{});
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
      // ---- Q3: no reads; retire K tile u+1's DMA (the B halves of K tile u+2 stay in flight,
      // and after an epilogue its S stores too: they were issued after K tile u+1's A halves)
      if (first) {
        if (P + 9 < total) {
          stage_next(P3{});
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(S + 4) : "memory");
        } else if (P + 8 < total) {
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(S + 2) : "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(S) : "memory");
        }
      } else if (P + 9 < total) {
        stage_next(P3{});
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

    // ================= epilogue of tile q (no LDS, no barrier) =================
    // 1) the next K tile's Q0 / Q1 DMA (A halves of K tile u+1) BEFORE the stores
    if (q + 1 < ntiles && cur_H < total) {
      stage_next(P0{});
      stage_next(P1{});
    }
    __builtin_amdgcn_sched_barrier(0);
    // this lane's rows: pair m (blocks 2m, 2m+1), j block b: 8 outputs at i = ib + 32m + io, row jb + 16b.
    // The lane index goes through an empty asm so hipcc cannot hoist the epilogue's per-lane
    // addresses out of the tile loop (kept live across the main loop they spill)
    int el = lane;
    asm volatile("" : "+v"(el));
    const int eg4 = el >> 4, el16 = el & 15;
    const int io = 16 * (eg4 & 1) + 8 * (eg4 >> 1);
    const int64_t ib = i0 + wr * 128, jb = j0 + wc * 64 + el16;
    if constexpr (EPI == kDGelu) {
      // two halves of two pairs: the second half's pre-activation is loaded BEFORE the first
      // half's stores are issued (loads, stores and DMA retire in issue order: a load issued
      // after a store would wait for that store's ack), while only 32 VGPRs of it are live
      float* crow = p.colsum + ((j0 / kT) * 4 + wc) * p.I + ib + io;
      u32x4 pv[2][4], ov[2][4];
      float cv[2];
      const int cidx = 4 * ((el16 >> 3) & 1) + 2 * ((el16 >> 2) & 1) + ((el16 >> 1) & 1);
      auto load_half = [&](int h) {
#pragma unroll
        for (int mm = 0; mm < 2; ++mm)
#pragma unroll
          for (int b = 0; b < 4; ++b)
            pv[mm][b] = *reinterpret_cast<const u32x4*>(p.pre + (jb + 16 * b) * p.ldo + ib + 32 * (2 * h + mm) + io);
      };
      auto compute_half = [&](int h) {
#pragma unroll
        for (int mm = 0; mm < 2; ++mm) {
          const int m = 2 * h + mm;
          float cs[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) cs[e] = 0.f;
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            const f32x4 X = ac4[2 * m][b], Y = ac4[2 * m + 1][b];
            const u32x4 d = swap_pairs(pack2(X[0], X[1]), pack2(X[2], X[3]), pack2(Y[0], Y[1]), pack2(Y[2], Y[3]));
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const float v0 = lo16(d[k]) * gelu_act_grad<GK>(lo16(pv[mm][b][k]));
              const float v1 = hi16(d[k]) * gelu_act_grad<GK>(hi16(pv[mm][b][k]));
              cs[2 * k] += v0;
              cs[2 * k + 1] += v1;
              ov[mm][b][k] = pack2(v0, v1);
            }
          }
          // column sums over this wave's 64 rows (the 16 lanes of a lane row hold 16 different
          // rows): a reduce-scatter over lane bits 3, 2, 1, then a sum over bit 0 -- this lane
          // ends with the total of output 4 b3 + 2 b2 + b1 of its 8 (lanes 2k, 2k+1 agree)
          const bool b3 = el16 & 8, b2 = el16 & 4, b1 = el16 & 2;
          float r4[4], r2[2];
#pragma unroll
          for (int k = 0; k < 4; ++k)
            r4[k] = (b3 ? cs[4 + k] : cs[k]) + __shfl_xor(b3 ? cs[k] : cs[4 + k], 8);
#pragma unroll
          for (int k = 0; k < 2; ++k)
            r2[k] = (b2 ? r4[2 + k] : r4[k]) + __shfl_xor(b2 ? r4[k] : r4[2 + k], 4);
          float v = (b1 ? r2[1] : r2[0]) + __shfl_xor(b1 ? r2[0] : r2[1], 2);
          v += __shfl_xor(v, 1);
          cv[mm] = v;
        }
      };
      auto store_half = [&](int h) {
#pragma unroll
        for (int mm = 0; mm < 2; ++mm) {
          const int m = 2 * h + mm;
#pragma unroll
          for (int b = 0; b < 4; ++b)
            *reinterpret_cast<u32x4*>(p.out + (jb + 16 * b) * p.ldo + ib + 32 * m + io) = ov[mm][b];
          if ((el16 & 1) == 0) crow[32 * m + cidx] = cv[mm];
        }
      };
      load_half(0);
      compute_half(0);
      __builtin_amdgcn_sched_barrier(0);
      load_half(1);
      __builtin_amdgcn_sched_barrier(0);
      store_half(0);
      __builtin_amdgcn_sched_barrier(0);
      compute_half(1);
      store_half(1);
    } else {
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        // this lane's bias for blocks 2m and 2m+1: rows 4g..4g+3 of each
        float bx[4] = {0.f, 0.f, 0.f, 0.f}, by[4] = {0.f, 0.f, 0.f, 0.f};
        if (has_bias) {
          const int r0 = (int)ib + 32 * m + 4 * eg4;
          const f32x4 vx = *reinterpret_cast<const f32x4*>(sbias + r0);
          const f32x4 vy = *reinterpret_cast<const f32x4*>(sbias + r0 + 16);
          bx[0] = vx[0]; bx[1] = vx[1]; bx[2] = vx[2]; bx[3] = vx[3];
          by[0] = vy[0]; by[1] = vy[1]; by[2] = vy[2]; by[3] = vy[3];
        }
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const f32x4 X = ac4[2 * m][b], Y = ac4[2 * m + 1][b];
          const u32x4 h = swap_pairs(pack2(X[0] + bx[0], X[1] + bx[1]), pack2(X[2] + bx[2], X[3] + bx[3]),
                                     pack2(Y[0] + by[0], Y[1] + by[1]), pack2(Y[2] + by[2], Y[3] + by[3]));
          uint16_t* dst = p.out + (jb + 16 * b) * p.ldo + ib + 32 * m + io;
          if constexpr (EPI == kGelu) {
            *reinterpret_cast<u32x4*>(p.aux + (jb + 16 * b) * p.ldo + ib + 32 * m + io) = h;
            u32x4 o;
#pragma unroll
            for (int k = 0; k < 4; ++k) o[k] = pack2(gelu_act<GK>(lo16(h[k])), gelu_act<GK>(hi16(h[k])));
            *reinterpret_cast<u32x4*>(dst) = o;
          } else {
            *reinterpret_cast<u32x4*>(dst) = h;
          }
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) ac4[a][b] = zero4();
  }
  if (wr == 0) barrier();  // balance the stagger: every wave has now passed the same barriers
}

// column-sum partial rows [R][I] -> bias gradient [I] (fixed order: deterministic).  One wave per
// 64 contiguous columns (256-byte row segments), 16 waves per workgroup splitting the rows, 8 loads
// in flight per lane: the 32 MB of partials at GPT-2 b128 are read at HBM rate by 64 workgroups.
template <bool F32OUT>
__global__ __launch_bounds__(1024) void colsum_finalize_kernel(const float* __restrict__ part, int R, int64_t I,
                                                               void* __restrict__ out) {
  constexpr int kSl = 16, kU = 8;
  __shared__ float red[kSl][64];
  const int c = threadIdx.x & 63, sl = threadIdx.x >> 6;
  const int64_t i = (int64_t)blockIdx.x * 64 + c;
  float a = 0.f;
  if (i < I) {
    int r = sl;
    for (; r + (kU - 1) * kSl < R; r += kU * kSl) {
      float v[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) v[u] = part[(int64_t)(r + u * kSl) * I + i];
#pragma unroll
      for (int u = 0; u < kU; ++u) a += v[u];
    }
    for (; r < R; r += kSl) a += part[(int64_t)r * I + i];
  }
  red[sl][c] = a;
  __syncthreads();
  if (sl == 0 && i < I) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < kSl; ++q) t += red[q][c];
    if (F32OUT) static_cast<float*>(out)[i] = t;
    else static_cast<uint16_t*>(out)[i] = f32_to_bf16(t);
  }
}

int g_num_cus = 0;

int num_cus() {
  if (g_num_cus == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                hipSuccess || n <= 0)
      n = kNumCU;
    g_num_cus = n;
  }
  return g_num_cus;
}

template <bool A_COL, int EPI, int GK = kGeluTanh>
hipError_t launch(PArgs& p, hipStream_t s) {
  p.i_tiles = (int)(p.I / kT);
  p.j_tiles = (int)(p.J / kT);
  p.nk = (int)(p.K / kBK);
  p.ntile = p.i_tiles * p.j_tiles;
  if (p.ntile <= 0 || (int64_t)p.i_tiles * p.j_tiles > 0x7fffffff) return hipErrorInvalidValue;
  const int grid = p.ntile < num_cus() ? p.ntile : num_cus();
  hipLaunchKernelGGL((gemmp_kernel<A_COL, false, EPI, GK>), dim3(grid), dim3(kThreads), 0, s, p);
  return hipGetLastError();
}

}  // namespace gemmp
}  // namespace madnn

using namespace madnn::gemmp;
using madnn::kGeluErf;
using madnn::kGeluTanh;

extern "C" {

// Shapes K12P takes: output features and tokens multiples of 256 (no edge tiles), reduction a
// multiple of 64, 32-bit-safe per-lane DMA offsets; a bias must fit the LDS bias slot.
int madnn_gemmp_supported(int64_t I, int64_t J, int64_t K, int has_bias) {
  if (I <= 0 || J <= 0 || K <= 0) return 0;
  if (I % kT || J % kT || K % kBK) return 0;
  if (has_bias && I > kBiasMax) return 0;
  // 32-bit per-lane DMA offsets: at most 64 rows of the longest leading dimension + 256 columns
  if ((I > K ? I : K) * 64 + 256 > 0x7fffffffLL) return 0;
  return 1;
}

// Y[m][n] = X[m][k] W[n][k] (+ bias[n]); act 1 / 2 (tanh / erf GELU): aux = that pre-activation,
// Y = gelu(aux)
hipError_t madnn_linear_fwd_p(const void* x, const void* w, const void* bias, int bias_f32, void* y, void* aux,
                              int act, int64_t M, int64_t N, int64_t K, hipStream_t s) {
  if (!madnn_gemmp_supported(N, M, K, bias != nullptr) || (act != 0 && aux == nullptr) || act < 0 || act > 2)
    return hipErrorInvalidValue;
  PArgs p{};
  p.a = static_cast<const uint16_t*>(w);
  p.lda = K;
  p.b = static_cast<const uint16_t*>(x);
  p.ldb = K;
  p.out = static_cast<uint16_t*>(y);
  p.aux = static_cast<uint16_t*>(aux);
  p.ldo = N;
  p.bias = bias;
  p.bias_f32 = bias_f32;
  p.I = N;
  p.J = M;
  p.K = K;
  return act == kGeluTanh ? launch<false, kGelu, kGeluTanh>(p, s)
         : act == kGeluErf ? launch<false, kGelu, kGeluErf>(p, s)
                           : launch<false, kPlain>(p, s);
}

// dX[m][k] = dY[m][n] W[n][k]; with pre: dX = that * gelu'(pre) (gelu_kind 1 tanh / 2 erf) and the
// fp32 column sums of dX as
// [M / 256 * 4][K] partial rows in colsum (madnn_colsum_finalize turns them into the bias grad)
hipError_t madnn_linear_dgrad_p(const void* dy, const void* w, const void* pre, void* dx, float* colsum, int64_t M,
                                int64_t N, int64_t K, int gelu_kind, hipStream_t s) {
  if (!madnn_gemmp_supported(K, M, N, 0) || (pre != nullptr && colsum == nullptr)) return hipErrorInvalidValue;
  PArgs p{};
  p.a = static_cast<const uint16_t*>(w);
  p.lda = K;
  p.b = static_cast<const uint16_t*>(dy);
  p.ldb = N;
  p.out = static_cast<uint16_t*>(dx);
  p.pre = static_cast<const uint16_t*>(pre);
  p.colsum = colsum;
  p.ldo = K;
  p.I = K;
  p.J = M;
  p.K = N;
  if (pre == nullptr) return launch<true, kPlain>(p, s);
  return gelu_kind == kGeluErf ? launch<true, kDGelu, kGeluErf>(p, s) : launch<true, kDGelu, kGeluTanh>(p, s);
}

hipError_t madnn_colsum_finalize(const float* part, int R, int64_t I, void* out, int out_f32, hipStream_t s) {
  const unsigned blocks = (unsigned)((I + 63) / 64);
  if (out_f32) {
    hipLaunchKernelGGL(colsum_finalize_kernel<true>, dim3(blocks), dim3(1024), 0, s, part, R, I, out);
  } else {
    hipLaunchKernelGGL(colsum_finalize_kernel<false>, dim3(blocks), dim3(1024), 0, s, part, R, I, out);
  }
  return hipGetLastError();
}

}  // extern "C"
