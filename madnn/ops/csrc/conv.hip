// K9 — NHWC 1x1 convolution (stride 1) as bf16 MFMA GEMMs for gfx950: forward (+ the
// following BatchNorm's batch statistics), data gradient and weight gradient.
//
// Why: 36 of ResNet-50's 53 convolutions are bottleneck 1x1s.  The MIOpen solvers that the
// shipped MI355X find-db picks for them (madnn/tuning/miopen, batch 512) reach 35-60 % of
// the HBM / MFMA bound outside layer1 and ~50 % on the data gradient inside it, and the
// BatchNorm after each one re-reads its whole output for the statistics.
//
// An NHWC activation is a dense [M = N*H*W, C] matrix and a 1x1 weight a [Cout, Cin]
// matrix, so the three passes are plain GEMMs:
//   forward   Y[m][co]   = sum_ci X[m][ci]  W[co][ci]
//   dgrad     dX[m][ci]  = sum_co dY[m][co] W[co][ci]
//   wgrad     dW[co][ci] = sum_m  dY[m][co] X[m][ci]
// One template computes D[i][j] = sum_k A(i, k) B(k, j) with j on the MFMA lane.  Each
// operand is staged from "row" memory (k contiguous: a [R][64] LDS tile read with
// ds_read_b128) or from "column" memory (k strided: a [64][C] tile read with the gfx950
// transpose read ds_read_b64_tr_b16), see mfma.h:
//   forward : i = co (A = W, row),     j = m  (B = X, row)    -> Y[j][i]
//   dgrad   : i = ci (A = W, column),  j = m  (B = dY, row)   -> dX[j][i]
//   wgrad   : i = co (A = dY, column), j = ci (B = X, column), the m reduction split over
//             workgroups; each split stores its fp32 partial [Cout][Cin] slab (one accumulator
//             register = two 128-B row segments per wave instruction) and one streaming pass sums
//             the slabs in split order -- deterministic, unlike float atomics (no -munsafe-fp-atomics
//             result that depends on arrival order).
// In the store epilogue a lane owns 4 consecutive i of one j: one 8-byte store.
//
// CDNA4 mapping: v_mfma_f32_32x32x16_bf16; 4 waves per workgroup, each owning a 64x64
// (64x32, 32x32) block of D; 64-deep k steps staged global -> VGPR -> LDS, double
// buffered with one barrier per step, so the next step's global loads are in flight
// during this step's MFMAs; 64 KiB of LDS and <= 256 VGPRs: 2 workgroups (8 waves) per
// CU.  Forward / dgrad workgroups are persistent: a workgroup keeps its i tile and walks
// its j tiles, so loading tile t+1 overlaps tile t's MFMAs and epilogue.
//
// Fused BatchNorm statistics (forward): the workgroup accumulates, per output channel,
// the sum and sum of squares of the bf16-rounded outputs it stores, in registers across
// all its tiles, and writes one [2][Cout] partial row.  That slab is the input format of
// bn.hip's finalize kernel, so the BatchNorm forward skips its statistics pass over Y.
//
// (A BatchNorm apply + ReLU prologue on the X operand, a BN-reduction epilogue over a residual
// ReLU's bit mask and a stride-2 residual epilogue were measured, lost their A/Bs and were removed
// in round 6: docs/PERF.md.)
#include "mfma.h"

namespace madnn {
namespace conv {

using namespace mf;

constexpr int kThreads = 256;
constexpr int kBK = 64;                // reduction depth of one pipeline step
constexpr int kTargetWG = 2 * kNumCU;  // resident workgroups: 2 per CU

// run-time tunables (swept through madnn_conv1x1_tune, profiles/r1_k9_tune.json)
struct Tune {
  int fwd_wg = kTargetWG;  // forward / dgrad persistent grid target
  int wgrad_wg = 2 * kNumCU;  // weight-grad workgroups (tiles x m splits)
  int xcd = 1;             // XCD-aware workgroup remap
};
inline Tune& tune() {
  static Tune t;
  return t;
}

enum Mode : int { kStoreT = 0, kSplit = 1 };

struct GemmArgs {
  const uint16_t* a;
  const uint16_t* b;
  void* out;
  const uint16_t* res;  // store epilogue: out = D + res (same layout as out), or null
  const unsigned char* resmask;  // with res: res element e counts only where bit e of resmask is set
                                 // (a ReLU bit mask over the same [J][I] elements, 8 per byte), or null
  float* stats;
  const uint16_t* bny;  // BNB epilogue (data grad): BN input y [J][I] whose backward sums are taken,
  const float* bnsc;    //   with its forward scale / shift (ReLU mask = y * sc + sh > 0)
  const float* bnsh;
  int64_t lda, ldb, ldo;
  int64_t I, J, K;                       // D is I x J, reduction length K
  int i_tiles, j_tiles, j_groups, k_chunk;
  int xcd;  // 1: remap workgroup ids so consecutive logical ids share an XCD (and its L2)
};

// One operand's 64-deep slice, register-staged: R rows of "row" memory ([x][ld], k
// contiguous) or 64 k-rows of "column" memory ([k][ld], R contiguous x).  Rows past the
// end load a valid row and are zeroed by a mask (no per-load branch).
template <bool COL, int R>
struct Stage {
  static constexpr int PER = R / 32;  // 16-B chunks per thread
  u32x4 r[PER];

  __device__ __forceinline__ void load(const uint16_t* __restrict__ base, int64_t ld, int64_t x0, int64_t xlim,
                                       int64_t k0, int64_t klim, int tid) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = tid + kThreads * i;
      int64_t row, lim, col;
      if constexpr (COL) {
        row = k0 + c / (R / 8);
        lim = klim;
        col = x0 + (c % (R / 8)) * 8;
      } else {
        row = x0 + (c >> 3);
        lim = xlim;
        col = k0 + (c & 7) * 8;
      }
      const bool ok = row < lim;
      const u32x4 v = *reinterpret_cast<const u32x4*>(base + (ok ? row : lim - 1) * ld + col);
      const unsigned keep = ok ? 0xffffffffu : 0u;
      r[i] = v & keep;
    }
  }

  __device__ __forceinline__ void store(uint16_t* tile, int tid) const {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = tid + kThreads * i;
      int boff;
      if constexpr (COL) {
        boff = swz<R>(c / (R / 8), c % (R / 8));
      } else {
        boff = swz<64>(c >> 3, c & 7);
      }
      *reinterpret_cast<u32x4*>(reinterpret_cast<char*>(tile) + boff) = r[i];
    }
  }

  // MFMA operand for k16 step s of the extent block starting at x (lane -> x + (lane & 31))
  static __device__ __forceinline__ bf16x8 frag(const uint16_t* tile, int s, int x, int lane) {
    if constexpr (COL) {
      return lds_col<R>(tile, 16 * s, x, lane);
    } else {
      return lds_row(tile, x + (lane & 31), 2 * s + (lane >> 5));
    }
  }
};

// BNB (store mode): besides the output D, accumulate per output channel the BatchNorm backward sums
// sum g and sum g*y, g = D * [y * sc + sh > 0], into the same [groups][2][I] partial rows STATS writes
// (the data grad of conv3 whose input was relu(bn2(y)): bn2's backward skips its reduction pass).
template <bool A_COL, bool B_COL, int BI, int BJ, int MODE, bool STATS, bool BNB = false>
__global__ __launch_bounds__(kThreads, 2) void gemm_kernel(const GemmArgs p) {
  static_assert(!(STATS && BNB), "one statistics epilogue per launch");
  constexpr int NI = (BI == 64 && BJ == 64) ? 1 : 2;  // 32-row i blocks per wave
  constexpr int WI = BI / (32 * NI), WJ = 4 / WI, NJ = BJ / (32 * WJ);
  static_assert(WI * WJ == 4 && NJ >= 1, "four waves tile the workgroup");
  constexpr int AE = BI * kBK, BE = BJ * kBK, SE = AE + BE;  // one pipeline buffer: [A | B]
  static_assert(SE >= BI * BJ, "a pipeline buffer holds the bf16 output tile");
  // output tile (store epilogue): [BJ][BI] bf16, 16-B chunks XOR-swizzled per row
  constexpr int CPR = BI / 8;               // 16-B chunks per output row
  constexpr int RPP = kThreads / CPR;       // rows per pass of the 256 threads
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * SE];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, l32 = lane & 31, hh = lane >> 5;
  const int wi = wave / WJ, wj = wave % WJ;
  // logical id: consecutive ids share the B (j) panel.  The dispatcher deals ids round-robin
  // over the 8 XCDs; the bijective remap of cdna_hip_programming.md T1 gives each XCD a
  // contiguous range of logical ids so the shared panels hit in that XCD's L2.
  int wid = blockIdx.x;
  if (p.xcd) {
    const int n = gridDim.x, x = wid % 8, q8 = n / 8, r8 = n % 8;
    wid = (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + wid / 8;
  }
  const int it = wid % p.i_tiles;
  const int grp = wid / p.i_tiles;
  const int64_t i0 = (int64_t)it * BI;
  const int nk = (int)((p.K + kBK - 1) / kBK);
  int jt, kbeg, kend, jstride;
  if constexpr (MODE == kSplit) {  // one j tile, k steps [kbeg, kend)
    jt = grp % p.j_tiles;
    kbeg = (grp / p.j_tiles) * p.k_chunk;
    kend = min(kbeg + p.k_chunk, nk);
    jstride = p.j_tiles;
  } else {  // persistent: j tiles grp, grp + j_groups, ...; all k
    jt = grp;
    kbeg = 0;
    kend = nk;
    jstride = p.j_groups;
  }
  if (jt >= p.j_tiles || kbeg >= kend) return;

  Stage<A_COL, BI> sta;
  Stage<B_COL, BJ> stb;
  f32x16 acc[NI][NJ];
#pragma unroll
  for (int a = 0; a < NI; ++a)
#pragma unroll
    for (int b = 0; b < NJ; ++b) acc[a][b] = zero16();
  // statistics: this thread's 8 output channels (chunk tid % CPR), summed over its rows of every tile
  float ssum[8], ssq[8], bs[8], bh[8];
  if constexpr (STATS || BNB) {
#pragma unroll
    for (int e = 0; e < 8; ++e) ssum[e] = ssq[e] = 0.f;
  }
  if constexpr (BNB) {  // this thread's 8 output channels (chunk tid % CPR of the i tile) are fixed
    const int cc = tid % (BI / 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      bs[e] = p.bnsc[i0 + 8 * cc + e];
      bh[e] = p.bnsh[i0 + 8 * cc + e];
    }
  }
  // byte offset of 16-B chunk c of output row r: rows of 256 B (BI = 128) or 128 B (BI = 64)
  auto out_off = [](int r, int c) {
    if constexpr (BI == 128) return r * 256 + 16 * (c ^ (r & 15));
    else return r * 128 + 16 * (c ^ ((r >> 1) & 7));
  };

  sta.load(p.a, p.lda, i0, p.I, (int64_t)kbeg * kBK, p.K, tid);
  stb.load(p.b, p.ldb, (int64_t)jt * BJ, p.J, (int64_t)kbeg * kBK, p.K, tid);
  sta.store(smem, tid);
  stb.store(smem + AE, tid);
  __syncthreads();
  int cur = 0, ks = kbeg;
  for (;;) {
    int njt = jt, nks = ks + 1;
    if (nks == kend) {
      nks = kbeg;
      njt = jt + jstride;
    }
    const bool more = njt < p.j_tiles;
    if (more) {
      sta.load(p.a, p.lda, i0, p.I, (int64_t)nks * kBK, p.K, tid);
      stb.load(p.b, p.ldb, (int64_t)njt * BJ, p.J, (int64_t)nks * kBK, p.K, tid);
    }
    uint16_t* buf = smem + cur * SE;
#pragma unroll
    for (int s = 0; s < kBK / 16; ++s) {
      bf16x8 af[NI], bv[NJ];
#pragma unroll
      for (int a = 0; a < NI; ++a) af[a] = Stage<A_COL, BI>::frag(buf, s, (wi * NI + a) * 32, lane);
#pragma unroll
      for (int b = 0; b < NJ; ++b) bv[b] = Stage<B_COL, BJ>::frag(buf + AE, s, (wj * NJ + b) * 32, lane);
#pragma unroll
      for (int a = 0; a < NI; ++a)
#pragma unroll
        for (int b = 0; b < NJ; ++b) acc[a][b] = mfma(af[a], bv[b], acc[a][b]);
    }
    if (more) {  // the other buffer was last read before the previous barrier
      sta.store(smem + (cur ^ 1) * SE, tid);
      stb.store(smem + (cur ^ 1) * SE + AE, tid);
    }
    if (ks == kend - 1) {  // tile done: epilogue
      if constexpr (MODE == kStoreT) {
        // D[i][j] (4 consecutive i per lane) -> LDS tile [j][i] -> full-row 16-B global stores
        __syncthreads();  // every wave is done reading buf
        char* ot = reinterpret_cast<char*>(buf);
#pragma unroll
        for (int b = 0; b < NJ; ++b) {
          const int jr = (wj * NJ + b) * 32 + l32;
#pragma unroll
          for (int a = 0; a < NI; ++a)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              const int ic = (wi * NI + a) * 32 + 8 * g + 4 * hh;  // first of the 4 i
              const unsigned lo = (unsigned)f32_to_bf16(acc[a][b][4 * g]) |
                                  ((unsigned)f32_to_bf16(acc[a][b][4 * g + 1]) << 16);
              const unsigned hi = (unsigned)f32_to_bf16(acc[a][b][4 * g + 2]) |
                                  ((unsigned)f32_to_bf16(acc[a][b][4 * g + 3]) << 16);
              *reinterpret_cast<u32x2*>(ot + out_off(jr, ic >> 3) + 8 * ((ic >> 2) & 1)) = u32x2{lo, hi};
            }
        }
        __syncthreads();
        uint16_t* out = static_cast<uint16_t*>(p.out);
        const int c = tid % CPR;
#pragma unroll
        for (int u = 0; u < BJ / RPP; ++u) {
          const int r = tid / CPR + RPP * u;
          const int64_t j = (int64_t)jt * BJ + r;
          if (j < p.J) {
            u32x4 v = *reinterpret_cast<const u32x4*>(ot + out_off(r, c));
            if (p.res != nullptr) {  // fused residual-gradient accumulation (fp32 add, one rounding)
              u32x4 rv = *reinterpret_cast<const u32x4*>(p.res + j * p.ldo + i0 + 8 * c);
              if (p.resmask != nullptr) {
                const unsigned bits = p.resmask[(j * p.ldo + i0 + 8 * c) >> 3];
#pragma unroll
                for (int e = 0; e < 4; ++e)
                  rv[e] &= ((bits >> (2 * e)) & 1u ? 0xffffu : 0u) | ((bits >> (2 * e + 1)) & 1u ? 0xffff0000u : 0u);
              }
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const float lo = bf16_to_f32((unsigned short)(v[e] & 0xffffu)) +
                                 bf16_to_f32((unsigned short)(rv[e] & 0xffffu));
                const float hi = bf16_to_f32((unsigned short)(v[e] >> 16)) + bf16_to_f32((unsigned short)(rv[e] >> 16));
                v[e] = (unsigned)f32_to_bf16(lo) | ((unsigned)f32_to_bf16(hi) << 16);
              }
            }
            *reinterpret_cast<u32x4*>(out + j * p.ldo + i0 + 8 * c) = v;
            if constexpr (BNB) {
              const u32x4 yv = *reinterpret_cast<const u32x4*>(p.bny + j * p.ldo + i0 + 8 * c);
#pragma unroll
              for (int e = 0; e < 4; ++e) {
#pragma unroll
                for (int hf = 0; hf < 2; ++hf) {
                  const int k = 2 * e + hf;
                  const float g = bf16_to_f32((unsigned short)(hf ? v[e] >> 16 : v[e] & 0xffffu));
                  const float yy = bf16_to_f32((unsigned short)(hf ? yv[e] >> 16 : yv[e] & 0xffffu));
                  const bool on = yy * bs[k] + bh[k] > 0.f;
                  const float gm = on ? g : 0.f;
                  ssum[k] += gm;
                  ssq[k] += gm * yy;
                }
              }
            }
            if constexpr (STATS) {
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const float x0 = bf16_to_f32((unsigned short)(v[e] & 0xffffu));
                const float x1 = bf16_to_f32((unsigned short)(v[e] >> 16));
                ssum[2 * e] += x0;
                ssq[2 * e] += x0 * x0;
                ssum[2 * e + 1] += x1;
                ssq[2 * e + 1] += x1 * x1;
              }
            }
          }
        }
      } else {
        // this split's partial slab (split = grp / j_tiles)
        const int64_t jw = (int64_t)jt * BJ + wj * NJ * 32 + l32;
        float* out = static_cast<float*>(p.out) + (int64_t)(grp / p.j_tiles) * p.I * p.ldo;
#pragma unroll
        for (int a = 0; a < NI; ++a)
#pragma unroll
          for (int b = 0; b < NJ; ++b)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int64_t i = i0 + (wi * NI + a) * 32 + acc_row(r, hh);
              out[i * p.ldo + jw + b * 32] = acc[a][b][r];
            }
      }
#pragma unroll
      for (int a = 0; a < NI; ++a)
#pragma unroll
        for (int b = 0; b < NJ; ++b) acc[a][b] = zero16();
    }
    if (!more) break;
    __syncthreads();  // next buffer filled; this one (or its output tile) fully consumed
    cur ^= 1;
    jt = njt;
    ks = nks;
  }

  if constexpr (STATS || BNB) {
    __syncthreads();  // smem is free
    float* red = reinterpret_cast<float*>(smem);  // [RPP][2][BI]
    const int c = tid % CPR, rg = tid / CPR;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[(rg * 2) * BI + 8 * c + e] = ssum[e];
      red[(rg * 2 + 1) * BI + 8 * c + e] = ssq[e];
    }
    __syncthreads();
    for (int k = tid; k < 2 * BI; k += kThreads) {
      const int which = k / BI, ii = k % BI;
      float v = 0.f;
      for (int g = 0; g < RPP; ++g) v += red[(g * 2 + which) * BI + ii];
      p.stats[((int64_t)grp * 2 + which) * p.I + i0 + ii] = v;
    }
  }
}

template <bool A_COL, bool B_COL, int BI, int BJ, int MODE, bool STATS, bool BNB = false>
hipError_t launch(const GemmArgs& p, int grid, hipStream_t s) {
  hipLaunchKernelGGL((gemm_kernel<A_COL, B_COL, BI, BJ, MODE, STATS, BNB>), dim3(grid), dim3(kThreads), 0, s, p);
  return hipGetLastError();
}

// forward / dgrad: i tiles x j groups, each workgroup walking an equal share of the j tiles.
// Shallow reductions (K < 512: one tile is a few k steps, HBM-bound) stay persistent so the next
// tile's loads overlap this tile's epilogue; deep ones get one tile per workgroup (measured
// faster: profiles/r1_k9_tune.json).
inline void plan_persistent(GemmArgs& p, int64_t J, int BI, int64_t I, int64_t K) {
  p.i_tiles = (int)(I / BI);
  p.j_tiles = (int)((J + 127) / 128);
  const int64_t total = (int64_t)p.i_tiles * p.j_tiles;
  const int64_t per = K >= 8 * kBK ? 1 : (total + tune().fwd_wg - 1) / tune().fwd_wg;
  p.j_groups = (int)((p.j_tiles + per - 1) / per);
  p.k_chunk = 0;
}

// dw[i] = sum over splits of slab[s][i], in split order (deterministic), fp32 or bf16; n % 4 == 0
template <bool BF16>
__global__ __launch_bounds__(256) void split_reduce_kernel(const float* __restrict__ slab, int splits, int64_t n,
                                                           void* __restrict__ dw) {
  const int64_t n4 = n / 4;
  for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < n4; v += (int64_t)gridDim.x * 256) {
    f32x4 acc = reinterpret_cast<const f32x4*>(slab)[v];
    for (int s = 1; s < splits; ++s) acc += reinterpret_cast<const f32x4*>(slab + (int64_t)s * n)[v];
    if constexpr (BF16) {
      const unsigned lo = (unsigned)f32_to_bf16(acc[0]) | ((unsigned)f32_to_bf16(acc[1]) << 16);
      const unsigned hi = (unsigned)f32_to_bf16(acc[2]) | ((unsigned)f32_to_bf16(acc[3]) << 16);
      reinterpret_cast<u32x2*>(dw)[v] = u32x2{lo, hi};
    } else {
      reinterpret_cast<f32x4*>(dw)[v] = acc;
    }
  }
}

// workgroup tiles and m splits of the weight gradient (shared by the launcher and the workspace size)
inline void wgrad_split(int64_t M, int64_t cin, int64_t cout, int& bi, int& bj, int64_t& tiles, int& k_chunk,
                        int64_t& splits) {
  bi = cout % 128 == 0 ? 128 : 64;
  bj = cin % 128 == 0 ? 128 : 64;
  tiles = (cout / bi) * (cin / bj);
  const int64_t nk = (M + kBK - 1) / kBK;
  splits = (tune().wgrad_wg + tiles - 1) / tiles;
  splits = splits < 1 ? 1 : (splits > nk ? nk : splits);
  k_chunk = (int)((nk + splits - 1) / splits);
  splits = (nk + k_chunk - 1) / k_chunk;
}

}  // namespace conv
}  // namespace madnn

using namespace madnn::conv;

extern "C" {

// key 0: forward/dgrad grid target, 1: weight-grad workgroups, 2: XCD remap (0/1); returns the old value
int madnn_conv1x1_tune(int key, int value) {
  int* f = key == 0 ? &tune().fwd_wg : key == 1 ? &tune().wgrad_wg : key == 2 ? &tune().xcd : nullptr;
  if (f == nullptr) return -1;
  const int old = *f;
  if (value >= 0) *f = value;
  return old;
}

int madnn_conv1x1_supported(int64_t cin, int64_t cout) {
  return (cin % 64 == 0 && cout % 64 == 0 && cin >= 64 && cout >= 64 && cin <= 16384 && cout <= 16384) ? 1 : 0;
}

// partial-statistics rows the forward writes ([rows][2][cout] fp32)
int madnn_conv1x1_stat_rows(int64_t M, int64_t cin, int64_t cout) {
  if (!madnn_conv1x1_supported(cin, cout) || M <= 0) return 0;
  GemmArgs p{};
  plan_persistent(p, M, cout % 128 == 0 ? 128 : 64, cout, cin);
  return p.j_groups;
}

// partial rows the BNB data grad writes ([rows][2][cin] fp32)
int madnn_conv1x1_dgrad_rows(int64_t M, int64_t cin, int64_t cout) {
  if (!madnn_conv1x1_supported(cin, cout) || M <= 0) return 0;
  GemmArgs p{};
  plan_persistent(p, M, cin % 128 == 0 ? 128 : 64, cin, cout);
  return p.j_groups;
}

hipError_t madnn_conv1x1_fwd(const void* x, const void* w, void* y, float* stats, int64_t M, int64_t cin,
                             int64_t cout, hipStream_t s) {
  if (!madnn_conv1x1_supported(cin, cout)) return hipErrorInvalidValue;
  if (M <= 0) return hipSuccess;
  GemmArgs p{};
  p.a = static_cast<const uint16_t*>(w);
  p.lda = cin;
  p.b = static_cast<const uint16_t*>(x);
  p.ldb = cin;
  p.out = y;
  p.ldo = cout;
  p.stats = stats;
  p.xcd = tune().xcd;
  p.I = cout;
  p.J = M;
  p.K = cin;
  const bool wide = cout % 128 == 0;
  plan_persistent(p, M, wide ? 128 : 64, cout, cin);
  const int grid = p.i_tiles * p.j_groups;
  if (wide) {
    return stats ? launch<false, false, 128, 128, kStoreT, true>(p, grid, s)
                 : launch<false, false, 128, 128, kStoreT, false>(p, grid, s);
  }
  return stats ? launch<false, false, 64, 128, kStoreT, true>(p, grid, s)
               : launch<false, false, 64, 128, kStoreT, false>(p, grid, s);
}

// dx = dY W (+ res: an accumulated gradient of the same layout, added in the epilogue)
// bny/bnsc/bnsh/partial (optional, all or none): dx is d relu(bn(bny)); the epilogue also writes bn's
// backward sums as partial [madnn_conv1x1_dgrad_rows][2][cin] (see BNB)
// resmask (with res): res counts only where its ReLU bit is set
hipError_t madnn_conv1x1_dgrad(const void* dy, const void* w, void* dx, const void* res, int64_t M, int64_t cin,
                               int64_t cout, const void* bny, const float* bnsc, const float* bnsh, float* partial,
                               hipStream_t s, const unsigned char* resmask) {
  if (!madnn_conv1x1_supported(cin, cout)) return hipErrorInvalidValue;
  if (M <= 0) return hipSuccess;
  GemmArgs p{};
  p.a = static_cast<const uint16_t*>(w);  // A[i = ci][k = co] = W[co][ci]: column memory
  p.lda = cin;
  p.b = static_cast<const uint16_t*>(dy);  // B[k = co][j = m] = dY[m][co]: row memory
  p.ldb = cout;
  p.out = dx;
  p.res = static_cast<const uint16_t*>(res);
  p.resmask = res != nullptr ? resmask : nullptr;
  p.xcd = tune().xcd;
  p.ldo = cin;
  p.I = cin;
  p.J = M;
  p.K = cout;
  const bool wide = cin % 128 == 0;
  plan_persistent(p, M, wide ? 128 : 64, cin, cout);
  const int grid = p.i_tiles * p.j_groups;
  if (bny != nullptr) {
    if (partial == nullptr || bnsc == nullptr || bnsh == nullptr || res != nullptr) return hipErrorInvalidValue;
    p.bny = static_cast<const uint16_t*>(bny);
    p.bnsc = bnsc;
    p.bnsh = bnsh;
    p.stats = partial;
    return wide ? launch<true, false, 128, 128, kStoreT, false, true>(p, grid, s)
                : launch<true, false, 64, 128, kStoreT, false, true>(p, grid, s);
  }
  return wide ? launch<true, false, 128, 128, kStoreT, false>(p, grid, s)
              : launch<true, false, 64, 128, kStoreT, false>(p, grid, s);
}

// fp32 floats of workspace madnn_conv1x1_wgrad needs (the per-split partial slabs)
int64_t madnn_conv1x1_wgrad_ws(int64_t M, int64_t cin, int64_t cout) {
  int bi, bj, kc;
  int64_t tiles, splits;
  wgrad_split(M, cin, cout, bi, bj, tiles, kc, splits);
  return splits * cin * cout;
}

// dw: [cout][cin] fp32 or (dw_bf16) bf16; ws: madnn_conv1x1_wgrad_ws floats (the per-split partial
// slabs, summed in split order into dw -- one pass that also casts)
hipError_t madnn_conv1x1_wgrad(const void* dy, const void* x, void* dw, int dw_bf16, float* ws, int64_t M, int64_t cin,
                               int64_t cout, hipStream_t s) {
  if (!madnn_conv1x1_supported(cin, cout)) return hipErrorInvalidValue;
  if (M <= 0) return hipMemsetAsync(dw, 0, (size_t)(cin * cout) * (dw_bf16 ? 2 : 4), s);
  GemmArgs p{};
  p.a = static_cast<const uint16_t*>(dy);  // A[i = co][k = m] = dY[m][co]: column memory
  p.lda = cout;
  p.b = static_cast<const uint16_t*>(x);  // B[k = m][j = ci] = X[m][ci]: column memory
  p.ldb = cin;
  p.xcd = tune().xcd;
  p.ldo = cin;
  p.I = cout;
  p.J = cin;
  p.K = M;
  int bi, bj;
  int64_t tiles, splits;
  wgrad_split(M, cin, cout, bi, bj, tiles, p.k_chunk, splits);
  if (ws == nullptr) return hipErrorInvalidValue;
  p.out = ws;
  p.i_tiles = (int)(cout / bi);
  p.j_tiles = (int)(cin / bj);
  const int grid = (int)(tiles * splits);
  p.j_groups = 0;
  hipError_t e;
  if (bi == 128 && bj == 128) e = launch<true, true, 128, 128, kSplit, false>(p, grid, s);
  else if (bi == 128) e = launch<true, true, 128, 64, kSplit, false>(p, grid, s);
  else if (bj == 128) e = launch<true, true, 64, 128, kSplit, false>(p, grid, s);
  else e = launch<true, true, 64, 64, kSplit, false>(p, grid, s);
  if (e != hipSuccess) return e;
  const int64_t n = cin * cout;
  const int64_t blocks = (n / 4 + 255) / 256;
  const dim3 grid_r((unsigned)(blocks < 4 * madnn::kNumCU ? blocks : 4 * madnn::kNumCU));
  if (dw_bf16) {
    hipLaunchKernelGGL(split_reduce_kernel<true>, grid_r, dim3(256), 0, s, ws, (int)splits, n, dw);
  } else {
    hipLaunchKernelGGL(split_reduce_kernel<false>, grid_r, dim3(256), 0, s, ws, (int)splits, n, dw);
  }
  return hipGetLastError();
}

}  // extern "C"
