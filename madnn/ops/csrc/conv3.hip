// K13 — NHWC 3x3 / stride 1 / pad 1 convolution on MFMA for gfx950 (forward with the following
// BatchNorm's batch statistics in the epilogue; the data gradient is the same kernel run on the
// flipped, transposed weight).
//
// Why: ResNet-50's 3x3 stride-1 convolutions on MIOpen's find-db solvers run at 0.18-0.34 of
// their roofline bound in every pass (profiles/r2_resnet50_conv_roofline_b1536.md: 26 ms/step
// against 6.5 ms at batch 1536) -- the furthest of any kernel family in the step.
//
// Structure: implicit GEMM  D[co][m] = sum_{tap, ci} W[co][tap][ci] X[pix(m) + off(tap)][ci]
// with the output pixel m on the MFMA lane and the output channel co on the accumulator rows
// (a lane owns 4 consecutive co of one pixel, the K9 orientation).  A workgroup (4 waves)
// owns 256 consecutive output pixels (NHWC order) x 64 output channels; each wave 64 pixels x 64
// channels = 2 x 2 v_mfma_f32_32x32x16_bf16 accumulators.  Per 64-channel input chunk the
// workgroup stages the input HALO once -- every input row the tile's 3x3 windows touch, a
// contiguous NHWC range -- into LDS, so the nine taps read it nine times from LDS instead of
// nine times from L2.  The weights of one (tap, chunk), [64 co][64 ci] = 8 KiB, stream through a
// two-slot LDS ring one tap ahead.  Both images are filled by LDS-DMA (global_load_lds, 16 B per
// lane, lane-linear destination) with the swz<64> XOR applied to the per-lane source address
// (cdna_hip_programming.md rule 21), and read conflict-free with ds_read_b128.
// A tap whose source pixel leaves the image (top/bottom rows, first/last column, image seams in
// the flattened NHWC order) reads a zero row in LDS instead: no data-dependent branches.
// Stages are 32 input channels (64-B pixel rows; `MADNN_K13_CH=64` selects 128-B rows): LDS =
// halo (<= (255/W + 4) * W pixels x 64 B, 28 KiB at W = 56) + zero row + 8 KiB of weights, so four
// workgroups share a CU and one workgroup's halo / weight loads and epilogue stores overlap the
// others' MFMAs (measured: a kernel with the MFMAs removed still took 70 % of the time at two
// workgroups per CU, and a persistent double-buffered variant at one workgroup per CU was 1.7x
// slower -- occupancy, not explicit double buffering, hides this kernel's memory latency).
// Epilogue: the K9 LDS-transposed row store (16-B stores of 64 contiguous channels per pixel)
// and, with `stats`, per-channel sum / sum of squares of the bf16-rounded outputs as one
// [2][Cout] partial row per pixel tile (the input of bn.hip's finalize).
#include <cstdlib>

#include "mfma.h"

namespace madnn {
namespace conv3 {

using namespace mf;

constexpr int kThreads = 256;
constexpr int kBJ = 256;  // output pixels per workgroup
constexpr int kBI = 64;   // output channels per workgroup
constexpr int kWElems = 64 * 64;  // one (tap, chunk) weight tile

typedef __attribute__((address_space(3))) void lds_void;

struct Args {
  const uint16_t* x;   // [M = N*H*W][Ci]
  const uint16_t* w;   // [Co][9][Ci] (channels_last weight)
  uint16_t* y;         // [M][Co]
  float* stats;        // [m_tiles][2][Co] or null
  const uint16_t* bny;  // BNB epilogue: the BatchNorm input y [M][Co] whose backward sums are taken
  const float* bnsc;    //   its forward scale / shift (ReLU mask = y * sc + sh > 0)
  const float* bnsh;
  int64_t M;           // output pixels
  int64_t Min;         // input pixels (= M at stride 1)
  int H, W, Ci, Co;    // INPUT image height / width
  int Wo;              // output width (W / SD)
  int halo_px;         // LDS halo capacity in pixels
  int m_tiles, co_tiles;
};

__device__ __forceinline__ int fswz(int row) { return (((row >> 1) & 1) << 2) | ((row >> 2) & 3); }

// chunk geometry: CH input channels per stage, pixel rows of RB = 2 CH bytes (NC 16-B chunks),
// swizzle f(row) (128-B rows: fswz; 64-B rows: (row >> 2) & 3 -- both conflict-free for the 16
// consecutive rows of a ds_read_b128 lane group at any row alignment, i.e. for every tap shift)
template <int CH>
struct Chunk {
  static constexpr int RB = 2 * CH, NC = CH / 8, RPI = 1024 / RB, KS = CH / 16, WE = 64 * CH;
  static __device__ __forceinline__ int f(int row) {
    if constexpr (CH == 64) return fswz(row);
    else return (row >> 2) & 3;
  }
  static __device__ __forceinline__ int off(int row, int ch) { return row * RB + 16 * (ch ^ f(row)); }
};

// halo capacity in pixels: a tile of kBJ output pixels spans at most (kBJ - 1) / Wo + 2 output rows,
// i.e. SD * ((kBJ - 1) / Wo + 1) + 3 input rows of W pixels (stride 1: (kBJ - 1) / W + 4)
__host__ __device__ inline int halo_rows_px(int W, int rpi, int sd = 1) {
  const int Wo = W / sd;
  return ((sd * ((kBJ - 1) / Wo + 1) + 3) * W + rpi - 1) / rpi * rpi;
}

__host__ inline size_t conv3x3_lds(int W, int CH, int sd = 1) {
  const size_t rb = 2 * CH, cap = (size_t)halo_rows_px(W, 1024 / (int)rb, sd) * rb + rb + 2 * 64 * rb;
  return cap > 32 * 1024 ? cap : 32 * 1024;  // the epilogue's [256][64] bf16 tile reuses the whole image
}

// BNB (data grad of a convolution whose input was relu(bn(y))): the epilogue also accumulates the
// BatchNorm backward's two sums over its output tile, sum g and sum g*y with g = out * [y*sc+sh > 0]
// (out = the bf16-rounded input gradient it stores), as the [m_tiles][2][Co] partial rows of
// bn.hip's backward finalize -- the BN backward then skips its reduction pass over (dx, y).
// SD = 2 (ResNet's stride-2 3x3, H and W even): output pixel (n, ho, wo) reads input rows 2 ho - 1 ..
// 2 ho + 1 -- global output row r maps to global input row 2 r (n H + 2 ho), so a tile's halo is still
// ONE contiguous NHWC range, rows 2 r_first - 1 .. 2 r_last + 1, and a tap is still a uniform shift
// of the lane's centre pixel (2 wo in its row); only the halo is about twice as tall.
template <int CH, bool STATS, bool BNB = false, int SD = 1>
__global__ __launch_bounds__(kThreads, CH == 32 ? 4 : 2) void conv3x3_kernel(const Args p) {
  static_assert(!(STATS && BNB), "one statistics epilogue per launch");
  using C = Chunk<CH>;
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t* halo = smem;                                     // [halo_px][CH]
  uint16_t* zrow = smem + (int64_t)p.halo_px * CH;           // [1][CH] zeros
  uint16_t* wring = zrow + CH;                               // [2][64][CH]
  const int tid = threadIdx.x, lane = tid & 63, l32 = lane & 31, hh = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  // XCD-grouped logical id; output-channel tile fastest (co tiles of one pixel tile share its halo in L2)
  int wid = blockIdx.x;
  {
    const int n = gridDim.x, x = wid % 8, q8 = n / 8, r8 = n % 8;
    wid = (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + wid / 8;
  }
  const int cot = wid % p.co_tiles, mt = wid / p.co_tiles;
  const int64_t j0 = (int64_t)mt * kBJ;
  const int co0 = cot * kBI;
  const int W = p.W, H = p.H, Wo = SD == 1 ? p.W : p.Wo, Ho = H / SD;
  const int64_t r_first = j0 / Wo;                     // output rows (global over N x Ho)
  const int64_t j_last = min(j0 + kBJ, p.M) - 1;
  const int64_t hrow0 = SD * r_first - 1;              // first halo row (may be -1: clamped, never read)
  const int hpx = (int)((SD * (j_last / Wo - r_first) + 3) * W);  // halo pixels this tile

  // per-lane output pixels (two 32-pixel blocks of this wave): centre-tap halo index + edge flags
  int hb[2];
  unsigned edge[2];  // bit0: h >= 1 (row above exists), bit1: h <= H-2, bit2: w >= 1, bit3: w <= W-2
#pragma unroll
  for (int jb = 0; jb < 2; ++jb) {
    int64_t m = j0 + wave * 64 + jb * 32 + l32;
    m = m < p.M ? m : p.M - 1;
    const int64_t r = m / Wo;
    const int wo = (int)(m - r * Wo);
    const int ho = (int)(r % Ho);
    // centre input pixel (SD ho, SD wo); with SD = 2 the row below / column right always exist
    const int h = SD * ho, wc = SD * wo;
    hb[jb] = (int)(SD * r - hrow0) * W + wc;
    edge[jb] = (h >= 1 ? 1u : 0u) | (h <= H - 2 ? 2u : 0u) | (wc >= 1 ? 4u : 0u) | (wc <= W - 2 ? 8u : 0u);
  }
  if (tid < C::NC) *reinterpret_cast<u32x4*>(zrow + tid * 8) = u32x4{0u, 0u, 0u, 0u};

  const int nchunk = p.Ci / CH;
  const int total = nchunk * 9;
  const int64_t ldw = 9LL * p.Ci;

  // LDS-DMA of the halo of input chunk c: RPI pixel rows (1 KiB) per wave-instruction
  auto stage_halo = [&](int c) {
    const int ninst = (hpx + C::RPI - 1) / C::RPI;
    for (int i = wave; i < ninst; i += 4) {
      const int prow = i * C::RPI + lane / C::NC;
      const int ch = (lane % C::NC) ^ C::f(prow);
      int64_t src = hrow0 * W + prow;
      src = src < 0 ? 0 : (src >= p.Min ? p.Min - 1 : src);
      __builtin_amdgcn_global_load_lds((const void*)(p.x + src * p.Ci + c * CH + 8 * ch),
                                       (lds_void*)(halo + i * 512), 16, 0, 0);
    }
  };
  // weights of (chunk c, tap t) into ring slot `slot`: 64 rows of RB bytes, 64 * RB / 1 KiB instructions
  auto stage_w = [&](int c, int t, int slot) {
    constexpr int NI = 64 * C::RB / 1024;
    for (int inst = wave; inst < NI; inst += 4) {
      const int row = inst * C::RPI + lane / C::NC;
      const int ch = (lane % C::NC) ^ C::f(row);
      __builtin_amdgcn_global_load_lds((const void*)(p.w + (int64_t)(co0 + row) * ldw + t * p.Ci + c * CH + 8 * ch),
                                       (lds_void*)(wring + slot * C::WE + inst * 512), 16, 0, 0);
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = zero16();

  stage_halo(0);
  stage_w(0, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const char* hbase = reinterpret_cast<const char*>(halo);
  const char* zbase = reinterpret_cast<const char*>(zrow);
  int c = 0, t = 0;
  for (int idx = 0; idx < total; ++idx) {
    // next step's weights into the other slot (its last reader finished before the last barrier)
    int cn = c, tn = t + 1;
    if (tn == 9) {
      tn = 0;
      ++cn;
    }
    if (idx + 1 < total) stage_w(cn, tn, (idx + 1) & 1);
    const char* wt = reinterpret_cast<const char*>(wring + (idx & 1) * C::WE);
    // this tap's B-fragment row addresses (halo pixel or the zero row)
    const int dh = t / 3, dw = t - 3 * (t / 3);
    const unsigned need = (dh == 0 ? 1u : dh == 2 ? 2u : 0u) | (dw == 0 ? 4u : dw == 2 ? 8u : 0u);
    const char* brow[2];
    int bsw[2];
#pragma unroll
    for (int jb = 0; jb < 2; ++jb) {
      const int hp = hb[jb] + (dh - 1) * W + (dw - 1);
      const bool ok = (edge[jb] & need) == need;
      brow[jb] = ok ? hbase + hp * C::RB : zbase;
      bsw[jb] = ok ? C::f(hp) : 0;
    }
#pragma unroll
    for (int s = 0; s < C::KS; ++s) {
      bf16x8 af[2], bv[2];
#pragma unroll
      for (int a = 0; a < 2; ++a) af[a] = *reinterpret_cast<const bf16x8*>(wt + C::off(a * 32 + l32, 2 * s + hh));
#pragma unroll
      for (int b = 0; b < 2; ++b) bv[b] = *reinterpret_cast<const bf16x8*>(brow[b] + 16 * ((2 * s + hh) ^ bsw[b]));
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = mfma(af[a], bv[b], acc[a][b]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // next weights landed; this tap's reads of the ring slot / halo are done
    if (tn == 0 && cn < nchunk) {  // next input chunk: restage the halo (every wave is past its reads)
      stage_halo(cn);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
    c = cn;
    t = tn;
  }

  // ---- epilogue: D[co][px] -> bf16 tile [256 px][64 co] in LDS (128-B rows) -> 16-B row stores
  char* ot = reinterpret_cast<char*>(smem);  // the whole image (>= 32 KiB) is free now
  auto out_off = [](int r, int ch) { return r * 128 + 16 * (ch ^ ((r >> 1) & 7)); };
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const int pr = wave * 64 + b * 32 + l32;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int ic = a * 32 + 8 * g + 4 * hh;
        const unsigned lo = (unsigned)f32_to_bf16(acc[a][b][4 * g]) | ((unsigned)f32_to_bf16(acc[a][b][4 * g + 1]) << 16);
        const unsigned hi = (unsigned)f32_to_bf16(acc[a][b][4 * g + 2]) | ((unsigned)f32_to_bf16(acc[a][b][4 * g + 3]) << 16);
        *reinterpret_cast<u32x2*>(ot + out_off(pr, ic >> 3) + 8 * ((ic >> 2) & 1)) = u32x2{lo, hi};
      }
  }
  // BNB: fetch this thread's 8 rows of y now -- the accumulators are dead, so the 8 x 16 B land in
  // their registers and the loads overlap the barrier and the LDS tile reads below
  constexpr int kRowsPerThread = kBJ / (kThreads / 8);
  u32x4 ypre[BNB ? kRowsPerThread : 1];
  if constexpr (BNB) {
#pragma unroll
    for (int k = 0; k < kRowsPerThread; ++k) {
      const int64_t m = j0 + (tid >> 3) + k * (kThreads / 8);
      ypre[k] = m < p.M ? *reinterpret_cast<const u32x4*>(p.bny + m * p.Co + co0 + 8 * (tid & 7)) : u32x4{0, 0, 0, 0};
    }
  }
  __syncthreads();
  const int ch = tid & 7;
  float ssum[8], ssq[8], bs[8], bh[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) ssum[e] = ssq[e] = 0.f;
  if constexpr (BNB) {  // this thread's 8 channels are fixed for the whole tile
    const f32x4* sc4 = reinterpret_cast<const f32x4*>(p.bnsc + co0 + 8 * ch);
    const f32x4* sh4 = reinterpret_cast<const f32x4*>(p.bnsh + co0 + 8 * ch);
    const f32x4 s0 = sc4[0], s1 = sc4[1], h0 = sh4[0], h1 = sh4[1];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      bs[e] = s0[e];
      bs[4 + e] = s1[e];
      bh[e] = h0[e];
      bh[4 + e] = h1[e];
    }
  }
#pragma unroll
  for (int k = 0; k < kRowsPerThread; ++k) {
    const int r = (tid >> 3) + k * (kThreads / 8);
    const int64_t m = j0 + r;
    if (m >= p.M) break;
    const u32x4 v = *reinterpret_cast<const u32x4*>(ot + out_off(r, ch));
    *reinterpret_cast<u32x4*>(p.y + m * p.Co + co0 + 8 * ch) = v;
    if constexpr (BNB) {
      const u32x4 yv = ypre[k];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          const int k = 2 * e + hf;
          const float g = bf16_to_f32((unsigned short)(hf ? v[e] >> 16 : v[e] & 0xffffu));
          const float yy = bf16_to_f32((unsigned short)(hf ? yv[e] >> 16 : yv[e] & 0xffffu));
          const float gm = yy * bs[k] + bh[k] > 0.f ? g : 0.f;
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
  if constexpr (STATS || BNB) {
    __syncthreads();  // the tile image is consumed
    float* red = reinterpret_cast<float*>(smem);  // [32 row groups][2][64], 16-B vector writes
    const int rg = tid >> 3;
    *reinterpret_cast<f32x4*>(red + (rg * 2) * 64 + 8 * ch) = f32x4{ssum[0], ssum[1], ssum[2], ssum[3]};
    *reinterpret_cast<f32x4*>(red + (rg * 2) * 64 + 8 * ch + 4) = f32x4{ssum[4], ssum[5], ssum[6], ssum[7]};
    *reinterpret_cast<f32x4*>(red + (rg * 2 + 1) * 64 + 8 * ch) = f32x4{ssq[0], ssq[1], ssq[2], ssq[3]};
    *reinterpret_cast<f32x4*>(red + (rg * 2 + 1) * 64 + 8 * ch + 4) = f32x4{ssq[4], ssq[5], ssq[6], ssq[7]};
    __syncthreads();
    if (tid < 128) {
      const int which = tid >> 6, ci = tid & 63;
      float v = 0.f;
      for (int g = 0; g < kThreads / 8; ++g) v += red[(g * 2 + which) * 64 + ci];
      p.stats[((int64_t)mt * 2 + which) * p.Co + co0 + ci] = v;
    }
  }
}

// ------------------------------------------------------------------ weight gradient
// dW[co][tap][ci] = sum_m dY[m][co] X[pix(m) + off(tap)][ci]: one wave per tap (9 waves), each
// a 64 (co) x 64 (ci) block = 2 x 2 accumulators, reducing over the pixels of a tile of R whole
// output rows of one image.  Both the dY tile and the input halo (R + 2 rows) sit in LDS in a
// zero-padded row layout of W + 2 slots per image row (pixel w at slot w + 1), so for every tap
// the halo slot of reduction index k is k + dh (W + 2) + dw - 1: a uniform shift, and taps that
// leave the image read the zero pad columns / zero rows.  Reduction index k runs over the padded
// dY slots (pads hold zero dY, rounded up to 16), read with the transposing ds_read_b64_tr_b16
// (k down the LDS rows, swz<64> images).  Workgroups split the tiles of a (co, ci) block; each
// writes fp32 partials [split][Co][9][Ci]; wgrad_reduce sums them in split order (deterministic)
// into the channels_last weight layout.  The next tile's loads are issued into registers before
// this tile's MFMAs and written to LDS after them.
constexpr int kWThreads = 576;  // 9 waves
constexpr int kWMaxChunks = 8;  // per thread per tile: dY + halo 16-B chunks

struct WArgs {
  const uint16_t* x;   // [M][Ci]
  const uint16_t* dy;  // [M][Co]
  float* ws;           // [splits][Co][9][Ci]
  int N, H, W, Ci, Co;
  int R, kpad, xslots, tiles_per_img, ntiles;
  int co_tiles, ci_tiles, splits;
};

__host__ __device__ inline int wgrad_rows(int H, int W) {
  int R = 1;
  for (int r = 1; r <= H; ++r)
    if (H % r == 0 && r * (W + 2) <= 256) R = r;
  return R;
}

__global__ __launch_bounds__(kWThreads) void conv3x3_wgrad_kernel(const WArgs p) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t* sdy = smem;                       // [kpad][64]
  uint16_t* sx = smem + (int64_t)p.kpad * 64;  // [xslots][64]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // = tap
  const int W = p.W, WP = p.W + 2;
  const int pair = blockIdx.x % (p.co_tiles * p.ci_tiles), split = blockIdx.x / (p.co_tiles * p.ci_tiles);
  const int co0 = (pair % p.co_tiles) * 64, ci0 = (pair / p.co_tiles) * 64;

  // zero both images once: pad columns, pad rows and slack stay zero (tile writes touch real pixels only)
  for (int i = tid; i < (p.kpad + p.xslots) * 8; i += kWThreads)
    *reinterpret_cast<u32x4*>(smem + (int64_t)i * 8) = u32x4{0u, 0u, 0u, 0u};

  // this thread's 16-B chunks of a tile (identical for every tile): LDS element offset, global
  // element offset relative to the tile's first pixel row, halo row (-1: a dY chunk)
  const int ndy = p.R * W * 8, nx = (p.R + 2) * W * 8;
  // loc[u]: LDS element offset (< 2^18) | (halo row + 1) << 24 (0: a dY chunk); -1: no chunk
  int loc[kWMaxChunks], gofs[kWMaxChunks];  // gofs < (R + 1) W Ci < 2^31
#pragma unroll
  for (int u = 0; u < kWMaxChunks; ++u) {
    const int i = tid + kWThreads * u;
    loc[u] = -1;
    gofs[u] = 0;
    if (i < ndy) {
      const int ch = i & 7, px = i >> 3, rr = px / W, w = px - rr * W;
      const int slot = rr * WP + w + 1;
      loc[u] = slot * 64 + 8 * (ch ^ fswz(slot));
      gofs[u] = (rr * W + w) * p.Co + co0 + 8 * ch;
    } else if (i < ndy + nx) {
      const int j = i - ndy, ch = j & 7, px = j >> 3, q = px / W, w = px - q * W;
      const int slot = 1 + q * WP + w + 1;
      loc[u] = (p.kpad * 64 + slot * 64 + 8 * (ch ^ fswz(slot))) | ((q + 1) << 24);
      gofs[u] = ((q - 1) * W + w) * p.Ci + ci0 + 8 * ch;
    }
  }
  u32x4 stg[kWMaxChunks];
  auto load_tile = [&](int t) {
    const int n = t / p.tiles_per_img, h0 = (t - n * p.tiles_per_img) * p.R;
    const int64_t pix0 = ((int64_t)n * p.H + h0) * W;
#pragma unroll
    for (int u = 0; u < kWMaxChunks; ++u) {
      stg[u] = u32x4{0u, 0u, 0u, 0u};
      if (loc[u] >= 0) {
        const int q1 = loc[u] >> 24;
        if (q1 == 0) {
          stg[u] = *reinterpret_cast<const u32x4*>(p.dy + pix0 * p.Co + gofs[u]);
        } else {
          const int hr = h0 + q1 - 2;
          if (hr >= 0 && hr < p.H) stg[u] = *reinterpret_cast<const u32x4*>(p.x + pix0 * p.Ci + gofs[u]);
        }
      }
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int u = 0; u < kWMaxChunks; ++u)
      if (loc[u] >= 0) *reinterpret_cast<u32x4*>(smem + (loc[u] & 0xffffff)) = stg[u];
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = zero16();
  const int dh = wave / 3, dw = wave - 3 * (wave / 3);
  const int shift = 1 + dh * WP + dw - 1;  // halo slot of reduction index k = k + shift
  const int nk = p.kpad / 16;

  int t = split;
  __syncthreads();  // zero fill done
  if (t < p.ntiles) {
    load_tile(t);
    store_tile();
  }
  __syncthreads();
  for (; t < p.ntiles; t += p.splits) {
    const int tn = t + p.splits;
    if (tn < p.ntiles) load_tile(tn);
    for (int ks = 0; ks < nk; ++ks) {
      bf16x8 af[2], bv[2];
#pragma unroll
      for (int a = 0; a < 2; ++a) af[a] = lds_col<64>(sdy, 16 * ks, a * 32, lane);
#pragma unroll
      for (int b = 0; b < 2; ++b) bv[b] = lds_col<64>(sx, 16 * ks + shift, b * 32, lane);
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = mfma(af[a], bv[b], acc[a][b]);
    }
    __syncthreads();  // every wave is done reading this tile
    if (tn < p.ntiles) store_tile();
    __syncthreads();
  }
  // partial [split][co][tap][ci]: lane holds D[co = a*32 + acc_row(r, h)][ci = b*32 + (lane & 31)]
  const int hh = lane >> 5, l32 = lane & 31;
  float* out = p.ws + (int64_t)split * p.Co * 9 * p.Ci;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = co0 + a * 32 + acc_row(r, hh);
        out[((int64_t)co * 9 + wave) * p.Ci + ci0 + b * 32 + l32] = acc[a][b][r];
      }
}

// out[e] = sum_s ws[s][e] (fixed order), fp32 or bf16
__global__ __launch_bounds__(256) void conv3x3_wgrad_reduce_kernel(const float* __restrict__ ws, int splits,
                                                                   int64_t n, void* __restrict__ out, int bf16) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * 4;
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n; i += stride) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < splits; ++s) acc += *reinterpret_cast<const f32x4*>(ws + (int64_t)s * n + i);
    if (bf16) {
      const unsigned lo = (unsigned)f32_to_bf16(acc[0]) | ((unsigned)f32_to_bf16(acc[1]) << 16);
      const unsigned hi = (unsigned)f32_to_bf16(acc[2]) | ((unsigned)f32_to_bf16(acc[3]) << 16);
      *reinterpret_cast<u32x2*>(static_cast<uint16_t*>(out) + i) = u32x2{lo, hi};
    } else {
      *reinterpret_cast<f32x4*>(static_cast<float*>(out) + i) = acc;
    }
  }
}

}  // namespace conv3
}  // namespace madnn

using namespace madnn::conv3;

extern "C" {

// chunk width: 32 input channels per LDS stage (LDS ~37 KiB at W = 56: four workgroups per CU; the
// 64-channel variant measured slower and was removed in round 6)
static int k13_ch(int) { return 32; }

int madnn_conv3x3_supported(int H, int W, int Ci, int Co) {
  if (H < 1 || W < 1 || Ci % 64 || Co % 64 || Ci < 64 || Co < 64 || Ci > 8192) return 0;
  return conv3x3_lds(W, k13_ch(Ci)) <= 80 * 1024 ? 1 : 0;  // at least two workgroups per CU
}

int madnn_conv3x3_stat_rows(int64_t M) { return (int)((M + kBJ - 1) / kBJ); }

// y = conv3x3(x, w) (stride 1, pad 1); x [N, H, W, Ci] NHWC, w [Co, 3, 3, Ci] (channels_last),
// y [N, H, W, Co]; stats (optional): [ceil(M/256)][2][Co] partial sums of y
hipError_t madnn_conv3x3_fwd(const void* x, const void* w, void* y, float* stats, int N, int H, int W, int Ci, int Co,
                             hipStream_t s) {
  if (!madnn_conv3x3_supported(H, W, Ci, Co)) return hipErrorInvalidValue;
  Args p{};
  p.x = static_cast<const uint16_t*>(x);
  p.w = static_cast<const uint16_t*>(w);
  p.y = static_cast<uint16_t*>(y);
  p.stats = stats;
  p.M = (int64_t)N * H * W;
  if (p.M <= 0) return hipSuccess;
  p.Min = p.M;
  p.H = H;
  p.W = W;
  p.Wo = W;
  p.Ci = Ci;
  p.Co = Co;
  const int CH = k13_ch(Ci);
  p.halo_px = halo_rows_px(W, 1024 / (2 * CH));
  p.m_tiles = (int)((p.M + kBJ - 1) / kBJ);
  p.co_tiles = Co / kBI;
  const int64_t grid = (int64_t)p.m_tiles * p.co_tiles;
  if (grid > 0x7fffffff) return hipErrorInvalidValue;
  const size_t lds = conv3x3_lds(W, CH);
  const dim3 g((unsigned)grid), b(kThreads);
  if (stats) hipLaunchKernelGGL((conv3x3_kernel<32, true>), g, b, lds, s, p);
  else hipLaunchKernelGGL((conv3x3_kernel<32, false>), g, b, lds, s, p);
  return hipGetLastError();
}

// Stride 2 (pad 1): x [N, H, W, Ci] with H, W even -> y [N, H/2, W/2, Co]; stats as above over the
// output.  The halo is about twice as tall as at stride 1: one workgroup per CU at W = 56 (82 KiB).
int madnn_conv3x3_s2_supported(int H, int W, int Ci, int Co) {
  if (H < 2 || W < 2 || (H & 1) || (W & 1) || Ci % 64 || Co % 64 || Ci < 64 || Co < 64 || Ci > 8192) return 0;
  return conv3x3_lds(W, k13_ch(Ci), 2) <= 160 * 1024 ? 1 : 0;
}

int madnn_conv3x3_s2_stat_rows(int N, int H, int W) { return (int)(((int64_t)N * (H / 2) * (W / 2) + kBJ - 1) / kBJ); }

hipError_t madnn_conv3x3_fwd_s2(const void* x, const void* w, void* y, float* stats, int N, int H, int W, int Ci,
                                int Co, hipStream_t s) {
  if (!madnn_conv3x3_s2_supported(H, W, Ci, Co)) return hipErrorInvalidValue;
  Args p{};
  p.x = static_cast<const uint16_t*>(x);
  p.w = static_cast<const uint16_t*>(w);
  p.y = static_cast<uint16_t*>(y);
  p.stats = stats;
  p.M = (int64_t)N * (H / 2) * (W / 2);
  if (p.M <= 0) return hipSuccess;
  p.Min = (int64_t)N * H * W;
  p.H = H;
  p.W = W;
  p.Wo = W / 2;
  p.Ci = Ci;
  p.Co = Co;
  const int CH = k13_ch(Ci);
  p.halo_px = halo_rows_px(W, 1024 / (2 * CH), 2);
  p.m_tiles = (int)((p.M + kBJ - 1) / kBJ);
  p.co_tiles = Co / kBI;
  const int64_t grid = (int64_t)p.m_tiles * p.co_tiles;
  if (grid > 0x7fffffff) return hipErrorInvalidValue;
  const size_t lds = conv3x3_lds(W, CH, 2);
  const dim3 g((unsigned)grid), b(kThreads);
  if (stats) hipLaunchKernelGGL((conv3x3_kernel<32, true, false, 2>), g, b, lds, s, p);
  else hipLaunchKernelGGL((conv3x3_kernel<32, false, false, 2>), g, b, lds, s, p);
  return hipGetLastError();
}

// Data grad with the BatchNorm-backward sums in the epilogue (see BNB): x = the output gradient,
// w = the flipped / transposed weight, y = dx; partial [ceil(M/256)][2][Co] = (sum g, sum g*bny)
hipError_t madnn_conv3x3_fwd_bnb(const void* x, const void* w, void* y, float* partial, const void* bny,
                                 const float* bnsc, const float* bnsh, int N, int H, int W, int Ci, int Co,
                                 hipStream_t s) {
  if (!madnn_conv3x3_supported(H, W, Ci, Co) || partial == nullptr || bny == nullptr) return hipErrorInvalidValue;
  Args p{};
  p.x = static_cast<const uint16_t*>(x);
  p.w = static_cast<const uint16_t*>(w);
  p.y = static_cast<uint16_t*>(y);
  p.stats = partial;
  p.bny = static_cast<const uint16_t*>(bny);
  p.bnsc = bnsc;
  p.bnsh = bnsh;
  p.M = (int64_t)N * H * W;
  if (p.M <= 0) return hipSuccess;
  p.Min = p.M;
  p.H = H;
  p.W = W;
  p.Wo = W;
  p.Ci = Ci;
  p.Co = Co;
  const int CH = k13_ch(Ci);
  p.halo_px = halo_rows_px(W, 1024 / (2 * CH));
  p.m_tiles = (int)((p.M + kBJ - 1) / kBJ);
  p.co_tiles = Co / kBI;
  const int64_t grid = (int64_t)p.m_tiles * p.co_tiles;
  if (grid > 0x7fffffff) return hipErrorInvalidValue;
  const size_t lds = conv3x3_lds(W, CH);
  const dim3 g((unsigned)grid), b(kThreads);
  hipLaunchKernelGGL((conv3x3_kernel<32, false, true>), g, b, lds, s, p);
  return hipGetLastError();
}

// weight-gradient plan: workspace floats needed (0 if unsupported)
static bool wgrad_plan(int N, int H, int W, int Ci, int Co, WArgs& p) {
  if (Ci % 64 || Co % 64 || Ci < 64 || Co < 64 || Ci > 8192 || Co > 8192 || N < 1 || H < 1 || W < 1) return false;
  p.N = N;
  p.H = H;
  p.W = W;
  p.Ci = Ci;
  p.Co = Co;
  p.R = wgrad_rows(H, W);
  const int kreal = p.R * (W + 2);
  if (kreal > 256) return false;
  p.kpad = (kreal + 15) / 16 * 16;
  p.xslots = p.kpad + 2 * (W + 2) + 2;
  if ((p.R * W * 8 + (p.R + 2) * W * 8 + kWThreads - 1) / kWThreads > kWMaxChunks) return false;
  if ((size_t)(p.kpad + p.xslots) * 128 > 160 * 1024) return false;
  p.tiles_per_img = H / p.R;
  p.ntiles = N * p.tiles_per_img;
  p.co_tiles = Co / 64;
  p.ci_tiles = Ci / 64;
  const int pairs = p.co_tiles * p.ci_tiles;
  int splits = (2 * 256 + pairs - 1) / pairs;  // ~2 workgroups per CU over the whole grid
  splits = splits > p.ntiles ? p.ntiles : splits;
  p.splits = splits < 1 ? 1 : splits;
  return true;
}

int64_t madnn_conv3x3_wgrad_ws(int N, int H, int W, int Ci, int Co) {
  WArgs p{};
  if (!wgrad_plan(N, H, W, Ci, Co, p)) return -1;
  return (int64_t)p.splits * Co * 9 * Ci;
}

// dw [Co][3][3][Ci] (channels_last weight layout), fp32 (out_bf16 = 0) or bf16; ws: madnn_conv3x3_wgrad_ws floats
hipError_t madnn_conv3x3_wgrad(const void* dy, const void* x, float* ws, void* dw, int out_bf16, int N, int H, int W,
                               int Ci, int Co, hipStream_t s) {
  WArgs p{};
  if (!wgrad_plan(N, H, W, Ci, Co, p)) return hipErrorInvalidValue;
  p.x = static_cast<const uint16_t*>(x);
  p.dy = static_cast<const uint16_t*>(dy);
  p.ws = ws;
  const size_t lds = (size_t)(p.kpad + p.xslots) * 128;
  const int grid = p.co_tiles * p.ci_tiles * p.splits;
  hipLaunchKernelGGL(conv3x3_wgrad_kernel, dim3(grid), dim3(kWThreads), lds, s, p);
  MADNN_HIP_CHECK(hipGetLastError());
  const int64_t n = (int64_t)Co * 9 * Ci;
  int rg = (int)((n / 4 + 255) / 256);
  rg = rg > 1024 ? 1024 : rg;
  hipLaunchKernelGGL(conv3x3_wgrad_reduce_kernel, dim3(rg), dim3(256), 0, s, ws, p.splits, n, dw, out_bf16);
  return hipGetLastError();
}

}  // extern "C"
