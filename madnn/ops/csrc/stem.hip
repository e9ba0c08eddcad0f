// K10 — the ResNet stem convolution (7x7, stride 2, pad 3, 3 input channels -> 64) on MFMA for
// gfx950, NHWC bf16, forward, with the following BatchNorm's batch statistics in the epilogue.
//
// Why: with 3 input channels the NHWC stem is a poor fit for MIOpen's implicit-GEMM solvers
// (0.9 ms forward at batch 512 on MI355X against a ~0.18 ms HBM bound; zero-padding the channels
// to 4 or 8 is slower still: round-1 A/B).
//
// Implicit GEMM, D[co][p] = sum_k W[co][k] X_patch[p][k], p = output pixel, with the reduction
// ordered k = (kh, kw, c) and padded to 7 x 8 x 4 = 224 (kw = 7 and c = 3 carry zero weights):
//  * a workgroup (4 waves) computes one output row (n, oh) = up to 128 pixels x 64 channels;
//    wave w owns channels 32 (w & 1) .. +31 of pixels 64 (w >> 1) .. +63; persistent
//    workgroups walk output rows;
//  * the 7 input rows a tile needs are staged global -> VGPR -> LDS (double-buffered, one
//    barrier per tile) into a [7][2*Wo+6][4] image: 3 zero pixels of padding on each side and a
//    zero 4th channel, so the 8 reduction elements an MFMA lane needs -- 2 adjacent input pixels
//    x 4 channels -- are one aligned 16-byte ds_read_b128 (pixel 2*ow + kw is even for even kw);
//  * the packed weights (64 x 224 bf16) live in registers for the whole kernel: each lane holds
//    the 14 A fragments of its wave's 32 channels (56 VGPRs), loaded once;
//  * epilogue as K9: accumulators -> LDS [pixel][64] tile -> 16-byte stores (a tile's output row
//    is one contiguous span), summing the bf16-rounded outputs per channel for the BatchNorm.
#include "mfma.h"

namespace madnn {
namespace stem {

using namespace mf;

constexpr int kThreads = 256;
constexpr int kCo = 64;    // output channels
constexpr int kKh = 7;     // kernel rows
constexpr int kKp = 224;   // padded reduction length per output channel: 7 x 8 x 4
constexpr int kSteps = kKp / 16;
constexpr int kMaxWo = 128;

struct StemArgs {
  const uint16_t* x;   // [N][H][W][3]
  const uint16_t* w;   // packed [64][7][8][4]
  uint16_t* y;         // [N][Ho][Wo][64]
  float* stats;        // [gridDim.x][2][64] or null
  int N, H, W, Ho, Wo;
  int rows;            // N * Ho output rows (tiles)
};

// input image for one tile: [7][WP][4] bf16, WP = 2*Wo + 6 (>= W + 6)
__device__ __forceinline__ int img_elem(int kh, int px, int c, int WP) { return (kh * WP + px) * 4 + c; }

template <bool STATS>
__global__ __launch_bounds__(kThreads, 2) void stem_fwd_kernel(const StemArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  const int WP = 2 * a.Wo + 6;
  const int IMG = kKh * WP * 4;                 // bf16 elements per input image
  uint16_t* img0 = smem;
  uint16_t* img1 = smem + IMG;
  char* otile = reinterpret_cast<char*>(smem + 2 * IMG);  // [128 pixels][64] bf16, 16-B chunks swizzled
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, l32 = lane & 31, hh = lane >> 5;
  const int row_elems = a.W * 3;                // one input row in global memory (contiguous)
  const int chunks = (row_elems + 7) / 8;       // 16-B chunks per input row
  const int PER = (kKh * chunks + kThreads - 1) / kThreads;

  // zero both images once: padding pixels and the 4th channel are never written again
  for (int i = tid; i < IMG; i += kThreads) {
    img0[i] = 0;
    img1[i] = 0;
  }

  // weights -> registers: A fragment (row co = 32*nb + l32, k = 16*s + 8*hh .. +7)
  const int nb = wave & 1, pb0 = 64 * (wave >> 1);  // this wave's channel block / first pixel
  bf16x8 wf[kSteps];
#pragma unroll
  for (int s = 0; s < kSteps; ++s)
    wf[s] = *reinterpret_cast<const bf16x8*>(a.w + (32 * nb + l32) * kKp + 16 * s + 8 * hh);

  float ssum[8], ssq[8];
  if constexpr (STATS) {
#pragma unroll
    for (int e = 0; e < 8; ++e) ssum[e] = ssq[e] = 0.f;
  }

  // staging: up to 4 chunks per thread (7 rows x ceil(3W/8) chunks; W <= 340)
  u32x4 stg[4];
  auto load = [&](int row) {
    const int n = row / a.Ho, oh = row % a.Ho;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + kThreads * i;
      stg[i] = u32x4{0u, 0u, 0u, 0u};
      if (i < PER && c < kKh * chunks) {
        const int kh = c / chunks, ch = c % chunks;
        const int ih = 2 * oh - 3 + kh;
        if (ih >= 0 && ih < a.H) {  // rows are 16-B aligned (W % 8 == 0); out-of-image rows stay zero
          stg[i] = *reinterpret_cast<const u32x4*>(a.x + ((int64_t)n * a.H + ih) * row_elems + ch * 8);
        }
      }
    }
  };
  auto store = [&](uint16_t* img) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + kThreads * i;
      if (i < PER && c < kKh * chunks) {
        const int kh = c / chunks, ch = c % chunks;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int e = ch * 8 + k;
          const unsigned v = (stg[i][k >> 1] >> (16 * (k & 1))) & 0xffffu;
          img[img_elem(kh, e / 3 + 3, e % 3, WP)] = (uint16_t)v;
        }
      }
    }
  };

  int row = blockIdx.x;
  if (row >= a.rows) return;
  __syncthreads();  // images zeroed
  load(row);
  store(img0);
  __syncthreads();
  int cur = 0;
  for (;;) {
    const int nrow = row + gridDim.x;
    const bool more = nrow < a.rows;
    if (more) load(nrow);
    const uint16_t* img = cur ? img1 : img0;
    f32x16 acc[2] = {zero16(), zero16()};
    if (pb0 < a.Wo) {
#pragma unroll
      for (int kh = 0; kh < kKh; ++kh)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            // kw = 4*s2 + 2*hh, +1: input pixels 2*pix + kw - 3 (+3 padding offset), 4 channels each
            const int pix = min(pb0 + 32 * q + l32, a.Wo - 1);
            const int px = 2 * pix + 4 * s2 + 2 * hh;
            const bf16x8 bx = *reinterpret_cast<const bf16x8*>(img + img_elem(kh, px, 0, WP));
            acc[q] = mfma(wf[2 * kh + s2], bx, acc[q]);
          }
        }
    }
    // epilogue: D[co][pixel] -> otile[pixel][co] (chunk c of pixel r at r*128 + 16*(c ^ ((r >> 1) & 7)))
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int pix = pb0 + 32 * q + l32;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int co = 32 * nb + 8 * g + 4 * hh;
        const unsigned lo = (unsigned)f32_to_bf16(acc[q][4 * g]) | ((unsigned)f32_to_bf16(acc[q][4 * g + 1]) << 16);
        const unsigned hi = (unsigned)f32_to_bf16(acc[q][4 * g + 2]) | ((unsigned)f32_to_bf16(acc[q][4 * g + 3]) << 16);
        *reinterpret_cast<u32x2*>(otile + pix * 128 + 16 * ((co >> 3) ^ ((pix >> 1) & 7)) + 8 * ((co >> 2) & 1)) =
            u32x2{lo, hi};
      }
    }
    __syncthreads();  // otile complete; every wave done reading img[cur]
    {
      uint16_t* yrow = a.y + (int64_t)row * a.Wo * kCo;
      const int c = tid & 7;
      for (int r = tid >> 3; r < a.Wo; r += kThreads / 8) {
        const u32x4 v = *reinterpret_cast<const u32x4*>(otile + r * 128 + 16 * (c ^ ((r >> 1) & 7)));
        *reinterpret_cast<u32x4*>(yrow + r * kCo + 8 * c) = v;
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
    if (!more) break;
    store(cur ? img0 : img1);
    __syncthreads();  // next image ready; otile consumed
    cur ^= 1;
    row = nrow;
  }

  if constexpr (STATS) {
    __syncthreads();
    float* red = reinterpret_cast<float*>(otile);  // [32 row groups][2][64]
    const int c = tid & 7, rg = tid >> 3;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[(rg * 2) * kCo + 8 * c + e] = ssum[e];
      red[(rg * 2 + 1) * kCo + 8 * c + e] = ssq[e];
    }
    __syncthreads();
    if (tid < 2 * kCo) {
      const int which = tid / kCo, co = tid % kCo;
      float v = 0.f;
      for (int g = 0; g < kThreads / 8; ++g) v += red[(g * 2 + which) * kCo + co];
      a.stats[((int64_t)blockIdx.x * 2 + which) * kCo + co] = v;
    }
  }
}

inline int stem_grid(int rows) { return rows < 2 * kNumCU ? rows : 2 * kNumCU; }

// ---------------------------------------------------------------------------------------------
// Weight gradient: dW[co][c][kh][kw] = sum_{n,oh,ow} dy[n][oh][ow][co] * xpad[n][2oh+kh][2ow+kw][c].
//
// GEMM D[co][k] (k = (kh, kw, c), kw and c padded to 8 x 4) reducing over output pixels.  Both
// operands are pixel-major in memory, so both are read "down the rows" with gfx950's transposing
// LDS read (ds_read_b64_tr_b16, mf::lds_col):
//  * A = dy: the output row's [Wo][64] tile is staged as-is (swizzled 128-B rows); lane half h
//    reads channels 32b + (l & 31) of pixels 16t + 8h .. +7;
//  * B = im2col patches, never materialised: for one kh, patch[ow][4 kw + c] = img[(2 ow + kw) * 4
//    + c] where img is the padded [pixel][4] input row, i.e. patch rows overlap with a 16-byte
//    stride and every 4-column group starts 8-byte aligned -- exactly what the transposing read
//    needs, so the B fragment is two ds_read_b64_tr_b16 straight from the staged image row.
// A workgroup walks a contiguous range of output rows.  Consecutive rows of one image share 5 of
// their 7 input rows, so input rows live in an 8-slot ring (slot = ih & 7, slot 8 = zeros for
// rows outside the image) and only the 2 new rows are staged per output row.  Global loads for
// row r + 1 are issued before row r's MFMAs.  Wave w owns channel block b = w & 1 and the kh
// tiles w >> 1, +2, +4, +6; accumulators stay in registers for the whole range and are written
// once to a per-workgroup partial, summed by stem_wgrad_reduce (deterministic, no atomics).
constexpr int kWMaxTiles = 4;

struct StemWArgs {
  const uint16_t* x;   // [N][H][W][3]
  const uint16_t* dy;  // [N][Ho][Wo][64]
  float* ws;           // [gridDim.x][64][3][7][7]
  int N, H, W, Ho, Wo;
  int rows, per;       // output rows, rows per workgroup
};

// B fragment: element j of lane half h = patch[ow0 + 8h + j][4 kw + c], kw = 4 (g & 1) + (i & 3)
__device__ __forceinline__ bf16x8 lds_patch(const uint16_t* img_row, int ow0, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int kw = 4 * (g & 1) + (i & 3);
  const int ow = ow0 + 8 * (g >> 1) + (i >> 2);
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const uint16_t* p = img_row + (2 * ow + kw) * 4;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p);
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p + 8 * 4));  // ow + 4
  const s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, r);
}

__global__ __launch_bounds__(kThreads, 2) void stem_wgrad_kernel(const StemWArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  const int WOP = (a.Wo + 15) & ~15;          // pixels padded to the MFMA reduction step
  const int ROW = (2 * WOP + 6) * 4;          // bf16 per staged input row (>= the padded image row)
  uint16_t* ring = smem;                      // [9][ROW]; slot 8 stays zero
  uint16_t* dyt = smem + 9 * ROW;             // [WOP][64], swz<64> rows
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, hh = lane >> 5, l32 = lane & 31;
  const int row_elems = a.W * 3, chunks = row_elems / 8;
  const int dchunks = a.Wo * 8;               // 16-B chunks of one dy row

  const int r0 = blockIdx.x * a.per;
  const int r1 = min(r0 + a.per, a.rows);
  if (r0 >= r1) return;
  for (int i = tid; i < 9 * ROW + WOP * kCo; i += kThreads) smem[i] = 0;

  const int b = wave & 1, kh0 = wave >> 1;    // channel block, first kh tile (then +2, +4, +6)
  f32x16 acc[kWMaxTiles];
#pragma unroll
  for (int q = 0; q < kWMaxTiles; ++q) acc[q] = zero16();

  u32x4 istg[4], dstg[4];
  int s_oh = 0, s_klo = 0;                    // row being staged: output row and first new kh
  auto load = [&](int r) {
    const int n = r / a.Ho, oh = r % a.Ho;
    const bool fresh = (r == r0) || (oh == 0);
    s_oh = oh;
    s_klo = fresh ? 0 : 5;
    const int total = (kKh - s_klo) * chunks;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + kThreads * i;
      istg[i] = u32x4{0u, 0u, 0u, 0u};
      if (c < total) {
        const int ih = 2 * oh - 3 + s_klo + c / chunks;
        if (ih >= 0 && ih < a.H)
          istg[i] = *reinterpret_cast<const u32x4*>(a.x + ((int64_t)n * a.H + ih) * row_elems + (c % chunks) * 8);
      }
      const int d = tid + kThreads * i;
      if (d < dchunks) dstg[i] = *reinterpret_cast<const u32x4*>(a.dy + ((int64_t)r * a.Wo) * kCo + d * 8);
    }
  };
  auto store = [&]() {
    const int total = (kKh - s_klo) * chunks;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + kThreads * i;
      if (c < total) {
        const int ih = 2 * s_oh - 3 + s_klo + c / chunks, ch = c % chunks;
        if (ih >= 0 && ih < a.H) {
          uint16_t* img = ring + (ih & 7) * ROW;
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const int e = ch * 8 + k;
            img[(e / 3 + 3) * 4 + e % 3] = (uint16_t)((istg[i][k >> 1] >> (16 * (k & 1))) & 0xffffu);
          }
        }
      }
      const int d = tid + kThreads * i;
      if (d < dchunks)
        *reinterpret_cast<u32x4*>(reinterpret_cast<char*>(dyt) + swz<64>(d >> 3, d & 7)) = dstg[i];
    }
  };

  __syncthreads();  // zeroed
  load(r0);
  store();
  __syncthreads();
  for (int r = r0;;) {
    const int oh = r % a.Ho;
    const bool more = r + 1 < r1;
    if (more) load(r + 1);
    const uint16_t* rows_kh[kWMaxTiles];
#pragma unroll
    for (int q = 0; q < kWMaxTiles; ++q) {
      const int ih = 2 * oh - 3 + kh0 + 2 * q;
      rows_kh[q] = ring + ((ih >= 0 && ih < a.H) ? (ih & 7) : 8) * ROW;
    }
    for (int t = 0; t < WOP; t += 16) {
      const bf16x8 af = lds_col<64>(dyt, t, 32 * b, lane);
#pragma unroll
      for (int q = 0; q < kWMaxTiles; ++q)
        if (kh0 + 2 * q < kKh) acc[q] = mfma(af, lds_patch(rows_kh[q], t, lane), acc[q]);
    }
    if (!more) break;
    __syncthreads();  // every wave done with dyt and the ring slots being replaced
    store();
    __syncthreads();
    ++r;
  }

  // D[co][4 kw + c] of tile q -> ws[block][co][c][kh][kw]
  const int kw = l32 >> 2, c = l32 & 3;
  if (kw < 7 && c < 3) {
    float* out = a.ws + (int64_t)blockIdx.x * kCo * 147;
#pragma unroll
    for (int q = 0; q < kWMaxTiles; ++q) {
      const int kh = kh0 + 2 * q;
      if (kh < kKh) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int co = 32 * b + acc_row(e, hh);
          out[co * 147 + c * 49 + kh * 7 + kw] = acc[q][e];
        }
      }
    }
  }
}

// dw[i] = sum_g ws[g][i], i < 64 * 147: a block sums 32 columns, its 8 waves-worth of lane groups
// each a strided eighth of the partials (8 independent loads in flight per lane), then LDS combine
__global__ __launch_bounds__(256) void stem_wgrad_reduce(const float* __restrict__ ws, float* __restrict__ dw, int parts) {
  __shared__ float red[8][32];
  const int col = threadIdx.x & 31, grp = threadIdx.x >> 5;
  const int i = blockIdx.x * 32 + col;
  const int64_t stride = (int64_t)kCo * 147;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (i < kCo * 147) {
    int g = grp;
    for (; g + 56 < parts; g += 64) {
#pragma unroll
      for (int u = 0; u < 8; ++u) s[u] += ws[(int64_t)(g + 8 * u) * stride + i];
    }
    for (; g < parts; g += 8) s[0] += ws[(int64_t)g * stride + i];
  }
  red[grp][col] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  __syncthreads();
  if (grp == 0 && i < kCo * 147) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) t += red[k][col];
    dw[i] = t;
  }
}

inline int wgrad_grid(int rows) { return rows < 2 * kNumCU ? rows : 2 * kNumCU; }

}  // namespace stem
}  // namespace madnn

using namespace madnn::stem;

extern "C" {

int madnn_stem_supported(int H, int W) {
  const int Wo = (W + 6 - 7) / 2 + 1;
  // rows of 3W bf16 must be whole 16-B chunks, 7 rows of chunks must fit 4 per thread
  return (H >= 7 && W >= 8 && W % 8 == 0 && Wo <= kMaxWo && kKh * (W * 3 / 8) <= 4 * kThreads) ? 1 : 0;
}

int madnn_stem_stat_rows(int N, int H, int W) {
  const int Ho = (H + 6 - 7) / 2 + 1;
  return stem_grid(N * Ho);
}

// x [N][H][W][3] bf16, wp packed [64][7][8][4] bf16 -> y [N][Ho][Wo][64]; stats [grid][2][64] or null
hipError_t madnn_stem_fwd(const void* x, const void* wp, void* y, float* stats, int N, int H, int W, hipStream_t s) {
  if (!madnn_stem_supported(H, W)) return hipErrorInvalidValue;
  StemArgs a{};
  a.x = static_cast<const uint16_t*>(x);
  a.w = static_cast<const uint16_t*>(wp);
  a.y = static_cast<uint16_t*>(y);
  a.stats = stats;
  a.N = N;
  a.H = H;
  a.W = W;
  a.Ho = (H + 6 - 7) / 2 + 1;
  a.Wo = (W + 6 - 7) / 2 + 1;
  a.rows = N * a.Ho;
  if (a.rows <= 0) return hipSuccess;
  const int WP = 2 * a.Wo + 6;
  const size_t lds = (size_t)2 * kKh * WP * 4 * sizeof(uint16_t) + (size_t)kMaxWo * kCo * sizeof(uint16_t);
  const int grid = stem_grid(a.rows);
  if (stats) {
    hipLaunchKernelGGL(stem_fwd_kernel<true>, dim3(grid), dim3(kThreads), lds, s, a);
  } else {
    hipLaunchKernelGGL(stem_fwd_kernel<false>, dim3(grid), dim3(kThreads), lds, s, a);
  }
  return hipGetLastError();
}

// fp32 workspace floats the weight gradient needs (per-workgroup partials)
int64_t madnn_stem_wgrad_ws(int N, int H, int W) {
  const int Ho = (H + 6 - 7) / 2 + 1;
  return (int64_t)wgrad_grid(N * Ho) * kCo * 147;
}

// x [N][H][W][3], dy [N][Ho][Wo][64] bf16 -> dw [64][3][7][7] fp32 (ws: madnn_stem_wgrad_ws floats)
hipError_t madnn_stem_wgrad(const void* x, const void* dy, float* ws, float* dw, int N, int H, int W,
                            hipStream_t s) {
  if (!madnn_stem_supported(H, W)) return hipErrorInvalidValue;
  StemWArgs a{};
  a.x = static_cast<const uint16_t*>(x);
  a.dy = static_cast<const uint16_t*>(dy);
  a.ws = ws;
  a.N = N;
  a.H = H;
  a.W = W;
  a.Ho = (H + 6 - 7) / 2 + 1;
  a.Wo = (W + 6 - 7) / 2 + 1;
  a.rows = N * a.Ho;
  if (a.rows <= 0) return hipMemsetAsync(dw, 0, sizeof(float) * kCo * 147, s);
  a.per = (a.rows + wgrad_grid(a.rows) - 1) / wgrad_grid(a.rows);
  const int grid = (a.rows + a.per - 1) / a.per;  // every workgroup owns >= 1 row (writes its partial)
  const int WOP = (a.Wo + 15) & ~15;
  const size_t lds = (size_t)(9 * (2 * WOP + 6) * 4 + WOP * kCo) * sizeof(uint16_t);
  hipLaunchKernelGGL(stem_wgrad_kernel, dim3(grid), dim3(kThreads), lds, s, a);
  MADNN_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(stem_wgrad_reduce, dim3((kCo * 147 + 31) / 32), dim3(256), 0, s, ws, dw, grid);
  return hipGetLastError();
}

}  // extern "C"
