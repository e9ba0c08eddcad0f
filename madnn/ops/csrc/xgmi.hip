// K5 — one-shot all-reduce over P2P-mapped peer buffers (xGMI inside one MI355X node), for the
// small, latency-bound messages of tensor parallelism (the reference's MP layers
// all-reduce [B, out] activations every layer, nodemodule.lua:52,103).
//
// Why: a ring all-reduce of a few hundred KB is latency-bound (2(W-1) dependent hops, each a
// kernel-side handshake).  With every peer's buffer mapped into this process (IPC handles,
// xGMI point-to-point: every MI355X of the node is one hop away), one kernel can read all W
// inputs directly and sum them -- one round of flags, W reads per element.
//
// Protocol (per call, epoch e = 1, 2, ... kept by the host, identical on every rank):
//   1. block b copies its chunk of the input into this rank's staging buffer, half (e & 1);
//   2. block b publishes "chunk b of epoch e is staged" by storing e into flag[rank][b] of EVERY
//      peer's flag array (system-scope release after a system-scope fence);
//   3. block b waits until its own flag[r][b] >= e for every rank r (system-scope acquire),
//      bounded: after `spin_limit` polls it records a timeout in *err and gives up on the
//      wait, so a missing peer can never leave the kernel running.  *err lives in pinned host
//      memory: the host reads it without synchronising (madnn_oneshot_error), so the Python
//      side raises at the next call / optimizer step instead of training on a partial sum;
//   4. block b sums chunk b of all W staging buffers (fp32 accumulation) into the output.
// Reuse safety: the staging half written at epoch e+1 was last read at epoch e-1; a rank only
// starts epoch e+1 after its epoch-e kernel saw every peer's epoch-e flag for that chunk, which
// each peer set only after its own epoch-(e-1) kernel had finished -- so two halves suffice.
// Flags live in uncached device memory (hipDeviceMallocUncached): stores from peers land in
// memory that no L2 keeps a stale copy of.  Staging buffers are ordinary device memory; the
// writer's system-scope release and the reader's system-scope acquire order them.
// Per-block flags mean no grid-wide barrier: chunk b only ever meets chunk b of the peers.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <map>
#include <mutex>

namespace madnn {
namespace xgmi {

constexpr int kMaxPeers = 8;
constexpr int kThreads = 256;
constexpr int kMaxBlocks = 64;  // flag slots per rank; also keeps W concurrent kernels co-resident

struct Peers {
  void* stage[kMaxPeers];     // each rank's staging buffer (2 halves of cap bytes)
  unsigned* flag[kMaxPeers];  // each rank's flag array [kMaxPeers][kMaxBlocks]
};

struct Args {
  const void* in;
  void* out;
  int* err;
  int64_t n;      // elements
  int64_t chunk;  // elements per block (multiple of 8)
  int64_t half;   // elements per staging half
  int rank, world, dtype;  // dtype 0: fp32, 1: bf16
  unsigned epoch;
  int spin_limit;
  Peers peers;
};

__device__ __forceinline__ float bf16f(unsigned short h) { return __uint_as_float((unsigned)h << 16); }
__device__ __forceinline__ unsigned short f2bf16(float f) {  // round to nearest even; NaN stays NaN
  const unsigned u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (unsigned short)((u >> 16) | 0x40u);
  return (unsigned short)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

__global__ __launch_bounds__(kThreads) void oneshot_kernel(const Args a) {
  const int b = blockIdx.x;
  const int64_t lo = (int64_t)b * a.chunk;
  const int64_t hi = lo + a.chunk < a.n ? lo + a.chunk : a.n;
  const int esz = a.dtype == 0 ? 4 : 2;
  const int64_t base = (int64_t)(a.epoch & 1u) * a.half;  // staging half of this epoch
  // 1. stage this rank's chunk (16-B accesses; chunk boundaries are multiples of 8 elements)
  {
    const char* src = static_cast<const char*>(a.in) + lo * esz;
    char* dst = static_cast<char*>(a.peers.stage[a.rank]) + (base + lo) * esz;
    const int64_t bytes = (hi - lo) * esz;
    for (int64_t o = (int64_t)threadIdx.x * 16; o < bytes; o += kThreads * 16) {
      if (o + 16 <= bytes) {
        *reinterpret_cast<uint4*>(dst + o) = *reinterpret_cast<const uint4*>(src + o);
      } else {
        for (int64_t k = o; k < bytes; ++k) dst[k] = src[k];
      }
    }
  }
  // 2. publish: every lane releases its own staged stores at system scope, the barrier orders
  //    all lanes' releases before the flag stores
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  __syncthreads();
  if (threadIdx.x < a.world) {
    __hip_atomic_store(a.peers.flag[threadIdx.x] + a.rank * kMaxBlocks + b, a.epoch, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // 3. wait for every rank's chunk b (bounded)
  __shared__ int timed_out;
  if (threadIdx.x == 0) timed_out = 0;
  __syncthreads();
  if (threadIdx.x < a.world) {
    unsigned* f = a.peers.flag[a.rank] + threadIdx.x * kMaxBlocks + b;
    int polls = 0;
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < a.epoch) {
      if (++polls > a.spin_limit) {
        timed_out = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  if (timed_out) {
    if (threadIdx.x == 0) __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  // 4. sum chunk b over all ranks' staging buffers, 8 elements per lane, fp32 accumulation
  for (int64_t i = lo + (int64_t)threadIdx.x * 8; i < hi; i += kThreads * 8) {
    const int cnt = hi - i >= 8 ? 8 : (int)(hi - i);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < a.world; ++r) {
      const char* s = static_cast<const char*>(a.peers.stage[r]) + (base + i) * esz;
      if (a.dtype == 0) {
        if (cnt == 8) {
          const float4 v0 = reinterpret_cast<const float4*>(s)[0], v1 = reinterpret_cast<const float4*>(s)[1];
          acc[0] += v0.x; acc[1] += v0.y; acc[2] += v0.z; acc[3] += v0.w;
          acc[4] += v1.x; acc[5] += v1.y; acc[6] += v1.z; acc[7] += v1.w;
        } else {
          for (int k = 0; k < cnt; ++k) acc[k] += reinterpret_cast<const float*>(s)[k];
        }
      } else {
        if (cnt == 8) {
          const uint4 v = *reinterpret_cast<const uint4*>(s);
          const unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            acc[2 * k] += bf16f((unsigned short)(w[k] & 0xffffu));
            acc[2 * k + 1] += bf16f((unsigned short)(w[k] >> 16));
          }
        } else {
          for (int k = 0; k < cnt; ++k) acc[k] += bf16f(reinterpret_cast<const unsigned short*>(s)[k]);
        }
      }
    }
    char* d = static_cast<char*>(a.out) + i * esz;
    if (a.dtype == 0) {
      for (int k = 0; k < cnt; ++k) reinterpret_cast<float*>(d)[k] = acc[k];
    } else if (cnt == 8) {
      uint4 v;
      v.x = f2bf16(acc[0]) | ((unsigned)f2bf16(acc[1]) << 16);
      v.y = f2bf16(acc[2]) | ((unsigned)f2bf16(acc[3]) << 16);
      v.z = f2bf16(acc[4]) | ((unsigned)f2bf16(acc[5]) << 16);
      v.w = f2bf16(acc[6]) | ((unsigned)f2bf16(acc[7]) << 16);
      *reinterpret_cast<uint4*>(d) = v;
    } else {
      for (int k = 0; k < cnt; ++k) reinterpret_cast<unsigned short*>(d)[k] = f2bf16(acc[k]);
    }
  }
}

// One communicator: this rank's own buffers plus the peers' mapped ones.
struct Ctx {
  int rank = 0, world = 1, device = 0;
  int64_t cap = 0;  // bytes per staging half
  void* stage = nullptr;
  unsigned* flag = nullptr;
  int* err = nullptr;      // pinned host word (host view)
  int* err_dev = nullptr;  // its device-side address
  Peers peers{};
  bool opened = false;
  unsigned epoch = 0;
};

std::mutex& mu() {
  static std::mutex m;
  return m;
}
std::map<int, Ctx>& ctxs() {
  static std::map<int, Ctx> c;
  return c;
}

}  // namespace xgmi
}  // namespace madnn

using namespace madnn::xgmi;

extern "C" {

int madnn_oneshot_max_peers() { return kMaxPeers; }
int madnn_oneshot_handle_bytes() { return (int)sizeof(hipIpcMemHandle_t); }

// Allocate this rank's staging buffer (2 x cap bytes) and uncached flag array, and return their
// IPC handles (2 x handle_bytes into `handles`).  Returns the context id (> 0) or -hipError.
int madnn_oneshot_create(int64_t cap, int world, int rank, int device, unsigned char* handles) {
  if (world < 1 || world > kMaxPeers || rank < 0 || rank >= world || cap <= 0) return -(int)hipErrorInvalidValue;
  Ctx c;
  c.rank = rank;
  c.world = world;
  c.device = device;
  c.cap = (cap + 255) / 256 * 256;
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipMalloc(&c.stage, 2 * c.cap);
  if (e == hipSuccess)
    e = hipExtMallocWithFlags(reinterpret_cast<void**>(&c.flag), kMaxPeers * kMaxBlocks * sizeof(unsigned),
                              hipDeviceMallocUncached);
  if (e == hipSuccess) e = hipMemset(c.flag, 0, kMaxPeers * kMaxBlocks * sizeof(unsigned));
  if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void**>(&c.err), sizeof(int), hipHostMallocMapped);
  if (e == hipSuccess) {
    *reinterpret_cast<volatile int*>(c.err) = 0;
    e = hipHostGetDevicePointer(reinterpret_cast<void**>(&c.err_dev), c.err, 0);
  }
  hipIpcMemHandle_t hs, hf;
  if (e == hipSuccess) e = hipIpcGetMemHandle(&hs, c.stage);
  if (e == hipSuccess) e = hipIpcGetMemHandle(&hf, c.flag);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    if (c.stage) (void)hipFree(c.stage);
    if (c.flag) (void)hipFree(c.flag);
    if (c.err) (void)hipHostFree(c.err);
    return -(int)e;
  }
  std::memcpy(handles, &hs, sizeof(hs));
  std::memcpy(handles + sizeof(hs), &hf, sizeof(hf));
  std::lock_guard<std::mutex> g(mu());
  const int id = ctxs().empty() ? 1 : ctxs().rbegin()->first + 1;
  ctxs()[id] = c;
  return id;
}

// Map every peer's buffers: all_handles = world x (2 x handle_bytes), rank-major.
int madnn_oneshot_open(int id, const unsigned char* all_handles) {
  std::lock_guard<std::mutex> g(mu());
  auto it = ctxs().find(id);
  if (it == ctxs().end()) return (int)hipErrorInvalidValue;
  Ctx& c = it->second;
  const size_t hb = sizeof(hipIpcMemHandle_t);
  hipError_t e = hipSetDevice(c.device);
  for (int r = 0; r < c.world && e == hipSuccess; ++r) {
    if (r == c.rank) {
      c.peers.stage[r] = c.stage;
      c.peers.flag[r] = c.flag;
      continue;
    }
    hipIpcMemHandle_t hs, hf;
    std::memcpy(&hs, all_handles + r * 2 * hb, hb);
    std::memcpy(&hf, all_handles + r * 2 * hb + hb, hb);
    e = hipIpcOpenMemHandle(&c.peers.stage[r], hs, hipIpcMemLazyEnablePeerAccess);
    if (e == hipSuccess) {
      void* f = nullptr;
      e = hipIpcOpenMemHandle(&f, hf, hipIpcMemLazyEnablePeerAccess);
      c.peers.flag[r] = static_cast<unsigned*>(f);
    }
  }
  c.opened = e == hipSuccess;
  return (int)e;
}

// out = sum over ranks of in (n elements, dtype 0 fp32 / 1 bf16; in/out may alias).  Every rank
// must call with the same n and dtype, in the same order.  Asynchronous on `stream`; a peer that
// never arrives sets the context's error word (madnn_oneshot_error) instead of hanging the GPU.
int madnn_oneshot_allreduce(int id, const void* in, void* out, int64_t n, int dtype, int spin_limit,
                            hipStream_t stream) {
  Args a{};
  {
    std::lock_guard<std::mutex> g(mu());
    auto it = ctxs().find(id);
    if (it == ctxs().end() || !it->second.opened) return (int)hipErrorInvalidValue;
    Ctx& c = it->second;
    const int esz = dtype == 0 ? 4 : 2;
    if ((dtype != 0 && dtype != 1) || n < 0 || n * esz > c.cap) return (int)hipErrorInvalidValue;
    if (n == 0) return (int)hipSuccess;
    a.peers = c.peers;
    a.rank = c.rank;
    a.world = c.world;
    a.err = c.err_dev;
    a.half = c.cap / esz;
    a.epoch = ++c.epoch;
  }
  a.in = in;
  a.out = out;
  a.n = n;
  a.dtype = dtype;
  a.spin_limit = spin_limit > 0 ? spin_limit : 1 << 21;
  // blocks: >= 16 KB per block, at most kMaxBlocks; chunk a multiple of 8 elements
  int64_t blocks = (n * (dtype == 0 ? 4 : 2) + 16383) / 16384;
  blocks = blocks < 1 ? 1 : (blocks > kMaxBlocks ? kMaxBlocks : blocks);
  a.chunk = ((n + blocks - 1) / blocks + 7) / 8 * 8;
  blocks = (n + a.chunk - 1) / a.chunk;
  hipLaunchKernelGGL(oneshot_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, stream, a);
  return (int)hipGetLastError();
}

// error word of the context (1 = a wait timed out).  flags bit 0: clear it after reading;
// bit 1: synchronise the device first (otherwise the word reflects the kernels that have
// finished so far -- a plain host read of pinned memory, no stall)
int madnn_oneshot_error(int id, int flags) {
  std::lock_guard<std::mutex> g(mu());
  auto it = ctxs().find(id);
  if (it == ctxs().end()) return -1;
  if ((flags & 2) && hipDeviceSynchronize() != hipSuccess) return -1;
  volatile int* w = it->second.err;
  const int v = *w;
  if ((flags & 1) && v) *w = 0;
  return v;
}

int madnn_oneshot_destroy(int id) {
  std::lock_guard<std::mutex> g(mu());
  auto it = ctxs().find(id);
  if (it == ctxs().end()) return (int)hipErrorInvalidValue;
  Ctx& c = it->second;
  (void)hipSetDevice(c.device);
  (void)hipDeviceSynchronize();
  for (int r = 0; r < c.world; ++r) {
    if (r == c.rank || !c.opened) continue;
    if (c.peers.stage[r]) (void)hipIpcCloseMemHandle(c.peers.stage[r]);
    if (c.peers.flag[r]) (void)hipIpcCloseMemHandle(c.peers.flag[r]);
  }
  (void)hipFree(c.stage);
  (void)hipFree(c.flag);
  (void)hipHostFree(c.err);
  ctxs().erase(it);
  return 0;
}

}  // extern "C"
