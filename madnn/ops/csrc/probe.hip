// Hardware-queue aliasing probe (diagnostic kernels, not on any training path).
//
// HIP multiplexes every stream of a process onto a small pool of hardware (AQL)
// queues: GPU_MAX_HW_QUEUES, 4 by default.  Dispatches that land on one queue
// may be serialised in submission order even when they came from different
// streams.  For a pipeline rank that matters: a receive kernel that spins until
// its peer's data arrives can, if it shares a queue with this rank's compute
// stream, hold back the very kernel that produces what the peer is waiting for.
//
// The probe measures it directly.  hwq_wait runs one lane that polls a device
// flag until it holds `expect` or until `timeout_us` has passed on the 100 MHz
// constant clock; hwq_set stores the flag.  Launch hwq_wait on stream A, then
// hwq_set on stream B: if the two streams share a serialised queue the setter
// cannot start before the waiter gives up, and the waiter reports a timeout.
// The wait is always bounded, so a blocked pair costs timeout_us and nothing
// else (no unbounded spin can outlive the process).
#include "common.h"

namespace {

__global__ void hwq_wait_kernel(const int* __restrict__ flag, int expect, long long timeout_ticks,
                                int* __restrict__ out) {
  if (threadIdx.x != 0) return;
  const long long t0 = wall_clock64();
  long long now = t0;
  int ok = 0;
  while (true) {
    int v = __hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    now = wall_clock64();
    if (v == expect) {
      ok = 1;
      break;
    }
    if (now - t0 > timeout_ticks) break;
    __builtin_amdgcn_s_sleep(4);
  }
  // vector stores: [0] = 1 if the flag arrived, [1] = ticks waited (100 MHz)
  out[0] = ok;
  out[1] = static_cast<int>(now - t0);
}

__global__ void hwq_set_kernel(int* __restrict__ flag, int val) {
  if (threadIdx.x == 0) __hip_atomic_store(flag, val, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace

extern "C" hipError_t madnn_hwq_wait(const int* flag, int expect, int64_t timeout_us, int* out, hipStream_t s) {
  // wall_clock64 ticks at 100 MHz on gfx9: 100 ticks per microsecond
  hipLaunchKernelGGL(hwq_wait_kernel, dim3(1), dim3(madnn::kWave), 0, s, flag, expect,
                     static_cast<long long>(timeout_us) * 100, out);
  return hipGetLastError();
}

extern "C" hipError_t madnn_hwq_set(int* flag, int val, hipStream_t s) {
  hipLaunchKernelGGL(hwq_set_kernel, dim3(1), dim3(madnn::kWave), 0, s, flag, val);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Pipeline replay on the hardware queues: a "batch" of point-to-point messages with RCCL's
// rendezvous semantics, one wave per message.  send: publish flag a[msg] = epoch, then wait
// until the receiver acknowledges (b[msg] == epoch); recv: wait for a[msg] == epoch, then
// acknowledge.  The batch kernel finishes only when every message of it met its peer -- as an
// RCCL batch kernel does -- and every wait is bounded (timeout_us), so a program that would
// deadlock shows up as timed-out messages instead of a hung queue.  ok[op] = 1 if the op met its
// peer in time.  hwq_spin is the stand-in for a compute kernel (one wave, busy for spin_us).
namespace {

__device__ __forceinline__ bool wait_eq(const int* f, int v, long long t0, long long limit) {
  while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != v) {
    if (wall_clock64() - t0 > limit) return false;
    __builtin_amdgcn_s_sleep(2);
  }
  return true;
}

__global__ void hwq_batch_kernel(const int* __restrict__ kinds, const int* __restrict__ msgs, int nops,
                                 int* __restrict__ a, int* __restrict__ b, int epoch, long long limit,
                                 int* __restrict__ ok, const int* __restrict__ ok_index) {
  const int op = blockIdx.x;
  if (op >= nops || threadIdx.x != 0) return;
  const int m = msgs[op];
  const long long t0 = wall_clock64();
  bool good;
  if (kinds[op] == 0) {  // send
    __hip_atomic_store(&a[m], epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    good = wait_eq(&b[m], epoch, t0, limit);
  } else {               // recv
    good = wait_eq(&a[m], epoch, t0, limit);
    if (good) __hip_atomic_store(&b[m], epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
  ok[ok_index[op]] = good ? 1 : 0;
}

__global__ void hwq_spin_kernel(long long ticks) {
  if (threadIdx.x != 0) return;
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

}  // namespace

extern "C" hipError_t madnn_hwq_batch(const int* kinds, const int* msgs, int nops, int* a, int* b, int epoch,
                                      int64_t timeout_us, int* ok, const int* ok_index, hipStream_t s) {
  if (nops <= 0) return hipSuccess;
  hipLaunchKernelGGL(hwq_batch_kernel, dim3(nops), dim3(madnn::kWave), 0, s, kinds, msgs, nops, a, b, epoch,
                     static_cast<long long>(timeout_us) * 100, ok, ok_index);
  return hipGetLastError();
}

extern "C" hipError_t madnn_hwq_spin(int64_t spin_us, hipStream_t s) {
  hipLaunchKernelGGL(hwq_spin_kernel, dim3(1), dim3(madnn::kWave), 0, s, static_cast<long long>(spin_us) * 100);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Attention-backward dQ floor probe: the f32 atomic traffic a ONE-pass backward (dQ accumulated
// inside the dK / dV kernel, cdna_hip_programming.md 'Attention backward') must issue, with no
// other work.  Workgroup (bh, key block) adds one value to every dQ[bh][q][d] with q >= the block's
// first key (causal) -- one global_atomic_add_f32 (no return) per dQ element per key block, 16 B
// apart per lane quad, exactly the fused design's add pattern.  Its time is a floor for that
// design; compare it with the separate dQ kernel it would replace (bench/attn_dq_floor.py).
namespace {

__global__ __launch_bounds__(256) void dq_atomic_floor_kernel(float* __restrict__ dq, int S, int D, int kblock,
                                                              int nkb, int causal, float v) {
  const int bh = blockIdx.x / nkb, kb = blockIdx.x % nkb;
  const int q0 = causal ? kb * kblock : 0;
  float* base = dq + (int64_t)bh * S * D;
  const int64_t n = (int64_t)(S - q0) * D;
  for (int64_t e = threadIdx.x; e < n; e += 256) unsafeAtomicAdd(base + (int64_t)q0 * D + e, v);
}

}  // namespace

extern "C" hipError_t madnn_dq_atomic_floor(float* dq, int BH, int S, int D, int kblock, int causal, hipStream_t s) {
  if (BH <= 0 || S <= 0 || D <= 0 || kblock <= 0) return hipErrorInvalidValue;
  const int nkb = (S + kblock - 1) / kblock;
  hipLaunchKernelGGL(dq_atomic_floor_kernel, dim3((unsigned)(BH * nkb)), dim3(256), 0, s, dq, S, D, kblock, nkb,
                     causal, 1.0e-3f);
  return hipGetLastError();
}
