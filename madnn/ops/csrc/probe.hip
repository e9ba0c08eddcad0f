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
