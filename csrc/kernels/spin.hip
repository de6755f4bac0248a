// Diagnostic: a one-wave kernel that occupies its stream until a host-written
// flag turns non-zero or a wall-clock bound passes (it always terminates).
//
// Used by tests/test_stream_queues_gpu.py to stand in for a pipeline stage's
// RCCL receive that is still waiting for its upstream peer: while it spins on
// a link stream, work on the compute stream must still run.  If the two
// streams shared a hardware queue (GPU_MAX_HW_QUEUES = 4 on the box, and a
// stage process owns more streams than that), every packet queued behind the
// spinner would wait for it.
//
// The flag lives in page-locked host memory (fine-grained, coherent), read
// with system-scope relaxed atomic loads; the verdict is written with an
// ordinary vector store by lane 0.  The bound uses s_memrealtime (100 MHz).
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace adapt {

__global__ __launch_bounds__(64) void spin_flag_kernel(const int* flag, int* out, unsigned long long max_ticks) {
  const unsigned long long t0 = wall_clock64();
  int seen = 0;
  while (true) {
    if (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) {
      seen = 1;
      break;
    }
    if (wall_clock64() - t0 > max_ticks) break;
    __builtin_amdgcn_s_sleep(8);
  }
  if (threadIdx.x == 0) out[0] = seen ? 1 : 2;     // 1: released by the flag, 2: timed out
}

hipError_t spin_flag(const int* flag, int* out, double timeout_ms, hipStream_t s) {
  // wall_clock64 ticks at 100 MHz on gfx9
  const unsigned long long ticks = static_cast<unsigned long long>(timeout_ms * 1e5);
  hipLaunchKernelGGL(spin_flag_kernel, dim3(1), dim3(64), 0, s, flag, out, ticks);
  return hipGetLastError();
}

}  // namespace adapt
