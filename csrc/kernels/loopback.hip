// Test-only stand-in for one 2-rank RCCL link between two processes that share ONE GPU
// (parallel/loopback_comm.py, selected only by tests through ADAPT_TEST_LOOPBACK_COMM=1; never a default or
// a fallback).  The data path of the RCCL branch of a pipeline stage (parallel/stage_runtime.py, nccl
// backend) otherwise runs only when every stage owns a GPU of its own.  A message is copied into a slot of
// a ring in device memory that the sender exported by IPC handle; the hand-off is two counters in a
// page-locked host control block mapped by both processes:
//   sender stream:   wait(consumed >= seq - depth) -> copies into slot seq % depth -> signal(posted = seq)
//   receiver stream: wait(posted >= seq) -> copies out of the slot -> signal(consumed = seq)
// A wait is one wave spinning on system-scope relaxed atomic loads of host memory; it ends when the
// counter is reached, when the shared abort word turns non-zero (the stand-in's ncclCommAbort) or at its
// wall-clock bound, and reports which into a host status word, so every wave always terminates.
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace adapt {

namespace {

__global__ __launch_bounds__(64) void lb_wait_kernel(const unsigned long long* ctr, unsigned long long target,
                                                     const int* abort_word, int* status,
                                                     unsigned long long max_ticks) {
  const unsigned long long t0 = wall_clock64();
  int why = 2;                                       // 1: reached, 2: timed out, 3: aborted
  while (true) {
    if (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= target) {
      why = 1;
      break;
    }
    if (__hip_atomic_load(abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) {
      why = 3;
      break;
    }
    if (wall_clock64() - t0 > max_ticks) break;
    __builtin_amdgcn_s_sleep(4);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");      // system scope: the copies behind this kernel read fresh
  if (threadIdx.x == 0 && why != 1) __hip_atomic_store(status, why, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(64) void lb_signal_kernel(unsigned long long* ctr, unsigned long long value) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");      // system scope, behind the stream's earlier copies
  if (threadIdx.x == 0) __hip_atomic_store(ctr, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace

hipError_t lb_wait(const unsigned long long* ctr, unsigned long long target, const int* abort_word, int* status,
                   double timeout_ms, hipStream_t s) {
  const unsigned long long ticks = static_cast<unsigned long long>(timeout_ms * 1e5);   // 100 MHz
  hipLaunchKernelGGL(lb_wait_kernel, dim3(1), dim3(64), 0, s, ctr, target, abort_word, status, ticks);
  return hipGetLastError();
}

hipError_t lb_signal(unsigned long long* ctr, unsigned long long value, hipStream_t s) {
  hipLaunchKernelGGL(lb_signal_kernel, dim3(1), dim3(64), 0, s, ctr, value);
  return hipGetLastError();
}

}  // namespace adapt
