// Per-CU L2 -> LDS feed rate microbenchmark (gfx950).
//
// Question it answers for the conv kernels: how many bytes per clock can one
// CU pull from an L2-resident operand into LDS, by LDS-DMA (global_load_lds,
// 16 B per lane) versus register staging (global_load_dwordx4 + ds_write_b128),
// as a function of waves per block and pieces kept in flight?
//
//   hipcc --offload-arch=gfx950 -O3 -o build/feed_bench tools/feed_bench.hip && build/feed_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef __attribute__((address_space(3))) void lds_void;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

// every block streams ITERS x (NW x PIECES) KiB from a REGION-byte window
// (L2-resident: the window is the same for all blocks of an XCD)
template <int NW, int PIECES, int DEPTH>
__global__ __launch_bounds__(NW * 64, 1) void glds_feed(const char* __restrict__ src, size_t region, int iters,
                                                        unsigned* sink) {
  __shared__ __attribute__((aligned(16))) char smem[DEPTH * NW * PIECES * 1024];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  size_t off = ((size_t)blockIdx.x * 65536 + wave * PIECES * 1024) & (region - 1);
  for (int it = 0; it < iters; ++it) {
    char* dst = smem + (it % DEPTH) * NW * PIECES * 1024 + wave * PIECES * 1024;
#pragma unroll
    for (int p = 0; p < PIECES; ++p) {
      const char* s = src + ((off + p * 1024 + lane * 16) & (region - 1));
      __builtin_amdgcn_global_load_lds((const void*)s, (lds_void*)(dst + p * 1024), 16, 0, 0);
    }
    off = (off + NW * PIECES * 1024) & (region - 1);
    // keep DEPTH-1 batches in flight
    if (DEPTH == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PIECES) : "memory");
    else if (DEPTH == 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PIECES) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * PIECES) : "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) sink[blockIdx.x] = *(unsigned*)(smem + lane * 4);
}

// register staging: every loaded dword is folded into an XOR that is stored at
// the end, so no load can be dropped (the first version kept only one LDS word
// live and hipcc removed the loads: its rows were invalid).  DSW = also write the
// batch to LDS (ds_write_b128) as a conv kernel's register-staged A/B would.
template <int NW, int PIECES, bool DSW>
__global__ __launch_bounds__(NW * 64, 1) void reg_feed(const char* __restrict__ src, size_t region, int iters,
                                                       unsigned* sink) {
  __shared__ __attribute__((aligned(16))) char smem[2 * NW * PIECES * 1024];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  size_t off = ((size_t)blockIdx.x * 65536 + wave * PIECES * 1024) & (region - 1);
  u32x4 r[PIECES];
  u32x4 acc = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int p = 0; p < PIECES; ++p) r[p] = *(const u32x4*)(src + ((off + p * 1024 + lane * 16) & (region - 1)));
  for (int it = 0; it < iters; ++it) {
    off = (off + NW * PIECES * 1024) & (region - 1);
    u32x4 n[PIECES];
#pragma unroll
    for (int p = 0; p < PIECES; ++p) n[p] = *(const u32x4*)(src + ((off + p * 1024 + lane * 16) & (region - 1)));
    if (DSW) {
      char* dst = smem + (it & 1) * NW * PIECES * 1024 + wave * PIECES * 1024;
#pragma unroll
      for (int p = 0; p < PIECES; ++p) *(u32x4*)(dst + p * 1024 + lane * 16) = r[p];
    }
#pragma unroll
    for (int p = 0; p < PIECES; ++p) acc ^= r[p];
#pragma unroll
    for (int p = 0; p < PIECES; ++p) r[p] = n[p];
  }
  if (DSW) {
    __syncthreads();
    acc.x ^= *(const unsigned*)(smem + threadIdx.x * 4);
  }
  sink[blockIdx.x * NW * 64 + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

template <typename F>
static float time_it(F launch, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  launch();
  hipDeviceSynchronize();
  hipEventRecord(a);
  for (int i = 0; i < reps; ++i) launch();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

int main() {
  const size_t big = 256ull << 20;
  char* src;
  unsigned* sink;
  CHECK(hipMalloc(&src, big));
  CHECK(hipMemset(src, 1, big));
  CHECK(hipMalloc(&sink, 256 * 1024 * 4));
  const int blocks = 256, iters = 400;
  printf("%-34s %8s %10s %12s\n", "variant", "region", "us", "B/clk/CU@2.1");
  for (size_t region : {(size_t)1 << 20, (size_t)16 << 20, big}) {
#define RUN(NAME, KERN, NW, PIECES)                                                                          \
  {                                                                                                          \
    float ms = time_it([&] { hipLaunchKernelGGL(KERN, dim3(blocks), dim3(NW * 64), 0, 0, src, region, iters, sink); }, 5); \
    double bytes = (double)blocks * iters * NW * PIECES * 1024;                                              \
    printf("%-34s %6zuMB %10.1f %12.1f\n", NAME, region >> 20, ms * 1e3, bytes / blocks / (ms * 1e-3 * 2.1e9)); \
  }
    RUN("glds nw4 p2 depth2", (glds_feed<4, 2, 2>), 4, 2);
    RUN("glds nw4 p4 depth3", (glds_feed<4, 4, 3>), 4, 4);
    RUN("glds nw8 p2 depth3", (glds_feed<8, 2, 3>), 8, 2);
    RUN("glds nw8 p4 depth2", (glds_feed<8, 4, 2>), 8, 4);
    RUN("glds nw8 p4 depth3", (glds_feed<8, 4, 3>), 8, 4);
    RUN("glds nw8 p4 depth4", (glds_feed<8, 4, 4>), 8, 4);
    RUN("glds nw16 p2 depth3", (glds_feed<16, 2, 3>), 16, 2);
    RUN("glds nw16 p2 depth4", (glds_feed<16, 2, 4>), 16, 2);
    RUN("reg nw4 p4", (reg_feed<4, 4, false>), 4, 4);
    RUN("reg nw8 p2", (reg_feed<8, 2, false>), 8, 2);
    RUN("reg nw8 p4", (reg_feed<8, 4, false>), 8, 4);
    RUN("reg nw16 p2", (reg_feed<16, 2, false>), 16, 2);
    RUN("reg nw16 p4", (reg_feed<16, 4, false>), 16, 4);
    RUN("reg+ds_write nw8 p4", (reg_feed<8, 4, true>), 8, 4);
    RUN("reg+ds_write nw16 p2", (reg_feed<16, 2, true>), 16, 2);
  }
  return 0;
}
