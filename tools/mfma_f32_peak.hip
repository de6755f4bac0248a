// fp32 matrix-core ceiling on this chip, under full load: every CU runs waves
// that issue v_mfma_f32_16x16x4_f32 back to back on independent accumulators
// with operands held in registers (random data, no memory traffic in the loop).
// Reports TFLOP/s and the in-kernel clock (s_memtime / s_memrealtime ticks).
// This is the roof the fp32 conv kernels are judged against.
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_f32_peak.hip -o /tmp/mfma_f32_peak && /tmp/mfma_f32_peak
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ __launch_bounds__(256) void peak(const float* __restrict__ seed, float* __restrict__ sink, int iters,
                                            unsigned long long* clk) {
  const int lane = threadIdx.x & 63;
  float a = seed[(blockIdx.x * 256 + threadIdx.x) % 4096];
  float b = seed[(blockIdx.x * 256 + threadIdx.x + 17) % 4096];
  f32x4 acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = (f32x4){a, b, a * b, (float)lane};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  sink[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) {
    clk[blockIdx.x * 2] = t1 - t0;
    clk[blockIdx.x * 2 + 1] = r1 - r0;
  }
}

int main(int argc, char** argv) {
  const int blocks = argc > 1 ? atoi(argv[1]) : 1024;   // 4 waves each: 1024 blocks = 4 per CU = 4 waves/SIMD
  const int iters = argc > 2 ? atoi(argv[2]) : 20000;
  std::vector<float> h(4096);
  srand(1);
  for (auto& v : h) v = (float)rand() / RAND_MAX - 0.5f;
  float *seed, *sink;
  unsigned long long* clk;
  hipMalloc(&seed, 4096 * 4);
  hipMalloc(&sink, (size_t)blocks * 256 * 4);
  hipMalloc(&clk, (size_t)blocks * 2 * 8);
  hipMemcpy(seed, h.data(), 4096 * 4, hipMemcpyHostToDevice);
  for (int nacc : {4, 8, 16}) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(e0);
      if (nacc == 4) hipLaunchKernelGGL(peak<4>, dim3(blocks), dim3(256), 0, 0, seed, sink, iters * 4, clk);
      if (nacc == 8) hipLaunchKernelGGL(peak<8>, dim3(blocks), dim3(256), 0, 0, seed, sink, iters * 2, clk);
      if (nacc == 16) hipLaunchKernelGGL(peak<16>, dim3(blocks), dim3(256), 0, 0, seed, sink, iters, clk);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
    }
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    const double flop = 2.0 * 16 * 16 * 4 * (double)iters * 16 * 4 * blocks;   // 16 MFMAs/iter-equiv x 4 waves
    std::vector<unsigned long long> c((size_t)blocks * 2);
    hipMemcpy(c.data(), clk, c.size() * 8, hipMemcpyDeviceToHost);
    double ghz = 0;
    for (int b = 0; b < blocks; ++b) ghz += (double)c[2 * b] / (double)c[2 * b + 1] * 0.1;   // realtime = 100 MHz
    ghz /= blocks;
    printf("{\"kernel\": \"v_mfma_f32_16x16x4_f32 back-to-back, %d independent accumulators\", \"blocks\": %d, "
           "\"ms\": %.3f, \"tflops\": %.1f, \"clock_ghz\": %.3f}\n", nacc, blocks, ms, flop / ms / 1e9, ghz);
  }
  return 0;
}
