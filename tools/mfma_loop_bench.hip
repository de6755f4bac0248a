// Where the F(4x4) consumer loop's time goes (conv_wino4pc_f32.hip measured 1.5 us per 72-MFMA chunk with the
// producers idle, against 1.03 us of MFMA): the same chunk body -- 18 groups of 4 v_mfma_f32_16x16x4_f32 on 2
// accumulators (each used twice: K steps s = 0, 1), 36 accumulators live -- in isolation, one block per CU:
//   mode 0: operands in registers, no LDS, one wave per SIMD (256 threads)
//   mode 1: + the A pair of the next group read from LDS (ds_read2st64) and waited before its group
//   mode 2: mode 1 + a block barrier per chunk (256 threads)
//   mode 3: mode 2 with 512 threads, waves 4-7 idle at the barriers (the producer slots)
//   mode 4: mode 0 with the 4 MFMAs of a group on 4 accumulators (no dependency inside a group)
//   mode 5: mode 1 with the read issued two groups ahead
//   mode 6: mode 3 with waves 4-7 issuing 180 independent v_fma_f32 per chunk (the producer's transform load)
//   mode 7: mode 6 with v_add_u32 (integer VALU) instead
//   mode 8: mode 6 with 180 v_pk_fma_f32-free v_mul_f32
// Reports cycles per MFMA from the in-kernel clock (median over blocks).
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_loop_bench.hip -o tools/mfma_loop_bench.bin
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(512, 1) void body(const float* __restrict__ seed, float* __restrict__ sink, int chunks,
                                               unsigned long long* clk) {
  __shared__ float lds[16384];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 16384; i += blockDim.x) lds[i] = seed[i & 4095];
  __syncthreads();
  const bool worker = wave < 4;
  (void)worker;
  float b[18][2];
#pragma unroll
  for (int g = 0; g < 18; ++g) {
    b[g][0] = seed[(lane + 7 * g) & 4095];
    b[g][1] = seed[(lane + 11 * g) & 4095];
  }
  f32x4 acc[18][2];
#pragma unroll
  for (int g = 0; g < 18; ++g) acc[g][0] = acc[g][1] = (f32x4){b[g][0], b[g][1], 0.f, 1.f};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (worker) {
    const float* src = lds + lane;
    for (int c = 0; c < chunks; ++c) {
      if constexpr (MODE == 2 || MODE == 3 || MODE >= 6) __builtin_amdgcn_s_barrier();
      float av[3][2];
      if constexpr (MODE == 1 || MODE == 2 || MODE == 3 || MODE == 5) {
        av[0][0] = src[0];
        av[0][1] = src[128];
        if constexpr (MODE == 5) {
          av[1][0] = src[256];
          av[1][1] = src[384];
        }
      }
#pragma unroll
      for (int g = 0; g < 18; ++g) {
        float a0, a1;
        if constexpr (MODE == 0 || MODE == 4) {
          a0 = b[g][1];
          a1 = b[(g + 1) % 18][1];
        } else if constexpr (MODE == 5) {
          if (g < 16) {
            av[(g + 2) % 3][0] = src[((g + 2) * 512) & 16383];
            av[(g + 2) % 3][1] = src[((g + 2) * 512 + 128) & 16383];
          }
          a0 = av[g % 3][0];
          a1 = av[g % 3][1];
        } else {
          if (g < 17) {
            av[(g + 1) & 1][0] = src[((g + 1) * 512) & 16383];
            av[(g + 1) & 1][1] = src[((g + 1) * 512 + 128) & 16383];
          }
          a0 = av[g & 1][0];
          a1 = av[g & 1][1];
        }
        if constexpr (MODE == 4) {
          f32x4 x0 = acc[g][0], x1 = acc[g][1], x2 = acc[(g + 9) % 18][0], x3 = acc[(g + 9) % 18][1];
          x0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b[g][0], x0, 0, 0, 0);
          x1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b[g][1], x1, 0, 0, 0);
          x2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b[g][0], x2, 0, 0, 0);
          x3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b[g][1], x3, 0, 0, 0);
          acc[g][0] = x0; acc[g][1] = x1; acc[(g + 9) % 18][0] = x2; acc[(g + 9) % 18][1] = x3;
        } else {
#pragma unroll
          for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int j = 0; j < 2; ++j)
              acc[g][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(s ? a1 : a0, b[g][j], acc[g][j], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  } else if constexpr (MODE == 6 || MODE == 8) {
    float x[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) x[k] = b[k][0];
    const float y = b[13][1], z = b[14][1];
    for (int c = 0; c < chunks; ++c) {
      __builtin_amdgcn_s_barrier();
#pragma unroll
      for (int r = 0; r < 15; ++r)
#pragma unroll
        for (int k = 0; k < 12; ++k) x[k] = MODE == 6 ? fmaf(x[k], y, z) : x[k] * y;
      asm volatile("" ::"v"(x[0]), "v"(x[5]), "v"(x[11]));
    }
#pragma unroll
    for (int k = 0; k < 12; ++k) acc[0][0][0] += x[k];
  } else if constexpr (MODE == 7) {
    unsigned x[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) x[k] = __float_as_uint(b[k][0]);
    const unsigned y = __float_as_uint(b[13][1]);
    for (int c = 0; c < chunks; ++c) {
      __builtin_amdgcn_s_barrier();
#pragma unroll
      for (int r = 0; r < 15; ++r)
#pragma unroll
        for (int k = 0; k < 12; ++k) {
          x[k] = x[k] + y;
          asm volatile("" : "+v"(x[k]));
        }
    }
#pragma unroll
    for (int k = 0; k < 12; ++k) acc[0][0][0] += (float)x[k];
  } else {
    for (int c = 0; c < chunks; ++c) __builtin_amdgcn_s_barrier();
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
#pragma unroll
  for (int g = 0; g < 18; ++g) s += acc[g][0][0] + acc[g][1][1] + acc[g][0][2] + acc[g][1][3];
  sink[blockIdx.x * 512 + threadIdx.x] = s;
  if (lane == 0) clk[blockIdx.x * 8 + wave] = t1 - t0;
}

template <int MODE>
void run(const float* seed, float* sink, unsigned long long* clk, int chunks, const char* what) {
  const int blocks = 256, threads = (MODE == 3 || MODE >= 6) ? 512 : 256;
  for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(body<MODE>, dim3(blocks), dim3(threads), 0, 0, seed, sink, chunks, clk);
  hipDeviceSynchronize();
  std::vector<unsigned long long> c((size_t)blocks * 8);
  hipMemcpy(c.data(), clk, c.size() * 8, hipMemcpyDeviceToHost);
  std::vector<double> v;
  std::vector<double> pv;
  for (int b = 0; b < blocks; ++b) {
    v.push_back((double)c[b * 8] / (chunks * 72.0));
    if (threads == 512) pv.push_back((double)c[b * 8 + 4] / chunks);
  }
  std::sort(v.begin(), v.end());
  std::sort(pv.begin(), pv.end());
  printf("{\"mode\": %d, \"what\": \"%s\", \"cycles_per_mfma_median\": %.2f, \"p90\": %.2f, "
         "\"partner_cycles_per_chunk\": %.0f}\n", MODE, what, v[v.size() / 2], v[v.size() * 9 / 10],
         pv.empty() ? 0.0 : pv[pv.size() / 2]);
}

int main() {
  std::vector<float> h(16384);
  srand(1);
  for (auto& v : h) v = (float)rand() / RAND_MAX - 0.5f;
  float *seed, *sink;
  unsigned long long* clk;
  hipMalloc(&seed, 16384 * 4);
  hipMalloc(&sink, 256 * 512 * 4);
  hipMalloc(&clk, 256 * 8 * 8);
  hipMemcpy(seed, h.data(), 16384 * 4, hipMemcpyHostToDevice);
  const int chunks = 2000;
  run<0>(seed, sink, clk, chunks, "registers only, 1 wave/SIMD");
  run<1>(seed, sink, clk, chunks, "+ LDS A pair one group ahead");
  run<2>(seed, sink, clk, chunks, "+ barrier per chunk");
  run<3>(seed, sink, clk, chunks, "+ idle partner waves (512 threads)");
  run<4>(seed, sink, clk, chunks, "registers, 4 accumulators per group (no in-group dependency)");
  run<5>(seed, sink, clk, chunks, "LDS A pair two groups ahead");
  run<6>(seed, sink, clk, chunks, "mode 3 + partner 180 v_fma_f32 per chunk");
  run<7>(seed, sink, clk, chunks, "mode 3 + partner 180 v_add_u32 per chunk");
  run<8>(seed, sink, clk, chunks, "mode 3 + partner 180 v_mul_f32 per chunk");
  return 0;
}
