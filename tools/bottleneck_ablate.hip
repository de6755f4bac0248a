// Ablation of the fused stage-2 bottleneck kernel (csrc/kernels/bottleneck.hip)
// on ResNet-50 bs=32 (56x56x256 identity block): time with the MFMAs, the
// x-halo loads, the weight loads, the output stores or the y1/y2 LDS writes
// removed, interleaved in one process (median of 7 rounds of 20 launches).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Icsrc/kernels -o tools/bin/bottleneck_ablate tools/bottleneck_ablate.hip
//   tools/bin/bottleneck_ablate
#include "../csrc/kernels/bottleneck.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHECK(x)                                                        \
  do {                                                                  \
    hipError_t e_ = (x);                                                \
    if (e_ != hipSuccess) {                                             \
      printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));  \
      exit(1);                                                          \
    }                                                                   \
  } while (0)

using namespace adapt;

static unsigned short f2bf_host(float f) {
  unsigned u;
  memcpy(&u, &f, 4);
  return (unsigned short)((u + 0x7fff + ((u >> 16) & 1)) >> 16);
}

template <typename T>
static T* upload_bf16(size_t n, float scale) {
  std::vector<unsigned short> h(n);
  for (auto& v : h) v = f2bf_host(((rand() / (float)RAND_MAX) * 2.f - 1.f) * scale);
  T* d;
  CHECK(hipMalloc(&d, n * 2));
  CHECK(hipMemcpy(d, h.data(), n * 2, hipMemcpyHostToDevice));
  return d;
}

template <int ABL>
static float run(const BottleneckParams& p, int launches) {
  const dim3 grid(p.B * (p.H / 8) * (p.W / 8)), block(256);
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((bottleneck_kernel<256, false, ABL>), grid, block, 0, 0, p);
  CHECK(hipEventRecord(a));
  for (int i = 0; i < launches; ++i) hipLaunchKernelGGL((bottleneck_kernel<256, false, ABL>), grid, block, 0, 0, p);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  CHECK(hipGetLastError());
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
  return ms * 1e3f / launches;
}

int main() {
  srand(1);
  BottleneckParams p;
  memset(&p, 0, sizeof(p));
  p.B = 32; p.H = 56; p.W = 56;
  p.x = upload_bf16<bf16>((size_t)p.B * p.H * p.W * 256, 1.f);
  p.w1 = upload_bf16<bf16>(64 * 256, 0.05f);
  p.w2 = upload_bf16<bf16>(64 * 576, 0.05f);
  p.w3 = upload_bf16<bf16>(256 * 64, 0.05f);
  float* bias;
  CHECK(hipMalloc(&bias, 256 * 4));
  CHECK(hipMemset(bias, 0, 256 * 4));
  p.b1 = p.b2 = p.b3 = bias;
  CHECK(hipMalloc(&p.out, (size_t)p.B * p.H * p.W * 256 * 2));
  constexpr int NV = 12;
  const char* names[NV] = {"base", "no MFMA", "no x load", "no W load", "no out store", "no y LDS writes",
                           "no loads", "no loads/MFMA", "skeleton", "no A ds_read", "no res/out LDS",
                           "bare"};
  std::vector<float> t[NV];
  for (int r = 0; r < 7; ++r) {
    t[0].push_back(run<0>(p, 20));
    t[1].push_back(run<1>(p, 20));
    t[2].push_back(run<2>(p, 20));
    t[3].push_back(run<4>(p, 20));
    t[4].push_back(run<8>(p, 20));
    t[5].push_back(run<16>(p, 20));
    t[6].push_back(run<6>(p, 20));
    t[7].push_back(run<7>(p, 20));
    t[8].push_back(run<31>(p, 20));
    t[9].push_back(run<32>(p, 20));
    t[10].push_back(run<64>(p, 20));
    t[11].push_back(run<127>(p, 20));
  }
  const double flop = 2.0 * p.B * p.H * p.W * (256.0 * 64 + 576.0 * 64 + 64.0 * 256);
  printf("stage-2 identity bottleneck, bs=32: %d tiles of 8x8, 256 threads, 2 blocks/CU\n", p.B * 49);
  for (int v = 0; v < NV; ++v) {
    std::sort(t[v].begin(), t[v].end());
    printf("  %-16s %8.2f us  (min %7.2f)  %6.1f TF/s-equiv\n", names[v], t[v][3], t[v][0], flop / (t[v][3] * 1e-6) / 1e12);
  }
  return 0;
}
