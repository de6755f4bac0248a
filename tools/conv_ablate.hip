// Ablation of the LDS-DMA implicit-GEMM conv kernel (csrc/kernels/conv_glds.hip)
// on the ResNet-50 bs=32 3x3 layers: what does a K tile cost with its MFMAs
// removed, with its LDS-DMA removed, with both removed (loop + barrier
// skeleton), and with every K tile re-fetching the block's first one
// (operands L2-hot)?  All variants of a problem run interleaved in one process
// (median of 7 rounds of 20 launches).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Icsrc/kernels -o tools/bin/conv_ablate tools/conv_ablate.hip
//   tools/bin/conv_ablate
#include "../csrc/kernels/conv_glds.hip"

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

struct Problem {
  const char* name;
  int B, H, W, Cin, Cout, ksplit;
  ConvParams p;
};

static unsigned short f2bf_host(float f) {
  unsigned u;
  memcpy(&u, &f, 4);
  return (unsigned short)((u + 0x7fff + ((u >> 16) & 1)) >> 16);
}

static void setup(Problem& pr) {
  ConvParams& p = pr.p;
  memset(&p, 0, sizeof(p));
  p.B = pr.B; p.H = pr.H; p.W = pr.W; p.Cin = pr.Cin;
  p.OH = pr.H; p.OW = pr.W; p.N = pr.Cout;
  p.KH = p.KW = 3; p.stride = 1; p.pad_t = p.pad_l = 1;
  p.M = pr.B * pr.H * pr.W;
  p.K = 9 * pr.Cin;
  p.Kpad = (p.K + 63) / 64 * 64;
  p.ldo = p.N;
  p.relu = 1;
  p.ksplit = pr.ksplit;
  const size_t nx = (size_t)pr.B * pr.H * pr.W * pr.Cin, nw = (size_t)p.N * p.Kpad;
  std::vector<unsigned short> hx(nx), hw(nw);
  srand(1);
  for (auto& v : hx) v = f2bf_host((rand() / (float)RAND_MAX) * 2.f - 1.f);
  for (auto& v : hw) v = f2bf_host(((rand() / (float)RAND_MAX) * 2.f - 1.f) * 0.02f);
  bf16 *dx, *dw, *dout;
  float *db, *dws = nullptr;
  CHECK(hipMalloc(&dx, nx * 2));
  CHECK(hipMalloc(&dw, nw * 2));
  CHECK(hipMalloc(&dout, (size_t)p.M * p.N * 2));
  CHECK(hipMalloc(&db, p.N * 4));
  CHECK(hipMemcpy(dx, hx.data(), nx * 2, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dw, hw.data(), nw * 2, hipMemcpyHostToDevice));
  CHECK(hipMemset(db, 0, p.N * 4));
  if (pr.ksplit > 1) CHECK(hipMalloc(&dws, (size_t)pr.ksplit * p.M * p.N * 4));
  p.x = dx; p.w = dw; p.bias = db; p.out = dout; p.ws = dws;
}

template <int BM, int BN, int WM, int WN, int S, int ABL, int NL>
static float run(const Problem& pr, const bf16* zero, int launches) {
  const ConvParams& p = pr.p;
  constexpr bool ILV = NL == 0;
  dim3 grid(((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN), p.ksplit), block((WM * WN + NL) * 64);
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i)
    hipLaunchKernelGGL((conv_glds_kernel<BM, BN, WM, WN, S, ILV, false, false, ABL, NL>), grid, block, 0, 0, p, zero);
  CHECK(hipEventRecord(a));
  for (int i = 0; i < launches; ++i)
    hipLaunchKernelGGL((conv_glds_kernel<BM, BN, WM, WN, S, ILV, false, false, ABL, NL>), grid, block, 0, 0, p, zero);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  CHECK(hipGetLastError());
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
  return ms * 1e3f / launches;
}

constexpr int kNV = 6;
static const char* kAblName[kNV] = {"base", "no-MFMA", "no-DMA", "DMA only", "barriers only", "no K loop"};

// checksum of the output (bf16 bits summed) to compare variants for equality
static double checksum(const Problem& pr) {
  const ConvParams& p = pr.p;
  std::vector<unsigned short> h((size_t)p.M * p.N);
  CHECK(hipMemcpy(h.data(), p.out, h.size() * 2, hipMemcpyDeviceToHost));
  double s = 0;
  for (auto v : h) {
    unsigned u = (unsigned)v << 16;
    float f;
    memcpy(&f, &u, 4);
    s += f;
  }
  return s;
}

template <int BM, int BN, int WM, int WN, int S, int NL>
static void study(Problem& pr, const bf16* zero) {
  const int rounds = 7, launches = 20;
  std::vector<float> t[kNV];
  for (int r = 0; r < rounds; ++r) {
    t[0].push_back(run<BM, BN, WM, WN, S, 0, NL>(pr, zero, launches));
    t[1].push_back(run<BM, BN, WM, WN, S, 1, NL>(pr, zero, launches));
    t[2].push_back(run<BM, BN, WM, WN, S, 2, NL>(pr, zero, launches));
    t[3].push_back(run<BM, BN, WM, WN, S, 9, NL>(pr, zero, launches));
    t[4].push_back(run<BM, BN, WM, WN, S, 11, NL>(pr, zero, launches));
    t[5].push_back(run<BM, BN, WM, WN, S, 19, NL>(pr, zero, launches));
  }
  run<BM, BN, WM, WN, S, 0, NL>(pr, zero, 1);
  CHECK(hipDeviceSynchronize());
  const double cs = pr.ksplit == 1 ? checksum(pr) : 0.0;
  const ConvParams& p = pr.p;
  const double flop = 2.0 * p.M * p.N * p.K;
  const int tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  const int ktiles = p.Kpad / 64 / p.ksplit;
  printf("%s: M=%d N=%d K=%d tile %dx%d waves %dx%d+%d loaders stages %d ksplit %d -> %d blocks x %d K tiles"
         " (checksum %.6e)\n", pr.name, p.M, p.N, p.K, BM, BN, WM, WN, NL, S, p.ksplit, tiles * p.ksplit, ktiles, cs);
  for (int v = 0; v < kNV; ++v) {
    std::sort(t[v].begin(), t[v].end());
    const float med = t[v][rounds / 2];
    printf("  %-14s %8.2f us  (min %7.2f)  %6.1f TF/s-equiv  %6.0f ns per K tile\n", kAblName[v], med, t[v][0],
           flop / (med * 1e-6) / 1e12, med * 1e3 / ktiles);
  }
}

int main() {
  bf16* zero = nullptr;
  CHECK(hipGetSymbolAddress((void**)&zero, HIP_SYMBOL(g_zero_page)));
  Problem s3{"stage3 3x3", 32, 28, 28, 128, 128, 1}, s4{"stage4 3x3", 32, 14, 14, 256, 256, 1},
      s4b{"stage4 3x3", 32, 14, 14, 256, 256, 2}, s5{"stage5 3x3", 32, 7, 7, 512, 512, 4};
  for (Problem* pr : {&s3, &s4, &s4b, &s5}) setup(*pr);
  study<128, 128, 4, 2, 3, 0>(s3, zero);     // tuned: cfg 20
  study<128, 128, 4, 2, 3, 4>(s3, zero);
  study<128, 128, 2, 2, 4, 4>(s3, zero);     // 64x64 per compute wave
  study<64, 128, 2, 4, 4, 0>(s4, zero);      // tuned: cfg 23
  study<64, 128, 2, 4, 4, 4>(s4, zero);
  study<64, 128, 2, 4, 6, 4>(s4, zero);
  study<128, 128, 2, 2, 4, 4>(s4b, zero);    // 64x64 per compute wave, split-K 2
  study<64, 256, 2, 4, 3, 0>(s5, zero);      // tuned: cfg 27, split-K 4 (slabs only)
  study<64, 256, 2, 4, 3, 4>(s5, zero);
  return 0;
}
