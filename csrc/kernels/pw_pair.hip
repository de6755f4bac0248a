// Fused pair of ResNet 1x1 convs across a block boundary (gfx950 MFMA):
//
//   y = relu(x . W3^T + b3 + res)     CIN -> CO   (block k's `_3_conv` + BN + add + ReLU = `_out`)
//   z = relu(y . W1^T + b1)           CO  -> CM   (block k+1's `_1_conv` + BN + ReLU)
//
// Unfused these are two launches; the second re-reads y (CO channels, the
// widest tensor of the stage) from L2 / HBM right after the first wrote it,
// and pays a dependent-launch gap (~2 us on MI355X, tools/launch_gap.py).
// Here y is computed for all CO channels of a BM-pixel tile and kept in LDS
// as bf16 (it is also written to HBM once, as the next block's residual), and
// z is computed from the LDS copy: y never makes the HBM round trip and the
// pair is one launch.
//
// Weights come in the host-packed MFMA fragment order of bottleneck.hip
// (ops/conv.py `pack_fragments`) and stay in registers.  GEMMs run transposed
// (A = weight fragment, B = activation fragment from LDS, D = [channel][pixel]):
// a lane's accumulator is four consecutive channels of one pixel, so the
// residual / y / z LDS accesses of the epilogues are 8 bytes.  Pixel rows >= M
// read row M-1 and store nothing.
#include "kernels.h"

namespace adapt {

namespace {

typedef __bf16 bf16x4v __attribute__((ext_vector_type(4)));

template <int NCH>
__device__ __forceinline__ int pswz(int r, int c) {   // 16-byte chunk c of row r, NCH chunks per row
  return r * (NCH * 16) + ((c ^ (r & 15)) << 4);
}

}  // namespace

// v4: persistent and software-pipelined, after pw_wide.hip.  v1-v3 gave each
// workgroup one tile and ran all workgroups in lock step, so HBM idled during
// the compute phases (profiles/r2/experiments/pair: 24.8 us against 24.0 us
// for the two tuned launches).  Here NWV = CO / 64 waves keep their W3
// fragments (64 output channels x KS1) AND their W1 fragments (CM / NWV output
// channels x KS2) in registers for the whole launch, and a persistent block
// walks BM-pixel tiles: the next tile's x and residual rows are loaded into
// registers under the current tile's MFMAs (16-byte row-contiguous loads) and
// go to the other LDS buffer at the end, so HBM streams continuously.  Per tile:
//   GEMM1   y = relu(x . W3 + b3 + res)  written in place over the residual rows in LDS
//   GEMM2   z = relu(y . W1 + b1)        from the y rows in LDS, z staged over the dead x rows
//   stores  y and z rows leave with 16-byte row-contiguous stores
template <int CIN, int CO, int CM, int BM, int NWV>
__global__ __launch_bounds__(NWV * 64, 1) void pw_pair_kernel(PwPairParams p) {
  constexpr int NT = NWV * 64;
  constexpr int KS1 = CIN / 32, KS2 = CO / 32;
  constexpr int XCH = CIN / 8, YCH = CO / 8, ZCH = CM / 8;
  constexpr int PF = BM / 16;
  constexpr int CFW = CO / 16 / NWV, CMW = CM / 16 / NWV;
  constexpr int AB = BM * CIN * 2, RB = BM * CO * 2;
  constexpr int XIT = (BM * XCH + NT - 1) / NT;
  constexpr int RIT = BM * YCH / NT;
  constexpr int ZIT = (BM * ZCH + NT - 1) / NT;
  static_assert(CFW * 16 * NWV == CO && CMW * 16 * NWV == CM && CMW >= 1 && (BM * YCH) % NT == 0 &&
                    XCH <= 16 && ZCH <= XCH && BM % 16 == 0,
                "pair shape");
  static_assert(2 * AB + 2 * RB <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[2 * AB + 2 * RB];
  char* const abuf = smem;
  char* const rbuf = smem + 2 * AB;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int ntiles = (p.M + BM - 1) / BM;
  if ((int)blockIdx.x >= ntiles) return;

  // resident weights and biases
  const bf16x8* w3 = (const bf16x8*)p.w3;
  const bf16x8* w1 = (const bf16x8*)p.w1;
  bf16x8 wa[CFW][KS1], wb[CMW][KS2];
  f32x4 ba[CFW], bz[CMW];
#pragma unroll
  for (int j = 0; j < CFW; ++j) {
#pragma unroll
    for (int k = 0; k < KS1; ++k) wa[j][k] = w3[((wave * CFW + j) * KS1 + k) * 64 + lane];
    ba[j] = *(const f32x4*)(p.b3 + (wave * CFW + j) * 16 + fq * 4);
  }
#pragma unroll
  for (int j = 0; j < CMW; ++j) {
#pragma unroll
    for (int k = 0; k < KS2; ++k) wb[j][k] = w1[((wave * CMW + j) * KS2 + k) * 64 + lane];
    bz[j] = *(const f32x4*)(p.b1 + (wave * CMW + j) * 16 + fq * 4);
  }

  u32x4 ra[XIT], rres[RIT];
  auto load_next = [&](int t) __attribute__((always_inline)) {
#pragma unroll
    for (int it = 0; it < XIT; ++it) {
      const int i = tid + it * NT;
      const int px = i / XCH, c = i - px * XCH;
      const int m = min(t * BM + px, p.M - 1);
      ra[it] = *(const u32x4*)(p.x + (size_t)m * CIN + c * 8);
    }
#pragma unroll
    for (int it = 0; it < RIT; ++it) {
      const int i = tid + it * NT;
      const int px = i / YCH, c = i - px * YCH;
      const int m = min(t * BM + px, p.M - 1);
      rres[it] = *(const u32x4*)(p.res + (size_t)m * CO + c * 8);
    }
  };
  auto stage_next = [&](int b) __attribute__((always_inline)) {
#pragma unroll
    for (int it = 0; it < XIT; ++it) {
      const int i = tid + it * NT;
      if (i < BM * XCH) *(u32x4*)(abuf + b * AB + pswz<XCH>(i / XCH, i % XCH)) = ra[it];
    }
#pragma unroll
    for (int it = 0; it < RIT; ++it) {
      const int i = tid + it * NT;
      *(u32x4*)(rbuf + b * RB + pswz<YCH>(i / YCH, i % YCH)) = rres[it];
    }
  };

  int t = blockIdx.x;
  load_next(t);
  stage_next(0);
  __syncthreads();
  int buf = 0;
  for (; t < ntiles; t += gridDim.x) {
    const int tn = t + gridDim.x;
    const bool more = tn < ntiles;
    const int m0 = t * BM;
    if (more) load_next(tn);                     // in flight under this tile's two GEMMs
    char* a = abuf + buf * AB;
    char* r = rbuf + buf * RB;
    // ---- GEMM1 + epilogue in place over the residual rows
    {
      f32x4 acc[CFW][PF];
#pragma unroll
      for (int j = 0; j < CFW; ++j)
#pragma unroll
        for (int i = 0; i < PF; ++i) acc[j][i] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < KS1; ++k)
#pragma unroll
        for (int i = 0; i < PF; ++i) {
          const bf16x8 af = *(const bf16x8*)(a + pswz<XCH>(i * 16 + fr, k * 4 + fq));
#pragma unroll
          for (int j = 0; j < CFW; ++j) acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[j][k], af, acc[j][i], 0, 0, 0);
        }
#pragma unroll
      for (int i = 0; i < PF; ++i)
#pragma unroll
        for (int j = 0; j < CFW; ++j) {
          const int n = (wave * CFW + j) * 16 + fq * 4;
          char* q = r + pswz<YCH>(i * 16 + fr, n >> 3) + (n & 7) * 2;
          const bf16x4v res = *(const bf16x4v*)q;
          bf16x4v o;
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = f2bf(fmaxf(acc[j][i][e] + ba[j][e] + bf2f(res[e]), 0.f));
          *(bf16x4v*)q = o;
        }
    }
    __syncthreads();                             // y complete in LDS; every read of x done
    // y rows leave now, under GEMM2
#pragma unroll
    for (int it = 0; it < RIT; ++it) {
      const int i = tid + it * NT;
      const int px = i / YCH, c = i - px * YCH;
      if (m0 + px < p.M) *(u32x4*)(p.y + (size_t)(m0 + px) * CO + c * 8) = *(const u32x4*)(r + pswz<YCH>(px, c));
    }
    // ---- GEMM2 from the y rows, z staged over the dead x rows
    {
      f32x4 acc[CMW][PF];
#pragma unroll
      for (int j = 0; j < CMW; ++j)
#pragma unroll
        for (int i = 0; i < PF; ++i) acc[j][i] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < KS2; ++k)
#pragma unroll
        for (int i = 0; i < PF; ++i) {
          const bf16x8 yf = *(const bf16x8*)(r + pswz<YCH>(i * 16 + fr, k * 4 + fq));
#pragma unroll
          for (int j = 0; j < CMW; ++j) acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[j][k], yf, acc[j][i], 0, 0, 0);
        }
#pragma unroll
      for (int i = 0; i < PF; ++i)
#pragma unroll
        for (int j = 0; j < CMW; ++j) {
          const int n = (wave * CMW + j) * 16 + fq * 4;
          bf16x4v o;
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = f2bf(fmaxf(acc[j][i][e] + bz[j][e], 0.f));
          *(bf16x4v*)(a + pswz<ZCH>(i * 16 + fr, n >> 3) + (n & 7) * 2) = o;
        }
    }
    __syncthreads();                             // z complete in LDS; every read of y done
#pragma unroll
    for (int it = 0; it < ZIT; ++it) {
      const int i = tid + it * NT;
      const int px = i / ZCH, c = i - px * ZCH;
      if (i < BM * ZCH && m0 + px < p.M)
        *(u32x4*)(p.z + (size_t)(m0 + px) * CM + c * 8) = *(const u32x4*)(a + pswz<ZCH>(px, c));
    }
    if (more) stage_next(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
}

// (CIN, CO, CM, BM, NWV) instances: ResNet stage 3 (28x28: 128 -> 512 -> 128).
// Stage 4 (256 -> 1024 -> 256) would hold 64 W1 fragments per wave for phase 2
// and spills; it stays on the two-launch path.
#define ADAPT_PAIR_CFGS(X) \
  X(128, 512, 128, 16, 8)

bool pw_pair_supported(int cin, int co, int cm, int bm) {
#define X(CI, CO_, CM_, BM_, NW_) if (cin == CI && co == CO_ && cm == CM_ && bm == BM_) return true;
  ADAPT_PAIR_CFGS(X)
#undef X
  return false;
}

hipError_t pw_pair_forward(const PwPairParams& p, int cin, int co, int cm, int bm, hipStream_t s) {
#define X(CI, CO_, CM_, BM_, NW_)                                                                     \
  if (cin == CI && co == CO_ && cm == CM_ && bm == BM_) {                                            \
    const int nt = (p.M + BM_ - 1) / BM_;                                                           \
    hipLaunchKernelGGL((pw_pair_kernel<CI, CO_, CM_, BM_, NW_>), dim3(nt < 256 ? nt : 256), dim3(NW_ * 64), 0, s, p); \
    return hipGetLastError();                                                                        \
  }
  ADAPT_PAIR_CFGS(X)
#undef X
  return hipErrorInvalidValue;
}

}  // namespace adapt
