// Fused pair of ResNet 1x1 convs across a block boundary at the reference's
// precision (fp32 in / fp32 accumulate on v_mfma_f32_16x16x4_f32):
//
//   y = relu(x . W3 + b3 + res)     64 -> 256   (block k's `_3_conv` + BN + add + ReLU = `_out`)
//   z = relu(y . W1 + b1)           256 -> 64   (block k+1's `_1_conv` + BN + ReLU)
//
// ResNet stage 2 (56x56, bs=32: 100,352 pixels) at fp32 moves 103 MB per
// 256-channel tensor.  Unfused, the `_out` conv writes y and the next `_1`
// conv reads it straight back (56 + 41 us per pair on the tile kernels,
// profiles/r3/r3k); here y is written once (it is the next residual) and the
// second GEMM reads it from LDS, in one launch.  The pw_pair.hip (bf16) v4
// structure carried to fp32:
//
// * 8 waves, persistent over BM-pixel tiles; every wave keeps its W3 fragments
//   (32 output channels x 64 k: 32 VGPRs) and its W1 fragments (16 output
//   channels x one 128-wide K half: 32 VGPRs) in registers for the launch;
// * GEMMs transposed (A = weight fragment, B = activation fragment from LDS,
//   D = [channel][pixel]): a lane's accumulator is 4 consecutive channels of
//   one pixel, so residual / y accesses are 16 bytes;
// * k permutation of the fp32 conv kernels: in half h, lane group q supplies
//   k = 16h + 4q + s to MFMA step s for both operands, so each operand fragment
//   of 4 steps is ONE 16-byte load (ds_read_b128 of the activation rows);
// * LDS rows are XOR-swizzled by 16-byte chunk (chunk ^ (row & 15)): the 16
//   pixels a ds_read_b128 lane group reads land in distinct bank slots;
// * the next tile's x and residual rows are loaded into registers (16-byte
//   row-contiguous loads) under this tile's GEMMs and staged into the other
//   LDS buffer at its end, so HBM streams continuously;
// * GEMM2 splits K over the two wave halves (waves 4-7 take k 128..255); their
//   partial z meets wave w-4's in LDS and leaves from registers.
#include "kernels.h"

namespace adapt {

namespace {

template <int NCH>
__device__ __forceinline__ int fswz(int r, int c) {   // 16-byte chunk c of row r (NCH chunks per row)
  return r * (NCH * 16) + (((c & ~15) | ((c ^ r) & 15)) << 4);
}

}  // namespace

template <int BM>
__global__ __launch_bounds__(512, 1) void pw_pair_f32_kernel(PwPairF32Params p) {
  constexpr int CIN = 64, CO = 256, CM = 64, NT = 512;
  constexpr int XCH = CIN / 4, YCH = CO / 4;          // 16-byte chunks per pixel row
  constexpr int PF = BM / 16;
  constexpr int AB = BM * CIN * 4, RB = BM * CO * 4, ZB = BM * CM * 4;
  constexpr int XIT = (BM * XCH + NT - 1) / NT;
  constexpr int RIT = BM * YCH / NT;
  static_assert((BM * YCH) % NT == 0 && BM % 16 == 0, "pair shape");
  static_assert(2 * AB + 2 * RB + ZB <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[2 * AB + 2 * RB + ZB];
  char* const abuf = smem;
  char* const rbuf = smem + 2 * AB;
  char* const zbuf = smem + 2 * AB + 2 * RB;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int ntiles = (p.M + BM - 1) / BM;
  if ((int)blockIdx.x >= ntiles) return;
  const int c2 = wave & 3, kh = wave >> 2;            // GEMM2: output fragment, K half

  // resident weights (host-packed in fragment order, lane-linear) and biases
  f32x4 wa[2][4], wb[8];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int h = 0; h < 4; ++h) wa[j][h] = *(const f32x4*)(p.w3 + (((wave * 2 + j) * 4 + h) * 64 + lane) * 4);
#pragma unroll
  for (int h = 0; h < 8; ++h) wb[h] = *(const f32x4*)(p.w1 + ((wave * 8 + h) * 64 + lane) * 4);
  f32x4 ba[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) ba[j] = *(const f32x4*)(p.b3 + (wave * 2 + j) * 16 + fq * 4);
  const f32x4 bz = *(const f32x4*)(p.b1 + c2 * 16 + fq * 4);

  f32x4 ra[XIT], rres[RIT];
  auto load_next = [&](int t) __attribute__((always_inline)) {
#pragma unroll
    for (int it = 0; it < XIT; ++it) {
      const int i = tid + it * NT;
      const int px = i / XCH, c = i - px * XCH;
      const int m = min(t * BM + px, p.M - 1);
      if (XIT * NT == BM * XCH || i < BM * XCH) ra[it] = *(const f32x4*)(p.x + (size_t)m * CIN + c * 4);
    }
#pragma unroll
    for (int it = 0; it < RIT; ++it) {
      const int i = tid + it * NT;
      const int px = i / YCH, c = i - px * YCH;
      const int m = min(t * BM + px, p.M - 1);
      rres[it] = *(const f32x4*)(p.res + (size_t)m * CO + c * 4);
    }
  };
  auto stage_next = [&](int b) __attribute__((always_inline)) {
#pragma unroll
    for (int it = 0; it < XIT; ++it) {
      const int i = tid + it * NT;
      if (XIT * NT == BM * XCH || i < BM * XCH) *(f32x4*)(abuf + b * AB + fswz<XCH>(i / XCH, i % XCH)) = ra[it];
    }
#pragma unroll
    for (int it = 0; it < RIT; ++it) {
      const int i = tid + it * NT;
      *(f32x4*)(rbuf + b * RB + fswz<YCH>(i / YCH, i % YCH)) = rres[it];
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
    if (more) load_next(tn);                         // in flight under this tile's two GEMMs
    const char* a = abuf + buf * AB;
    char* r = rbuf + buf * RB;
    // ---- GEMM1: y^T[256][BM] = W3^T . x^T, this wave's 32 channels; epilogue in place over the residual
    {
      f32x4 acc[2][PF];
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < PF; ++i) acc[j][i] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int h = 0; h < 4; ++h)
#pragma unroll
        for (int i = 0; i < PF; ++i) {
          const f32x4 xf = *(const f32x4*)(a + fswz<XCH>(i * 16 + fr, h * 4 + fq));
#pragma unroll
          for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int j = 0; j < 2; ++j)
              acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[j][h][s], xf[s], acc[j][i], 0, 0, 0);
        }
#pragma unroll
      for (int i = 0; i < PF; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          // acc[j][i][e] = y[pixel 16i + fr][channel 32 wave + 16 j + 4 fq + e]
          const int ch = (wave * 2 + j) * 16 + fq * 4;
          f32x4* q = (f32x4*)(r + fswz<YCH>(i * 16 + fr, ch >> 2));
          const f32x4 res = *q;
          f32x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = fmaxf(acc[j][i][e] + ba[j][e] + res[e], 0.f);
          *q = o;
          if (m0 + i * 16 + fr < p.M) *(f32x4*)(p.y + (size_t)(m0 + i * 16 + fr) * CO + ch) = o;
        }
    }
    __syncthreads();                                 // y complete in LDS; every read of x done
    // ---- GEMM2: z^T[64][BM] = W1^T . y^T, channels 16 c2.., K half kh; halves meet in LDS
    {
      f32x4 acc[PF];
#pragma unroll
      for (int i = 0; i < PF; ++i) acc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int h = 0; h < 8; ++h)
#pragma unroll
        for (int i = 0; i < PF; ++i) {
          const f32x4 yf = *(const f32x4*)(r + fswz<YCH>(i * 16 + fr, kh * 32 + h * 4 + fq));
#pragma unroll
          for (int s = 0; s < 4; ++s) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(wb[h][s], yf[s], acc[i], 0, 0, 0);
        }
      const int ch = c2 * 16 + fq * 4;
      if (kh == 1) {
#pragma unroll
        for (int i = 0; i < PF; ++i) *(f32x4*)(zbuf + fswz<CM / 4>(i * 16 + fr, ch >> 2)) = acc[i];
      }
      __syncthreads();                               // the upper K half's partial z is in LDS
      if (kh == 0) {
#pragma unroll
        for (int i = 0; i < PF; ++i) {
          const f32x4 o2 = *(const f32x4*)(zbuf + fswz<CM / 4>(i * 16 + fr, ch >> 2));
          f32x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = fmaxf(acc[i][e] + o2[e] + bz[e], 0.f);
          if (m0 + i * 16 + fr < p.M) *(f32x4*)(p.z + (size_t)(m0 + i * 16 + fr) * CM + ch) = o;
        }
      }
    }
    if (more) stage_next(buf ^ 1);
    __syncthreads();                                 // next tile staged; zbuf and this tile's rows free
    buf ^= 1;
  }
}

// BM instances (pixels per tile): ResNet stage 2 at fp32 (56x56, 64 -> 256 -> 64)
#define ADAPT_PAIR_F32_CFGS(X) \
  X(16)                        \
  X(32)

bool pw_pair_f32_supported(int cin, int co, int cm, int bm) {
  if (cin != 64 || co != 256 || cm != 64) return false;
#define X(BM_) if (bm == BM_) return true;
  ADAPT_PAIR_F32_CFGS(X)
#undef X
  return false;
}

hipError_t pw_pair_f32_forward(const PwPairF32Params& p, int cin, int co, int cm, int bm, int grid,
                               hipStream_t s) {
  if (!pw_pair_f32_supported(cin, co, cm, bm) || p.M < 1) return hipErrorInvalidValue;
#define X(BM_)                                                                                              \
  if (bm == BM_) {                                                                                          \
    const int nt = (p.M + BM_ - 1) / BM_;                                                                   \
    const int g = grid > 0 ? grid : 256;                                                                    \
    hipLaunchKernelGGL((pw_pair_f32_kernel<BM_>), dim3(nt < g ? nt : g), dim3(512), 0, s, p);              \
    return hipGetLastError();                                                                               \
  }
  ADAPT_PAIR_F32_CFGS(X)
#undef X
  return hipErrorInvalidValue;
}

}  // namespace adapt
