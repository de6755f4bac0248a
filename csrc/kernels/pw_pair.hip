// Fused pair of ResNet 1x1 convs across a block boundary (gfx950 MFMA):
//
//   y = relu(x . W3^T + b3 + res)     CIN -> CO   (block k's `_3_conv` + BN + add + ReLU = `_out`)
//   z = relu(y . W1^T + b1)           CO  -> CM   (block k+1's `_1_conv` + BN + ReLU)
//
// Unfused these are two launches; the second re-reads y (CO channels, the
// widest tensor of the stage) from L2 / HBM right after the first wrote it,
// and pays a dependent-launch gap (~2 us on MI355X, tools/launch_gap.py).
// Here a workgroup owns BM pixels: x is staged in LDS, y is computed for all
// CO channels and kept in LDS as bf16 (it is also written to HBM once, as the
// next block's residual), and z is computed from the LDS copy.  y never makes
// the HBM round trip and the pair is one launch.
//
// Weights stay in the host-packed MFMA fragment order of bottleneck.hip
// (ops/conv.py `pack_fragments`): one coalesced 1 KiB global/L2 load per wave
// per fragment, no LDS.  GEMMs run transposed (A = weight fragment, B =
// activation fragment from LDS, D = [channel][pixel]): a lane's accumulator is
// four consecutive channels of one pixel, so the bias / residual / output
// accesses are 8-byte vectors and each wave covers whole 128-byte row segments.
// NWV waves; phase 1 gives wave w the channel fragments [w*CFW, (w+1)*CFW) of
// y, phase 2 the fragments [w*CMW, (w+1)*CMW) of z.  Pixel rows >= M read row
// M-1 and store nothing.
#include "kernels.h"

namespace adapt {

namespace {

typedef __bf16 bf16x4v __attribute__((ext_vector_type(4)));

template <int NCH>
__device__ __forceinline__ int pswz(int r, int c) {   // 16-byte chunk c of row r, NCH chunks per row
  return r * (NCH * 16) + ((c ^ (r & 15)) << 4);
}

template <int CIN, int CO, int CM, int BM, int NWV>
struct PairShape {
  static constexpr int PF = BM / 16;                  // pixel fragments
  static constexpr int KS1 = CIN / 32, KS2 = CO / 32;
  static constexpr int CFW = CO / 16 / NWV;           // y channel fragments per wave
  static constexpr int CMW = CM / 16 / NWV;           // z channel fragments per wave
  static constexpr int CC = CFW < 2 ? CFW : 2;        // y fragments per accumulator chunk
  static constexpr int NCK = CFW / CC;                // chunks
  static constexpr int XS = BM * CIN * 2, YS = BM * CO * 2;
  static_assert(BM % 16 == 0 && CIN % 32 == 0 && CO % 32 == 0 && CFW * 16 * NWV == CO && CMW * 16 * NWV == CM &&
                    CFW % CC == 0 && CIN >= 128 && CO >= 128,
                "pair tile split");
  static_assert(XS + YS <= 160 * 1024, "LDS");
};

}  // namespace

// One workgroup per BM-pixel tile, sized so the whole grid is one round of
// workgroups (ResNet stage 3: 112 px -> 224 tiles for 256 CUs): a workgroup's
// dependent memory round trips are its critical path, so every load is issued
// as early as its registers allow --
//   prologue   x tile, chunk 0's residual / bias / W3 fragments (LDS-only barrier after x -> LDS)
//   chunk c    chunk c+1's residual / W3 fragments (or, under the last chunk, ALL of
//              phase 2's W1 fragments and bias) go out before chunk c's MFMAs
//   phase 2    only LDS reads and MFMAs, then the z stores
// so a workgroup waits on HBM about twice (x, then the last chunk's data), not
// once per chunk and weight group.
template <int CIN, int CO, int CM, int BM, int NWV>
__global__ __launch_bounds__(NWV * 64, 2) void pw_pair_kernel(PwPairParams p) {
  using S = PairShape<CIN, CO, CM, BM, NWV>;
  constexpr int PF = S::PF, KS1 = S::KS1, KS2 = S::KS2, CFW = S::CFW, CMW = S::CMW, CC = S::CC, NCK = S::NCK;
  constexpr int NT = NWV * 64;
  __shared__ __attribute__((aligned(16))) char smem[S::XS + S::YS];
  char* xs = smem;
  char* ys = smem + S::XS;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int tiles = (p.M + BM - 1) / BM;
  const int m0 = xcd_remap(blockIdx.x, tiles) * BM;
  const bf16x8* w3 = (const bf16x8*)p.w3;
  const bf16x8* w1 = (const bf16x8*)p.w1;
  constexpr int XCH = CIN / 8, YCH = CO / 8;

  // ---- prologue: x tile -> registers, chunk 0's operands, x -> LDS
  constexpr int XIT = (BM * XCH + NT - 1) / NT;
  u32x4 xr[XIT];
#pragma unroll
  for (int it = 0; it < XIT; ++it) {
    const int i = tid + it * NT;
    const int r = i / XCH, c = i - r * XCH;
    const int m = min(m0 + (i < BM * XCH ? r : 0), p.M - 1);
    xr[it] = *(const u32x4*)(p.x + (size_t)m * CIN + c * 8);
  }
  uint2 rr[2][CC][PF];
  bf16x8 wf[2][CC][KS1];
  f32x4 bb[2][CC];
  auto load_chunk = [&](int buf, int nf0) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < CC; ++j)
#pragma unroll
      for (int k = 0; k < KS1; ++k) wf[buf][j][k] = w3[((nf0 + j) * KS1 + k) * 64 + lane];
#pragma unroll
    for (int j = 0; j < CC; ++j) {
      bb[buf][j] = *(const f32x4*)(p.b3 + (nf0 + j) * 16 + fq * 4);
#pragma unroll
      for (int i = 0; i < PF; ++i) {
        const int m = min(m0 + i * 16 + fr, p.M - 1);
        rr[buf][j][i] = *(const uint2*)(p.res + (size_t)m * CO + (nf0 + j) * 16 + fq * 4);
      }
    }
  };
  load_chunk(0, wave * CFW);
#pragma unroll
  for (int it = 0; it < XIT; ++it) {
    const int i = tid + it * NT;
    if (i < BM * XCH) *(u32x4*)(xs + pswz<XCH>(i / XCH, i % XCH)) = xr[it];
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  const int nz0 = wave * CMW;
  bf16x8 wz[CMW][KS2];
  f32x4 bz[CMW];

  // ---- phase 1: y chunks (CC channel fragments x all pixel fragments)
#pragma unroll
  for (int ck = 0; ck < NCK; ++ck) {
    const int cur = ck & 1;
    const int nf0 = wave * CFW + ck * CC;
    if (ck + 1 < NCK) {
      load_chunk(cur ^ 1, nf0 + CC);
    } else {
#pragma unroll
      for (int j = 0; j < CMW; ++j) {
        bz[j] = *(const f32x4*)(p.b1 + (nz0 + j) * 16 + fq * 4);
#pragma unroll
        for (int k = 0; k < KS2; ++k) wz[j][k] = w1[((nz0 + j) * KS2 + k) * 64 + lane];
      }
    }
    f32x4 acc[CC][PF];
#pragma unroll
    for (int j = 0; j < CC; ++j)
#pragma unroll
      for (int i = 0; i < PF; ++i) acc[j][i] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < KS1; ++k) {
#pragma unroll
      for (int i = 0; i < PF; ++i) {
        const bf16x8 a = *(const bf16x8*)(xs + pswz<XCH>(i * 16 + fr, k * 4 + fq));
#pragma unroll
        for (int j = 0; j < CC; ++j)
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[cur][j][k], a, acc[j][i], 0, 0, 0);
      }
    }
#pragma unroll
    for (int j = 0; j < CC; ++j) {
      const int ch = (nf0 + j) * 16 + fq * 4;
#pragma unroll
      for (int i = 0; i < PF; ++i) {
        const int px = i * 16 + fr;
        const bf16x4v rv = __builtin_bit_cast(bf16x4v, rr[cur][j][i]);
        bf16x4v o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = f2bf(fmaxf(acc[j][i][r] + bb[cur][j][r] + bf2f(rv[r]), 0.f));
        *(bf16x4v*)(ys + pswz<YCH>(px, ch >> 3) + (ch & 4) * 2) = o;
        if (m0 + px < p.M) *(bf16x4v*)(p.y + (size_t)(m0 + px) * CO + ch) = o;
      }
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  // ---- phase 2: z[ch][px] = relu(W1 . y + b1), y read from LDS
  f32x4 acc[CMW][PF];
#pragma unroll
  for (int j = 0; j < CMW; ++j)
#pragma unroll
    for (int i = 0; i < PF; ++i) acc[j][i] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < KS2; ++ks) {
#pragma unroll
    for (int i = 0; i < PF; ++i) {
      const bf16x8 a = *(const bf16x8*)(ys + pswz<YCH>(i * 16 + fr, ks * 4 + fq));
#pragma unroll
      for (int j = 0; j < CMW; ++j) acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wz[j][ks], a, acc[j][i], 0, 0, 0);
    }
  }
#pragma unroll
  for (int j = 0; j < CMW; ++j) {
    const int ch = (nz0 + j) * 16 + fq * 4;
#pragma unroll
    for (int i = 0; i < PF; ++i) {
      const int m = m0 + i * 16 + fr;
      bf16x4v o;
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = f2bf(fmaxf(acc[j][i][r] + bz[j][r], 0.f));
      if (m < p.M) *(bf16x4v*)(p.z + (size_t)m * CM + ch) = o;
    }
  }
}

// (CIN, CO, CM, BM, NWV) instances: ResNet stage 3 (28x28: 128 -> 512 -> 128).
// Stage 4 (256 -> 1024 -> 256) would hold 64 W1 fragments per wave for phase 2
// and spills; it stays on the two-launch path.
#define ADAPT_PAIR_CFGS(X) \
  X(128, 512, 128, 112, 8) \
  X(128, 512, 128, 64, 8)

bool pw_pair_supported(int cin, int co, int cm, int bm) {
#define X(CI, CO_, CM_, BM_, NW_) if (cin == CI && co == CO_ && cm == CM_ && bm == BM_) return true;
  ADAPT_PAIR_CFGS(X)
#undef X
  return false;
}

hipError_t pw_pair_forward(const PwPairParams& p, int cin, int co, int cm, int bm, hipStream_t s) {
#define X(CI, CO_, CM_, BM_, NW_)                                                                     \
  if (cin == CI && co == CO_ && cm == CM_ && bm == BM_) {                                            \
    hipLaunchKernelGGL((pw_pair_kernel<CI, CO_, CM_, BM_, NW_>), dim3((p.M + BM_ - 1) / BM_), dim3(NW_ * 64), 0, s, p); \
    return hipGetLastError();                                                                        \
  }
  ADAPT_PAIR_CFGS(X)
#undef X
  return hipErrorInvalidValue;
}

}  // namespace adapt
