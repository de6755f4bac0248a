// 3x3 / stride-1 / pad-1 convolution with register-resident weights (gfx950
// MFMA), for ResNet stage 3 (28x28, 128 -> 128 channels, BN folded, ReLU).
//
// The implicit-GEMM kernels (conv_glds.hip) stream the weights through LDS per
// K tile: for this layer two thirds of their LDS-DMA bytes are weights, and the
// fragment reads of both operands serialise with the MFMAs
// (profiles/r2/roofline/conv_ablate_v2.txt).  Here the whole filter (128 x 1152
// bf16 = 295 KB) lives in the VGPRs of one block: wave w holds output channels
// 16w .. 16w+15 for all 36 k-steps (36 fragments, 144 VGPRs) for the whole
// launch.  A block owns TR whole output rows of one image; their (TR+2) x (W+2)
// input halo is staged in LDS once (zero outside the image), and each tap reads
// a shifted window of it as the MFMA B operand.  So the only per-k-step LDS
// traffic is the activation fragment, and HBM sees the input once (+ halo rows)
// and the output once.
//
// GEMM transposed as in pw_wide.hip / pw_pair.hip (A = weight fragment from
// registers, B = activation fragment from LDS, D = [channel][pixel]); the output
// tile is staged through LDS (over the dead halo) and leaves with 16-byte
// row-contiguous stores.  K order k = (kh, kw, ci) is PackedConv's, fragment-
// packed by ops/conv.py `pw_fragments`.
#include "kernels.h"

namespace adapt {

namespace {

typedef __bf16 bf16x4v __attribute__((ext_vector_type(4)));

// 16-byte chunk c of a 256-byte pixel row r.  The 16 pixels of a B fragment are
// consecutive output pixels, which wrap from one 28-wide output row to the next
// inside the 30-wide halo, and the taps shift them by 0..2 columns: a plain
// c ^ (r & 15) leaves 624 extra LDS cycles per tile in the ds_read_b128 lane
// groups; the rotation (c + 10 r) mod 16 was the best of an exhaustive search
// over affine swizzles (432).
__device__ __forceinline__ int rswz(int r, int c) {
  return r * 256 + (((c + 10 * r) & 15) << 4);
}

}  // namespace

// KG > 1: KG groups of C/16 waves split the k-steps (fewer resident fragments per
// wave, KG times the waves per CU for latency hiding); the groups' partial sums
// meet in an fp32 LDS buffer before the epilogue.
template <int C, int H, int W, int TR, int KG = 1>
__global__ __launch_bounds__(C / 16 * KG * 64, 1) void conv3x3_rr_kernel(Conv3x3RRParams p) {
  constexpr int NCF = C / 16, NWV = NCF * KG, NT = NWV * 64;
  constexpr int KSA = 9 * C / 32;                // k-steps of the filter (36 for C = 128)
  constexpr int KS = KSA / KG;                   // k-steps per wave
  static_assert(KSA % KG == 0, "K groups");
  constexpr int CCH = C / 8;                     // 16-byte chunks per pixel
  constexpr int HW2 = W + 2, HP = (TR + 2) * HW2;
  constexpr int PX = TR * W, PF = (PX + 15) / 16;
  constexpr int HIT = (HP * CCH + NT - 1) / NT;
  constexpr int OIT = (PX * CCH + NT - 1) / NT;
  static_assert(C == 128 && CCH == 16, "rswz assumes 256-byte pixel rows");
  static_assert(H % TR == 0 && HP * C * 2 <= 160 * 1024 && PF * 16 * C * 2 <= HP * C * 2, "tile");
  constexpr int RED = KG > 1 ? PX * C * 4 : 0;   // fp32 partial sums of the other K groups
  __shared__ __attribute__((aligned(16))) char halo[HP * C * 2 + RED];
  static_assert(HP * C * 2 + RED <= 160 * 1024, "LDS");

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int cf = wave % NCF, kg = wave / NCF;    // channel fragment, K group
  const int tiles = p.B * (H / TR);
  const int t = xcd_remap(blockIdx.x, tiles);
  const int img = t / (H / TR), oh0 = (t % (H / TR)) * TR;

  // halo rows oh0-1 .. oh0+TR, cols -1 .. W -> registers (zero outside the image)
  u32x4 hr[HIT];
#pragma unroll
  for (int it = 0; it < HIT; ++it) {
    const int i = tid + it * NT;
    const int hp = i / CCH, c = i - hp * CCH;
    const int ih = oh0 - 1 + hp / HW2, iw = hp % HW2 - 1;
    const bool in = i < HP * CCH && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
    hr[it] = in ? *(const u32x4*)(p.x + (((size_t)img * H + ih) * W + iw) * C + c * 8) : (u32x4){0u, 0u, 0u, 0u};
  }
  // this wave's 16 output channels: all k-steps of the filter, resident for the launch
  const bf16x8* wf = (const bf16x8*)p.wfrag;
  bf16x8 wr[KS];
#pragma unroll
  for (int k = 0; k < KS; ++k) wr[k] = wf[(cf * KSA + kg * KS + k) * 64 + lane];
  const f32x4 bias = *(const f32x4*)(p.bias + cf * 16 + fq * 4);
#pragma unroll
  for (int it = 0; it < HIT; ++it) {
    const int i = tid + it * NT;
    if (i < HP * CCH) *(u32x4*)(halo + rswz(i / CCH, i % CCH)) = hr[it];
  }
  __syncthreads();

  // per-lane halo index of each pixel fragment's top-left tap
  int hb[PF];
#pragma unroll
  for (int f = 0; f < PF; ++f) {
    const int px = min(f * 16 + fr, PX - 1);
    hb[f] = (px / W) * HW2 + px % W;
  }
  f32x4 acc[PF];
#pragma unroll
  for (int f = 0; f < PF; ++f) acc[f] = (f32x4){0.f, 0.f, 0.f, 0.f};
  if constexpr (KG == 1) {
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int toff = (tap / 3) * HW2 + tap % 3;
#pragma unroll
      for (int cc = 0; cc < C / 32; ++cc) {
#pragma unroll
        for (int f = 0; f < PF; ++f) {
          const bf16x8 a = *(const bf16x8*)(halo + rswz(hb[f] + toff, cc * 4 + fq));
          acc[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wr[tap * (C / 32) + cc], a, acc[f], 0, 0, 0);
        }
      }
    }
  } else {
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      const int ks = kg * KS + k, tap = ks / (C / 32), cc = ks % (C / 32);   // wave-uniform
      const int toff = (tap / 3) * HW2 + tap % 3;
#pragma unroll
      for (int f = 0; f < PF; ++f) {
        const bf16x8 a = *(const bf16x8*)(halo + rswz(hb[f] + toff, cc * 4 + fq));
        acc[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wr[k], a, acc[f], 0, 0, 0);
      }
    }
    // K groups 1.. park their partial sums (fp32, [pixel][channel]) past the halo
    float* red = (float*)(halo + HP * C * 2);
    const int chr = cf * 16 + fq * 4;
    for (int g = 1; g < KG; ++g) {
      if (kg == g) {
#pragma unroll
        for (int f = 0; f < PF; ++f) {
          const int px = f * 16 + fr;
          if (px < PX) {
            f32x4* q = (f32x4*)(red + px * C + chr);
            *q = g == 1 ? acc[f] : *q + acc[f];
          }
        }
      }
      __syncthreads();
    }
    if (kg == 0) {
#pragma unroll
      for (int f = 0; f < PF; ++f) {
        const int px = f * 16 + fr;
        if (px < PX) acc[f] += *(const f32x4*)(red + px * C + chr);
      }
    }
  }
  __syncthreads();                               // every halo read done: stage the output tile over it
  const int ch = cf * 16 + fq * 4;
#pragma unroll
  for (int f = 0; f < PF; ++f) {
    const int px = f * 16 + fr;
    if (kg == 0 && px < PX) {
      bf16x4v o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = f2bf(p.relu ? fmaxf(acc[f][e] + bias[e], 0.f) : acc[f][e] + bias[e]);
      *(bf16x4v*)(halo + rswz(px, ch >> 3) + (ch & 4) * 2) = o;
    }
  }
  __syncthreads();
  bf16* out = p.out + ((size_t)img * H + oh0) * W * C;
#pragma unroll
  for (int it = 0; it < OIT; ++it) {
    const int i = tid + it * NT;
    if (i < PX * CCH) *(u32x4*)(out + (size_t)(i / CCH) * C + (i % CCH) * 8) = *(const u32x4*)(halo + rswz(i / CCH, i % CCH));
  }
}

bool conv3x3_rr_supported(int C, int H, int W) { return C == 128 && H == 28 && W == 28; }

hipError_t conv3x3_rr_forward(const Conv3x3RRParams& p, int C, int H, int W, int kg, hipStream_t s) {
  if (!conv3x3_rr_supported(C, H, W) || p.B < 1) return hipErrorInvalidValue;
  constexpr int TR = 4;
  if (kg == 2) hipLaunchKernelGGL((conv3x3_rr_kernel<128, 28, 28, TR, 2>), dim3(p.B * (28 / TR)), dim3(1024), 0, s, p);
  else if (kg == 1) hipLaunchKernelGGL((conv3x3_rr_kernel<128, 28, 28, TR, 1>), dim3(p.B * (28 / TR)), dim3(512), 0, s, p);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace adapt
