// 3x3 / stride-1 / pad-1 bf16 convolution with a channel SLICE of the filter
// resident in VGPRs, for ResNet stages 4 (14x14, 256 -> 256) and 5 (7x7,
// 512 -> 512), BN folded, ReLU.
//
// conv3x3_rr.hip keeps a whole filter in one block's registers, which only
// fits stage 3 (295 KB); stage 4's filter is 1.18 MB and stage 5's 4.7 MB, so
// those layers ran on the LDS-DMA tiles at 5.8x / 7.5x their roofline floor
// (17 / 22 us at bs=32, profiles/r2/roofline/roofline_r50_bs32_final.txt).
// Here a block owns NCF x 16 output channels (its slice of the filter, 295 KB:
// the stage-3 footprint) and KG K-groups of NCF waves split the 9*C/32 k-steps,
// 36 resident fragments (144 VGPRs) per wave.  The grid is slices x pixel
// tiles; a block walks its tiles persistently, so the weights cross L2 -> VGPR
// once per block, and each tile's (TR+2) x (W+2) input halo is staged in LDS
// and read as shifted windows for the 9 taps (the only per-k-step LDS traffic
// is the activation fragment).
//
// Halo pixel rows are C*2 bytes on a PITCH-pixel grid; the low four bits of the
// 16-byte chunk index rotate by (SA*r + SB*(r >> SSH)) so the 16 consecutive
// pixels of a B fragment (which wrap from one output row to the next inside the
// halo) hit distinct bank slots in every ds_read_b128 lane group: zero extra
// LDS cycles for both shapes (tools/cs3x3_swizzle_search.py; 12.4k extra cycles
// per tile unswizzled).
//
// GEMM transposed (A = weight fragment from registers, B = activation fragment
// from LDS, D = [channel][pixel]).  The K-groups' partial sums meet in fp32 in
// the dead halo; the output tile is staged over it and leaves with 16-byte
// stores (a slice is CS * 2 contiguous bytes of each output pixel).
#include "kernels.h"

namespace adapt {

namespace {

template <int C, int SA, int SB, int SSH>
__device__ __forceinline__ int cs_off(int r, int c) {
  return r * (C * 2) + (((c & ~15) | ((c + SA * r + SB * (r >> SSH)) & 15)) << 4);
}

}  // namespace

template <int C, int H, int W, int TR, int NCF, int KG, int PITCH, int SA, int SB, int SSH, int TPB, int HB>
__global__ __launch_bounds__(NCF * KG * 64, 1) void conv3x3_cs_kernel(Conv3x3RRParams p) {
  constexpr int NW = NCF * KG, NT = NW * 64;
  constexpr int CS = NCF * 16;                   // output channels per block
  constexpr int KSA = 9 * C / 32;                // k-steps of the filter
  constexpr int KS = KSA / KG;                   // resident k-steps per wave
  constexpr int CPT = C / 32;                    // k-steps per tap
  constexpr int CCH = C / 8;                     // 16-byte chunks per pixel
  constexpr int HR = TR + 2, HP = HR * PITCH;
  constexpr int PX = TR * W, PF = (PX + 15) / 16;
  constexpr int HIT = (HR * (W + 2) * CCH + NT - 1) / NT;
  constexpr int OCH = CS / 8;                    // 16-byte output chunks per pixel
  constexpr int OIT = (PX * OCH + NT - 1) / NT;
  static_assert(KSA % KG == 0 && H % TR == 0 && PITCH >= W + 2, "shape");
  static_assert(HP * C * 2 <= 160 * 1024, "halo");
  static_assert(PX * CS * 4 <= HP * C * 2, "partials fit in the dead halo");
  __shared__ __attribute__((aligned(16))) char halo[HP * C * 2];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int cf = wave % NCF, kg = wave / NCF;
  constexpr int RB = H / TR;                     // row blocks per image
  const int tiles_per_slice = p.B * RB;
  const int groups = (tiles_per_slice + TPB - 1) / TPB;   // blocks per slice
  // slice-major: a slice's blocks are consecutive logical ids -> the same XCD (shared weights in its L2)
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int slice = logical / groups, grp = logical - slice * groups;

  // this wave's 16 output channels of the slice, its K-group's k-steps: resident for the launch
  const bf16x8* wf = (const bf16x8*)p.wfrag;
  const int cfg_ = slice * NCF + cf;             // global channel fragment
  bf16x8 wr[KS];
#pragma unroll
  for (int k = 0; k < KS; ++k) wr[k] = wf[(cfg_ * KSA + kg * KS + k) * 64 + lane];
  const f32x4 bias = *(const f32x4*)(p.bias + cfg_ * 16 + fq * 4);

  int hb[PF];
#pragma unroll
  for (int f = 0; f < PF; ++f) {
    const int px = min(f * 16 + fr, PX - 1);
    hb[f] = (px / W) * PITCH + px % W;
  }

  for (int tt = 0; tt < TPB; ++tt) {
    const int t = grp * TPB + tt;
    if (t >= tiles_per_slice) break;             // block-uniform
    const int img = t / RB, oh0 = (t % RB) * TR;
    // the per-(fragment, tap, chunk) LDS addresses are tile-invariant; without this the
    // compiler hoists all of them out of the tile loop and spills the resident weights
#pragma unroll
    for (int f = 0; f < PF; ++f) asm volatile("" : "+v"(hb[f]));
    if (tt > 0) __syncthreads();                 // the previous tile's output reads of the halo are done
    // halo rows oh0-1 .. oh0+TR, cols -1 .. W -> LDS (zero outside the image); loads are
    // issued in batches of HB before their stores so the round trips overlap (HB bounds
    // the staging registers next to the 144 resident weight VGPRs)
#pragma unroll
    for (int b0 = 0; b0 < HIT; b0 += HB) {
      u32x4 hv[HB];
#pragma unroll
      for (int j = 0; j < HB; ++j) {
        const int i = tid + (b0 + j) * NT;
        const int hp = i / CCH, c = i - hp * CCH;
        const int hr = hp / (W + 2), hc = hp - hr * (W + 2);
        const int ih = oh0 - 1 + hr, iw = hc - 1;
        const bool in = b0 + j < HIT && i < HR * (W + 2) * CCH && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
        hv[j] = in ? *(const u32x4*)(p.x + (((size_t)img * H + ih) * W + iw) * C + c * 8) : (u32x4){0u, 0u, 0u, 0u};
      }
#pragma unroll
      for (int j = 0; j < HB; ++j) {
        const int i = tid + (b0 + j) * NT;
        const int hp = i / CCH, c = i - hp * CCH;
        const int hr = hp / (W + 2), hc = hp - hr * (W + 2);
        if (b0 + j < HIT && i < HR * (W + 2) * CCH) *(u32x4*)(halo + cs_off<C, SA, SB, SSH>(hr * PITCH + hc, c)) = hv[j];
      }
    }
    __syncthreads();

    f32x4 acc[PF];
#pragma unroll
    for (int f = 0; f < PF; ++f) acc[f] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      const int ks = kg * KS + k, tap = ks / CPT, cc = ks - tap * CPT;   // wave-uniform
      const int toff = (tap / 3) * PITCH + tap % 3;
#pragma unroll
      for (int f = 0; f < PF; ++f) {
        const bf16x8 a = *(const bf16x8*)(halo + cs_off<C, SA, SB, SSH>(hb[f] + toff, cc * 4 + fq));
        acc[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wr[k], a, acc[f], 0, 0, 0);
      }
    }
    __syncthreads();                             // every halo read done: partials / output over it
    const int chr = cf * 16 + fq * 4;            // this lane's 4 channels within the slice
    if constexpr (KG > 1) {
      float* red = (float*)halo;                 // [PX][CS] fp32
      for (int g = 1; g < KG; ++g) {
        if (kg == g) {
#pragma unroll
          for (int f = 0; f < PF; ++f) {
            const int px = f * 16 + fr;
            if (px < PX) {
              f32x4* q = (f32x4*)(red + px * CS + chr);
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
          if (px < PX) acc[f] += *(const f32x4*)(red + px * CS + chr);
        }
      }
      __syncthreads();                           // partials consumed: the bf16 output tile goes over them
    }
    bf16* ot = (bf16*)halo;                      // [PX][CS] bf16
    if (kg == 0) {
#pragma unroll
      for (int f = 0; f < PF; ++f) {
        const int px = f * 16 + fr;
        if (px < PX) {
          union { bf16 e[4]; uint2 u; } o;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float v = acc[f][e] + bias[e];
            o.e[e] = f2bf(p.relu ? fmaxf(v, 0.f) : v);
          }
          *(uint2*)(ot + px * CS + chr) = o.u;
        }
      }
    }
    __syncthreads();
    bf16* out = p.out + ((size_t)img * H + oh0) * W * C + slice * CS;
#pragma unroll
    for (int it = 0; it < OIT; ++it) {
      const int i = tid + it * NT;
      if (i < PX * OCH) {
        const int px = i / OCH, c = i - px * OCH;
        *(u32x4*)(out + (size_t)px * C + c * 8) = *(const u32x4*)(ot + px * CS + c * 8);
      }
    }
  }
}

bool conv3x3_cs_supported(int C, int H, int W) { return (C == 256 && H == 14 && W == 14) || (C == 512 && H == 7 && W == 7); }

// grid = (C / CS slices) x ceil(B * H/TR / TPB) blocks
hipError_t conv3x3_cs_forward(const Conv3x3RRParams& p, int C, int H, int W, hipStream_t s) {
  if (!conv3x3_cs_supported(C, H, W) || p.B < 1) return hipErrorInvalidValue;
  if (C == 256) {
    // stage 4: 4 slices of 64 channels x (32 images x 2 row blocks of 7 rows): 256 blocks, 8 waves
    constexpr int TR = 7, NCF = 4, KG = 2, TPB = 1;
    const int groups = (p.B * (14 / TR) + TPB - 1) / TPB;
    hipLaunchKernelGGL((conv3x3_cs_kernel<256, 14, 14, TR, NCF, KG, 16, 2, 12, 4, TPB, 9>), dim3((256 / (NCF * 16)) * groups),
                       dim3(NCF * KG * 64), 0, s, p);
  } else {
    // stage 5: 16 slices of 32 channels x 32 images: 512 blocks of 8 waves, one per CU at a time (147 KB LDS).
    // TPB = 2 (weights loaded once per 2 images) spills: the unrolled tile loop keeps its LDS addresses live
    constexpr int TR = 7, NCF = 2, KG = 4, TPB = 1;
    const int groups = (p.B + TPB - 1) / TPB;
    hipLaunchKernelGGL((conv3x3_cs_kernel<512, 7, 7, TR, NCF, KG, 16, 2, 14, 4, TPB, 6>), dim3((512 / (NCF * 16)) * groups),
                       dim3(NCF * KG * 64), 0, s, p);
  }
  return hipGetLastError();
}

}  // namespace adapt
