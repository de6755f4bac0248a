// Channel-sliced persistent pointwise (1x1, stride 1) bf16 conv with the fused bias + residual + ReLU
// epilogue:  out[m][n] = act(x[m] . W[n] + b[n] (+ res[m][n])), for the wide-K / wide-N 1x1s of ResNet
// stages 3-5 (K = 128 -> N = 512 + residual, K = 256 -> N = 1024 + residual, K = 1024 -> N = 256,
// K = 512 -> N = 2048 + residual).
//
// Those layers are memory-bound at bs=32 (stage-4 `_out`: 3.2 MB in, 12.8 MB residual, 12.8 MB out against
// 3.3 GFLOP), yet the tuned LDS-DMA tile GEMM runs them at ~3 TB/s (9.7 us,
// profiles/r5/roofline_r50_bf16_bs32_v4.txt): 196 one-shot blocks, each a dependent chain of prologue loads,
// four K chunks and a residual / store epilogue, one block per CU.  pw_wide.hip (stage 3) streams instead,
// but every block holds all N output channels' weights in VGPRs, which caps it at K x N = 64 K.
//
// Here a block owns a SLICE of NS = WAVES x CF x 16 output channels and walks pixel tiles:
// * the slice's weight fragments stay in VGPRs for the launch (CF x K / 32 fragments per wave, <= 128 VGPRs);
// * grid = walkers x slices, XCD-ordered so the slices of one walker (the blocks that read the same
//   activation tiles) run on one XCD and share its L2;
// * the next tile's activation rows (PT x K) and residual row segments (PT x NS) are loaded into registers
//   under the current tile's MFMAs, staged to the other LDS buffer after the epilogue (pw_wide's pipeline);
// * the GEMM runs transposed (weight fragment = A operand), so a lane's accumulator holds four consecutive
//   channels of one pixel: the epilogue reads its residual and writes its output as 8-byte LDS accesses in
//   place, and the tile leaves as 16-byte row-contiguous segment stores.
#include "kernels.h"

namespace adapt {

namespace {

typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

// byte offset of 16-byte chunk c of LDS row r (NCH chunks a row), XOR-swizzled by the row's low bits so the
// 16 rows of a fragment read at one logical chunk hit distinct banks
template <int NCH>
__device__ __forceinline__ int ps_sw(int r, int c) {
  constexpr int MASK = (NCH < 16 ? NCH : 16) - 1;
  return r * (NCH * 16) + ((c ^ (r & MASK)) << 4);
}

// LDS-only barrier: the tile's global stores and the next tile's loads stay in flight across it
__device__ __forceinline__ void ps_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int K, int CF, int WAVES, int PT>
__global__ __launch_bounds__(WAVES * 64, 1) void pw_slice_kernel(PwParams p, int N, int slices) {
  constexpr int NT = WAVES * 64;
  constexpr int NS = WAVES * CF * 16;        // output channels of a slice
  constexpr int KS = K / 32;                 // MFMA k-steps
  constexpr int XCH = K / 8;                 // 16-byte chunks per activation row
  constexpr int OCH = NS / 8;                // 16-byte chunks per residual / output row segment
  constexpr int PF = PT / 16;                // pixel fragments per tile
  constexpr int AB = PT * K * 2;             // bytes of one activation tile
  constexpr int RB = PT * NS * 2;            // bytes of one residual / output tile
  constexpr int XIT = (PT * XCH + NT - 1) / NT;
  constexpr int RIT = (PT * OCH + NT - 1) / NT;
  static_assert(CF * KS * 4 <= 128, "weight fragments must fit 128 VGPRs");
  static_assert(PT % 16 == 0 && 2 * (AB + RB) <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[2 * AB + 2 * RB];
  char* const abuf = smem;
  char* const rbuf = smem + 2 * AB;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int ntiles = (p.M + PT - 1) / PT;
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int slice = logical % slices;
  const int walker = logical / slices;
  const int walkers = gridDim.x / slices;    // host: gridDim.x is a multiple of slices
  const int n0 = slice * NS;
  if (walker >= ntiles) return;

  // this wave's weight fragments (CF channel fragments x KS k-steps), resident for the launch
  const bf16x8* wf = (const bf16x8*)p.w;
  const int cf0 = (n0 >> 4) + wave * CF;     // first 16-channel fragment of this wave
  bf16x8 wr[CF][KS];
#pragma unroll
  for (int cf = 0; cf < CF; ++cf)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) wr[cf][ks] = wf[((cf0 + cf) * KS + ks) * 64 + lane];
  f32x4 bias[CF];
#pragma unroll
  for (int cf = 0; cf < CF; ++cf) {
    const int n = (cf0 + cf) * 16 + fq * 4;
    bias[cf] = p.bias ? *(const f32x4*)(p.bias + n) : (f32x4){0.f, 0.f, 0.f, 0.f};
  }

  // next tile's activation rows and residual row segments: 16-byte, row-contiguous loads into registers
  u32x4 ra[XIT], rres[RIT];
  auto load_next = [&](int t) __attribute__((always_inline)) {
#pragma unroll
    for (int it = 0; it < XIT; ++it) {
      const int i = tid + it * NT;
      const int px = i / XCH, c = i - px * XCH;
      const int m = t * PT + px;
      ra[it] = (i < PT * XCH && m < p.M) ? *(const u32x4*)(p.x + (size_t)m * K + c * 8) : (u32x4){0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int it = 0; it < RIT; ++it) {
      const int i = tid + it * NT;
      const int px = i / OCH, c = i - px * OCH;
      const int m = t * PT + px;
      rres[it] = (p.res && i < PT * OCH && m < p.M) ? *(const u32x4*)(p.res + (size_t)m * N + n0 + c * 8)
                                                     : (u32x4){0u, 0u, 0u, 0u};
    }
  };
  auto stage_next = [&](int b) __attribute__((always_inline)) {
#pragma unroll
    for (int it = 0; it < XIT; ++it) {
      const int i = tid + it * NT;
      if (i < PT * XCH) *(u32x4*)(abuf + b * AB + ps_sw<XCH>(i / XCH, i % XCH)) = ra[it];
    }
#pragma unroll
    for (int it = 0; it < RIT; ++it) {
      const int i = tid + it * NT;
      if (i < PT * OCH) *(u32x4*)(rbuf + b * RB + ps_sw<OCH>(i / OCH, i % OCH)) = rres[it];
    }
  };

  int t = walker;
  load_next(t);
  stage_next(0);
  ps_barrier();
  int buf = 0;
  for (; t < ntiles; t += walkers) {
    const int tn = t + walkers;
    const bool more = tn < ntiles;
    const int m0 = t * PT;
    if (more) load_next(tn);                 // in flight under this tile's MFMAs and epilogue
    const char* a = abuf + buf * AB;
    char* r = rbuf + buf * RB;
    f32x4 acc[CF][PF];
#pragma unroll
    for (int cf = 0; cf < CF; ++cf)
#pragma unroll
      for (int pf = 0; pf < PF; ++pf) acc[cf][pf] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int pf = 0; pf < PF; ++pf) {
        const bf16x8 af = *(const bf16x8*)(a + ps_sw<XCH>(pf * 16 + fr, ks * 4 + fq));
#pragma unroll
        for (int cf = 0; cf < CF; ++cf)
          acc[cf][pf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wr[cf][ks], af, acc[cf][pf], 0, 0, 0);
      }
    // epilogue in LDS: each lane reads its residual (4 channels of one pixel) and overwrites the same 8 bytes
    // with its output (zeros were staged when there is no residual)
#pragma unroll
    for (int pf = 0; pf < PF; ++pf)
#pragma unroll
      for (int cf = 0; cf < CF; ++cf) {
        const int nl = (wave * CF + cf) * 16 + fq * 4;   // channel within the slice
        char* q = r + ps_sw<OCH>(pf * 16 + fr, nl >> 3) + (nl & 7) * 2;
        const bf16x4 res = *(const bf16x4*)q;
        bf16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = f2bf(act_relu(acc[cf][pf][e] + bias[cf][e] + bf2f(res[e]), p.relu));
        *(bf16x4*)q = o;
      }
    ps_barrier();
    // the tile's output row segments, 16 bytes per lane, row-contiguous
#pragma unroll
    for (int it = 0; it < RIT; ++it) {
      const int i = tid + it * NT;
      const int px = i / OCH, c = i - px * OCH;
      const int m = m0 + px;
      if (i < PT * OCH && m < p.M) *(u32x4*)(p.out + (size_t)m * N + n0 + c * 8) = *(const u32x4*)(r + ps_sw<OCH>(px, c));
    }
    if (more) stage_next(buf ^ 1);
    ps_barrier();
    buf ^= 1;
  }
}

}  // namespace

// config code -> (CF, WAVES, PT); the K instantiations a code supports follow from CF x K <= 1024
bool pw_slice_cfg(int code, int* cf, int* waves, int* pt) {
  switch (code) {
    case 0: *cf = 4; *waves = 8; *pt = 16; return true;
    case 1: *cf = 2; *waves = 8; *pt = 16; return true;
    case 2: *cf = 1; *waves = 8; *pt = 16; return true;
    case 3: *cf = 2; *waves = 4; *pt = 32; return true;
    case 4: *cf = 1; *waves = 4; *pt = 32; return true;
    case 5: *cf = 4; *waves = 4; *pt = 16; return true;
    default: return false;
  }
}

int pw_slice_supported(int K, int N, int code) {
  int cf, waves, pt;
  if (!pw_slice_cfg(code, &cf, &waves, &pt)) return 0;
  if (K != 128 && K != 256 && K != 512 && K != 1024) return 0;
  if (cf * K > 1024) return 0;
  const int ns = cf * waves * 16;
  return N % ns == 0 && N / ns <= 256;
}

hipError_t pw_slice_forward(const PwParams& p, int K, int N, int code, int blocks, hipStream_t s) {
  if (!pw_slice_supported(K, N, code) || p.M < 1 || blocks < 1) return hipErrorInvalidValue;
  int cf, waves, pt;
  pw_slice_cfg(code, &cf, &waves, &pt);
  const int slices = N / (cf * waves * 16);
  const int ntiles = (p.M + pt - 1) / pt;
  int walkers = blocks / slices;
  if (walkers < 1) walkers = 1;
  if (walkers > ntiles) walkers = ntiles;
  const dim3 grid(walkers * slices);
#define PS_LAUNCH(KK, CC, WW, PP) \
  hipLaunchKernelGGL(HIP_KERNEL_NAME(pw_slice_kernel<KK, CC, WW, PP>), grid, dim3(WW * 64), 0, s, p, N, slices)
#define PS_CODE(KK)                          \
  switch (code) {                            \
    case 0: PS_LAUNCH(KK, 4, 8, 16); break;  \
    case 1: PS_LAUNCH(KK, 2, 8, 16); break;  \
    case 2: PS_LAUNCH(KK, 1, 8, 16); break;  \
    case 3: PS_LAUNCH(KK, 2, 4, 32); break;  \
    case 4: PS_LAUNCH(KK, 1, 4, 32); break;  \
    case 5: PS_LAUNCH(KK, 4, 4, 16); break;  \
  }
  if (K == 128) {
    PS_CODE(128)
  } else if (K == 256) {
    PS_CODE(256)
  } else if (K == 512) {
    switch (code) {
      case 1: PS_LAUNCH(512, 2, 8, 16); break;
      case 2: PS_LAUNCH(512, 1, 8, 16); break;
      case 3: PS_LAUNCH(512, 2, 4, 32); break;
      case 4: PS_LAUNCH(512, 1, 4, 32); break;
    }
  } else {
    switch (code) {
      case 2: PS_LAUNCH(1024, 1, 8, 16); break;
      case 4: PS_LAUNCH(1024, 1, 4, 32); break;
    }
  }
#undef PS_CODE
#undef PS_LAUNCH
  return hipGetLastError();
}

}  // namespace adapt
