// Persistent pointwise (1x1, stride 1) conv for short K and wide N, with the
// fused bias + residual + ReLU epilogue:  out[m][n] = act(x[m] . W[n] + b[n] (+ res[m][n]))
//
// ResNet stage 3's "_out" convs (K = 128 -> N = 512, + the block input) run
// memory-bound: 25.7 MB of residual in and 25.7 MB out per bs=32 launch against
// 3.3 GFLOP.  The implicit-GEMM tiles (conv_igemm / conv_glds) re-read the
// weights per tile and stage them through LDS; here every wave keeps its 64
// output channels' weight fragments in registers for the whole launch (K = 128:
// 64 VGPRs), and a persistent block walks pixel tiles, so only activations,
// residual and output stream:
//   * the next tile's activation and residual rows are loaded into registers
//     under the current tile's MFMAs and go to the other LDS buffer afterwards;
//   * the residual rows come in with the activation rows (16-byte, row-
//     contiguous loads) and go to LDS; the GEMM runs transposed (weight
//     fragment = A operand), so a lane's accumulator holds four consecutive
//     channels of one pixel and the epilogue reads its residual and writes its
//     output as 8-byte LDS accesses in place; the output rows then leave with
//     16-byte row-contiguous stores.  (A first version with 8-byte global
//     residual loads / output stores straight from the accumulators touched 16
//     cache lines per instruction and ran 18.1 us against 16.0 us for the tuned
//     implicit-GEMM tile.)
// Waves = N / 64 (8 for N = 512); PT output pixels per tile.
#include "kernels.h"

namespace adapt {

namespace {

typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

// byte offset of 16-byte chunk c of LDS row r (rows of NCH chunks), the chunk XOR-swizzled
// by the row's low bits so 16 consecutive rows read at one logical chunk hit distinct banks
template <int NCH>
__device__ __forceinline__ int pw_sw(int r, int c) {
  constexpr int MASK = (NCH < 16 ? NCH : 16) - 1;
  return r * (NCH * 16) + ((c ^ (r & MASK)) << 4);
}

template <int K, int N, int PT>
__global__ __launch_bounds__(N, 1) void pw_res_kernel(PwParams p) {
  constexpr int KS = K / 32;                 // MFMA k-steps
  constexpr int XCH = K / 8;                 // 16-byte chunks per activation row
  constexpr int OCH = N / 8;                 // 16-byte chunks per residual / output row
  constexpr int PF = PT / 16;                // pixel fragments per tile
  constexpr int AB = PT * K * 2;             // bytes of one activation tile
  constexpr int RB = PT * N * 2;             // bytes of one residual / output tile
  constexpr int XIT = (PT * XCH + N - 1) / N;
  constexpr int RIT = PT * OCH / N;
  static_assert(K % 32 == 0 && N % 64 == 0 && PT % 16 == 0 && XCH <= 16 && (PT * OCH) % N == 0, "shape");
  __shared__ __attribute__((aligned(16))) char smem[2 * AB + 2 * RB];
  char* const abuf = smem;
  char* const rbuf = smem + 2 * AB;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int ntiles = (p.M + PT - 1) / PT;
  if ((int)blockIdx.x >= ntiles) return;

  // this wave's weight fragments (4 channel fragments x KS k-steps), resident for the launch
  const bf16x8* wf = (const bf16x8*)p.w;
  bf16x8 wr[4][KS];
#pragma unroll
  for (int cf = 0; cf < 4; ++cf)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) wr[cf][ks] = wf[((wave * 4 + cf) * KS + ks) * 64 + lane];
  f32x4 bias[4];
#pragma unroll
  for (int cf = 0; cf < 4; ++cf) {
    const int n = wave * 64 + cf * 16 + fq * 4;
    bias[cf] = p.bias ? *(const f32x4*)(p.bias + n) : (f32x4){0.f, 0.f, 0.f, 0.f};
  }

  // next tile's activation and residual rows: 16-byte, row-contiguous loads into registers
  // (one tile ahead; a two-deep register ring measured slower: 15.7 vs 14.5 us)
  u32x4 ra[XIT], rres[RIT];
  auto load_next = [&](int t) __attribute__((always_inline)) {
#pragma unroll
    for (int it = 0; it < XIT; ++it) {
      const int i = tid + it * N;
      const int px = i / XCH, c = i - px * XCH;
      const int m = t * PT + px;
      ra[it] = (i < PT * XCH && m < p.M) ? *(const u32x4*)(p.x + (size_t)m * K + c * 8) : (u32x4){0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int it = 0; it < RIT; ++it) {
      const int i = tid + it * N;
      const int px = i / OCH, c = i - px * OCH;
      const int m = t * PT + px;
      rres[it] = (p.res && m < p.M) ? *(const u32x4*)(p.res + (size_t)m * N + c * 8) : (u32x4){0u, 0u, 0u, 0u};
    }
  };
  auto stage_next = [&](int b) __attribute__((always_inline)) {
#pragma unroll
    for (int it = 0; it < XIT; ++it) {
      const int i = tid + it * N;
      if (i < PT * XCH) *(u32x4*)(abuf + b * AB + pw_sw<XCH>(i / XCH, i % XCH)) = ra[it];
    }
#pragma unroll
    for (int it = 0; it < RIT; ++it) {
      const int i = tid + it * N;
      *(u32x4*)(rbuf + b * RB + pw_sw<OCH>(i / OCH, i % OCH)) = rres[it];
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
    const int m0 = t * PT;
    if (more) load_next(tn);                 // in flight under this tile's MFMAs and epilogue
    const char* a = abuf + buf * AB;
    char* r = rbuf + buf * RB;
    f32x4 acc[4][PF];
#pragma unroll
    for (int cf = 0; cf < 4; ++cf)
#pragma unroll
      for (int pf = 0; pf < PF; ++pf) acc[cf][pf] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int pf = 0; pf < PF; ++pf) {
        const bf16x8 af = *(const bf16x8*)(a + pw_sw<XCH>(pf * 16 + fr, ks * 4 + fq));
#pragma unroll
        for (int cf = 0; cf < 4; ++cf)
          acc[cf][pf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wr[cf][ks], af, acc[cf][pf], 0, 0, 0);
      }
    // epilogue in LDS: each lane reads its residual (4 channels of one pixel) and
    // overwrites the same 8 bytes with its output
#pragma unroll
    for (int pf = 0; pf < PF; ++pf)
#pragma unroll
      for (int cf = 0; cf < 4; ++cf) {
        const int n = wave * 64 + cf * 16 + fq * 4;
        char* q = r + pw_sw<OCH>(pf * 16 + fr, n >> 3) + (n & 7) * 2;
        const bf16x4 res = *(const bf16x4*)q;
        bf16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = f2bf(act_relu(acc[cf][pf][e] + bias[cf][e] + bf2f(res[e]), p.relu));
        *(bf16x4*)q = o;
      }
    __syncthreads();
    // the tile's output rows, 16 bytes per lane, row-contiguous
#pragma unroll
    for (int it = 0; it < RIT; ++it) {
      const int i = tid + it * N;
      const int px = i / OCH, c = i - px * OCH;
      const int m = m0 + px;
      if (m < p.M) *(u32x4*)(p.out + (size_t)m * N + c * 8) = *(const u32x4*)(r + pw_sw<OCH>(px, c));
    }
    if (more) stage_next(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
}

}  // namespace

int pw_res_supported(int K, int N) { return (K == 128 && N == 512) || (K == 64 && N == 256); }

hipError_t pw_res_forward(const PwParams& p, int K, int N, int pt, int blocks, hipStream_t s) {
  if (!pw_res_supported(K, N) || p.M < 1 || (pt != 16 && pt != 32)) return hipErrorInvalidValue;
  const int ntiles = (p.M + pt - 1) / pt;
  const dim3 grid(blocks > 0 && blocks < ntiles ? blocks : ntiles);
#define PW_LAUNCH(KK, NN, PP) hipLaunchKernelGGL((pw_res_kernel<KK, NN, PP>), grid, dim3(NN), 0, s, p)
  // (64-pixel tiles would need more than the 256 VGPRs a wave of an N-thread block gets: they spilled)
  if (K == 128) {
    if (pt == 16) PW_LAUNCH(128, 512, 16);
    else PW_LAUNCH(128, 512, 32);
  } else {
    if (pt == 16) PW_LAUNCH(64, 256, 16);
    else PW_LAUNCH(64, 256, 32);
  }
#undef PW_LAUNCH
  return hipGetLastError();
}

}  // namespace adapt
