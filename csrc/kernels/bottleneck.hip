// Fused ResNet bottleneck block on MFMA (gfx950): one launch per block of
//
//   y1 = relu(conv1x1(x) + b1)                 CIN -> 64
//   y2 = relu(conv3x3(y1, pad 1) + b2)          64 -> 64
//   out = relu(conv1x1(y2) + b3 + shortcut)     64 -> 256
//   shortcut = x (identity, CIN = 256) or conv1x1(x) (projection, CIN = 64,
//              folded into the last GEMM as extra K: [y2 | x] . [W3 ; Wp])
//
// with BN folded into every conv on the host.  These are ResNet stage 2's
// three blocks (56x56, 256 channels): unfused they stream 51 MB tensors
// through HBM three times per block and run as memory-bound 1x1 GEMMs
// (profiles/r50_bs32_steps_v14.json: 56 us per block).  Here a workgroup owns
// an 8x8 output tile: it loads the 10x10 halo of x into LDS once, computes y1
// on the halo (zero outside the image: the 3x3's padding applies to y1), y2
// on the tile, and the block output, and writes only `out` back: one read of
// x and one write of out per block.
//
// MFMA v_mfma_f32_16x16x32_bf16; A fragments come from LDS (activations,
// 16-byte chunks XOR-swizzled per row so a fragment read is conflict-free),
// B fragments straight from global/L2 in a host-packed fragment order (one
// coalesced 1 KiB load per wave per fragment; every workgroup reads the same
// 136 KB of weights, which stay L2-resident).  Four waves:
//   GEMM1  wave w: channels 16w..16w+15, M = 100 halo px (7 frags), K = CIN
//   GEMM2  wave w: channels 16w..16w+15, M = 64 px, K = 9 taps x 64
//   GEMM3  wave w: channels 64w..64w+63, M = 64 px, K = 64 (+64 projection)
// The output tile is staged through LDS (over the then-dead x / y buffers) so
// the global stores are 16-byte row segments.
#include "kernels.h"

namespace adapt {

namespace {

constexpr int BT = 8;                 // output tile edge
constexpr int HT = BT + 2;            // halo tile edge
constexpr int HP = HT * HT;           // halo pixels (100)
constexpr int CM = 64;                // bottleneck width
constexpr int CO = 256;               // block output channels

// byte offset of 16-byte chunk c of row r in an LDS image with `nch` chunks per row
template <int NCH>
__device__ __forceinline__ int sw(int r, int c) {
  if constexpr (NCH >= 16) return r * (NCH * 16) + ((c ^ (r & 15)) << 4);
  else return r * (NCH * 16) + ((c ^ ((r >> 1) & 7)) << 4);
}

template <int CIN, bool PROJ>
struct BnShape {
  static constexpr int XCH = CIN / 8;                 // 16-byte chunks per x pixel
  static constexpr int XS = HP * CIN * 2;             // x halo image
  static constexpr int Y1S = HP * CM * 2;
  static constexpr int Y2S = BT * BT * CM * 2;
  static constexpr int OS = BT * BT * CO * 2;         // output tile, staged over the dead images
  static constexpr int BODY = XS + Y1S + Y2S;
  static constexpr int LDS = BODY > OS ? BODY : OS;
  static constexpr int KS1 = CIN / 32;
  static constexpr int KS3 = PROJ ? 4 : 2;
};

template <int CIN, bool PROJ>
__global__ __launch_bounds__(256, 2) void bottleneck_kernel(BottleneckParams p) {
  using S = BnShape<CIN, PROJ>;
  constexpr int XCH = S::XCH;
  __shared__ __attribute__((aligned(16))) char smem[S::LDS];
  char* xs = smem;
  char* y1s = smem + S::XS;
  char* y2s = y1s + S::Y1S;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int tw = p.W / BT, th = p.H / BT;
  const int ntiles = p.B * th * tw;
  const int tile = xcd_remap(blockIdx.x, ntiles);
  const int img = tile / (th * tw);
  const int ty = (tile / tw) % th, tx = tile % tw;
  const int gy0 = ty * BT - 1, gx0 = tx * BT - 1;

  // ---- x halo -> LDS (zeros outside the image): every load of the thread in flight at once
  const u32x4 z4 = {0u, 0u, 0u, 0u};
  constexpr int XIT = (HP * XCH + 255) / 256;
  {
    u32x4 v[XIT];
#pragma unroll
    for (int it = 0; it < XIT; ++it) {
      const int i = tid + it * 256;
      const int px = i / XCH, c = i - px * XCH;
      const int gy = gy0 + px / HT, gx = gx0 + px % HT;
      v[it] = z4;
      if (i < HP * XCH && (unsigned)gy < (unsigned)p.H && (unsigned)gx < (unsigned)p.W)
        v[it] = *(const u32x4*)(p.x + (((size_t)img * p.H + gy) * p.W + gx) * CIN + c * 8);
    }
#pragma unroll
    for (int it = 0; it < XIT; ++it) {
      const int i = tid + it * 256;
      if (i < HP * XCH) *(u32x4*)(xs + sw<XCH>(i / XCH, i % XCH)) = v[it];
    }
  }
  __syncthreads();

  // Each wave owns ONE 16-channel n-fragment in GEMM1 and GEMM2, so the four
  // waves load disjoint weight fragments (no 4x redundant L2 traffic) and all
  // of a wave's fragments for a GEMM are requested before its first MFMA.
  // ---- GEMM1: y1[halo px][64] = relu(x . W1^T + b1), zero outside the image
  {
    f32x4 acc[7];
#pragma unroll
    for (int i = 0; i < 7; ++i) acc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
    const bf16x8* w1 = (const bf16x8*)p.w1;
    bf16x8 b[S::KS1];
#pragma unroll
    for (int ks = 0; ks < S::KS1; ++ks) b[ks] = w1[(wave * S::KS1 + ks) * 64 + lane];
#pragma unroll
    for (int ks = 0; ks < S::KS1; ++ks) {
#pragma unroll
      for (int mf = 0; mf < 7; ++mf) {
        // rows >= 100 of fragment 6 read the next LDS image: their results are dropped
        const bf16x8 a = *(const bf16x8*)(xs + sw<XCH>(mf * 16 + fr, ks * 4 + fq));
        acc[mf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[ks], acc[mf], 0, 0, 0);
      }
    }
    const int n = wave * 16 + fr;
    const float bias = p.b1[n];
#pragma unroll
    for (int mf = 0; mf < 7; ++mf)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int px = mf * 16 + fq * 4 + r;
        if (px >= HP) continue;
        const int gy = gy0 + px / HT, gx = gx0 + px % HT;
        const bool in = (unsigned)gy < (unsigned)p.H && (unsigned)gx < (unsigned)p.W;
        const float v = in ? fmaxf(acc[mf][r] + bias, 0.f) : 0.f;
        *(bf16*)(y1s + sw<8>(px, n >> 3) + (n & 7) * 2) = f2bf(v);
      }
  }
  __syncthreads();

  // ---- GEMM2: y2[64 px][64] = relu(conv3x3(y1) + b2); wave w: channels 16w..16w+15
  {
    f32x4 acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    const bf16x8* w2 = (const bf16x8*)p.w2;
#pragma unroll
    for (int half = 0; half < 2; ++half) {             // 18 k-steps in two register-resident halves
      bf16x8 b[9];
#pragma unroll
      for (int t = 0; t < 9; ++t) b[t] = w2[(wave * 18 + half * 9 + t) * 64 + lane];
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int ks = half * 9 + t, tap = ks >> 1, h = ks & 1;
#pragma unroll
        for (int mf = 0; mf < 4; ++mf) {
          const int opx = mf * 16 + fr;
          const int hp = ((opx >> 3) + tap / 3) * HT + (opx & 7) + tap % 3;
          const bf16x8 a = *(const bf16x8*)(y1s + sw<8>(hp, h * 4 + fq));
          acc[mf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[t], acc[mf], 0, 0, 0);
        }
      }
    }
    const int n = wave * 16 + fr;
    const float bias = p.b2[n];
#pragma unroll
    for (int mf = 0; mf < 4; ++mf)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int px = mf * 16 + fq * 4 + r;
        *(bf16*)(y2s + sw<8>(px, n >> 3) + (n & 7) * 2) = f2bf(fmaxf(acc[mf][r] + bias, 0.f));
      }
  }
  __syncthreads();

  // ---- GEMM3: out[64 px][256] = relu(y2 . W3^T (+ x . Wp^T) + b3 (+ x)); wave w: channels 64w..64w+63
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  {
    const bf16x8* w3 = (const bf16x8*)p.w3;
    bf16x8 bw[S::KS3][4];
#pragma unroll
    for (int ks = 0; ks < S::KS3; ++ks)
#pragma unroll
      for (int j = 0; j < 4; ++j) bw[ks][j] = w3[((wave * 4 + j) * S::KS3 + ks) * 64 + lane];
#pragma unroll
    for (int ks = 0; ks < S::KS3; ++ks) {
      const bf16x8* b = bw[ks];
#pragma unroll
      for (int mf = 0; mf < 4; ++mf) {
        const int px = mf * 16 + fr;
        bf16x8 a;
        if (ks < 2) {
          a = *(const bf16x8*)(y2s + sw<8>(px, ks * 4 + fq));
        } else {                                        // projection shortcut: the x pixel under px
          const int hp = ((px >> 3) + 1) * HT + (px & 7) + 1;
          a = *(const bf16x8*)(xs + sw<XCH>(hp, (ks - 2) * 4 + fq));
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[mf][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[j], acc[mf][j], 0, 0, 0);
      }
    }
  }
  // epilogue values in registers (the residual is read from the x image first)
  bf16 o[4][4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = (wave * 4 + j) * 16 + fr;
    const float bias = p.b3[n];
#pragma unroll
    for (int mf = 0; mf < 4; ++mf)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int px = mf * 16 + fq * 4 + r;
        float v = acc[mf][j][r] + bias;
        if constexpr (!PROJ) {
          const int hp = ((px >> 3) + 1) * HT + (px & 7) + 1;
          v += bf2f(*(const bf16*)(xs + sw<XCH>(hp, n >> 3) + (n & 7) * 2));
        }
        o[mf][j][r] = f2bf(fmaxf(v, 0.f));
      }
  }
  __syncthreads();                                     // every read of x / y2 is done: reuse LDS for the tile
  char* os = smem;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = (wave * 4 + j) * 16 + fr;
#pragma unroll
    for (int mf = 0; mf < 4; ++mf)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int px = mf * 16 + fq * 4 + r;
        *(bf16*)(os + sw<32>(px, n >> 3) + (n & 7) * 2) = o[mf][j][r];
      }
  }
  __syncthreads();
  for (int i = tid; i < BT * BT * 32; i += 256) {
    const int px = i >> 5, c = i & 31;
    const int gy = ty * BT + (px >> 3), gx = tx * BT + (px & 7);
    *(u32x4*)(p.out + (((size_t)img * p.H + gy) * p.W + gx) * CO + c * 8) = *(const u32x4*)(os + sw<32>(px, c));
  }
}

}  // namespace

hipError_t bottleneck_forward(const BottleneckParams& p, int cin, bool proj, hipStream_t s) {
  if (p.H % BT || p.W % BT || p.B < 1) return hipErrorInvalidValue;
  const dim3 grid(p.B * (p.H / BT) * (p.W / BT)), block(256);
  if (cin == 256 && !proj) hipLaunchKernelGGL((bottleneck_kernel<256, false>), grid, block, 0, s, p);
  else if (cin == 64 && proj) hipLaunchKernelGGL((bottleneck_kernel<64, true>), grid, block, 0, s, p);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace adapt
