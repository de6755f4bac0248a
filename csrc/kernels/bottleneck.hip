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
// MFMA v_mfma_f32_16x16x32_bf16, run transposed (weights as the A operand):
// activation fragments come from LDS (16-byte chunks XOR-swizzled per row so
// a fragment read is conflict-free), weight fragments straight from global/L2
// in a host-packed fragment order (one coalesced 1 KiB load per wave per
// fragment; every workgroup reads the same 136 KB of weights, which stay
// L2-resident).  Four waves, (wm, wn) = (w >> 1, w & 1):
//   GEMM1  channels 32wn..32wn+31, halo px frags 4wm.. (4 / 3 of 7: 100 px), K = CIN
//   GEMM2  channels 32wn..32wn+31, px frags 2wm, 2wm+1, K = 9 taps x 64
//   GEMM3  channels 64w..64w+63, M = 64 px, K = 64 (+64 projection)
// The output tile is staged through LDS (over the then-dead x / y buffers) so
// the global stores are 16-byte row segments.
#include "kernels.h"

namespace adapt {

namespace {

typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

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

__device__ __attribute__((aligned(64))) bf16 g_bn_zero[64];   // 16-byte zero source for halo padding

// LDS-only barrier: the waves exchange data through LDS alone, so a barrier
// must not drain the global loads kept in flight across it (__syncthreads'
// release fence would wait vmcnt(0)).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// ABL: ablation switches for tools/bottleneck_ablate.hip (0 in production):
// 1 = no MFMA, 2 = no x-halo global loads, 4 = no weight loads, 8 = no output
// global stores, 16 = no y1 / y2 LDS writes, 32 = no A-fragment LDS reads,
// 64 = no residual LDS reads / output LDS staging.
//
// Every global load is issued ahead of its use: the x-halo loads are
// unconditional (padding pixels read a zero page, so hipcc cannot branch and
// wait around each one) and all in flight at once, GEMM1's weights ride with
// them, and each later group of weight fragments is requested one group
// ahead, under the MFMAs of the previous one.  (tools/bottleneck_ablate.hip:
// with every load issued just before its use, the x loads and the weight
// loads each cost 7-11 us of the 42 us block.)  A persistent variant that
// also prefetched the next tile's halo into registers spilled (hipcc hoists
// the halo index math out of the tile loop) and was dropped.
template <int CIN, bool PROJ, int ABL = 0>
__global__ __launch_bounds__(256, 2) void bottleneck_kernel(BottleneckParams p) {
  using S = BnShape<CIN, PROJ>;
  constexpr int XCH = S::XCH;
  constexpr int KS1 = S::KS1, KS3 = S::KS3;
  __shared__ __attribute__((aligned(16))) char smem[S::LDS];
  char* xs = smem;
  char* y1s = smem + S::XS;
  char* y2s = y1s + S::Y1S;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int wm = wave >> 1, wn = wave & 1;
  const int tw = p.W / BT, th = p.H / BT;
  const int ntiles = p.B * th * tw;
  const int t = xcd_remap(blockIdx.x, ntiles);
  const int img = t / (th * tw);
  const int ty = (t / tw) % th, tx = t % tw;
  const int gy0 = ty * BT - 1, gx0 = tx * BT - 1;
  const bf16x8* w1 = (const bf16x8*)p.w1;
  const bf16x8* w2 = (const bf16x8*)p.w2;
  const bf16x8* w3 = (const bf16x8*)p.w3;

  // ---- x halo of a tile -> registers (zero page outside the image: no load is conditional)
  constexpr int XIT = (HP * XCH + 255) / 256;
  u32x4 xr[XIT];
  auto load_x = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int it = 0; it < XIT; ++it) {
      const int i = tid + it * 256;
      const int px = i / XCH, c = i - px * XCH;
      const int gy = gy0 + px / HT, gx = gx0 + px % HT;
      const bool in = !(ABL & 2) && i < HP * XCH && (unsigned)gy < (unsigned)p.H && (unsigned)gx < (unsigned)p.W;
      const bf16* src = in ? p.x + (((size_t)img * p.H + gy) * p.W + gx) * CIN + c * 8 : g_bn_zero;
      xr[it] = *(const u32x4*)src;
    }
  };
  auto store_x = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int it = 0; it < XIT; ++it) {
      const int i = tid + it * 256;
      if (i < HP * XCH) *(u32x4*)(xs + sw<XCH>(i / XCH, i % XCH)) = xr[it];
    }
  };

  // weight fragments: GEMM1 in two K halves (2 channel frags x KS1/2 each), GEMM2 in
  // sixths (2 x 3), GEMM3 (KS3 x 4); each group is requested one group ahead of its use
  constexpr int KH1 = KS1 / 2;
  bf16x8 b1lo[2][KH1], b1hi[2][KH1];
  auto load_w1 = [&](bf16x8 (&b)[2][KH1], int half) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int k = 0; k < KH1; ++k)
        b[j][k] = (ABL & 4) ? bf16x8{} : w1[((2 * wn + j) * KS1 + half * KH1 + k) * 64 + lane];
  };
  auto load_w2 = [&](bf16x8 (&b)[2][3], int sixth) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int t = 0; t < 3; ++t) b[j][t] = (ABL & 4) ? bf16x8{} : w2[((2 * wn + j) * 18 + sixth * 3 + t) * 64 + lane];
  };
  bf16x8 b3[KS3][4];
  auto load_w3 = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int ks = 0; ks < KS3; ++ks)
#pragma unroll
      for (int j = 0; j < 4; ++j) b3[ks][j] = (ABL & 4) ? bf16x8{} : w3[((wave * 4 + j) * KS3 + ks) * 64 + lane];
  };

  load_x();
  load_w1(b1lo, 0);
  load_w1(b1hi, 1);
  store_x();
  lds_barrier();
  {
    bf16x8 b2a[2][3], b2b[2][3];

    // Every GEMM runs TRANSPOSED (A = weight fragment, B = activation
    // fragment, C = [channel][pixel]): a lane's four accumulator values are four
    // consecutive channels of one pixel, so the y1 / y2 / output-tile LDS writes
    // and the residual reads are 8-byte accesses instead of four 2-byte ones.
    // GEMM1 and GEMM2 split their tiles 2 (pixels) x 2 (channels) over the
    // waves: every activation fragment is read from LDS by two waves, not four.
    // ---- GEMM1: y1[halo px][64] = relu(x . W1^T + b1), zero outside the image
    //      wave (wm, wn): halo pixel frags 4wm.. (4 or 3 of 7), channel frags 2wn, 2wn+1
    {
      constexpr int MF0 = 4;                             // pixel frags of wm = 0 (wm = 1 takes the other 3)
      const int mfb = wm * MF0, mfn = wm ? 7 - MF0 : MF0;
      f32x4 acc[MF0][2];
#pragma unroll
      for (int i = 0; i < MF0; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS1; ++ks) {
        if (ks == KH1) load_w2(b2a, 0);                  // GEMM2's first sixth, under GEMM1's second half
#pragma unroll
        for (int i = 0; i < MF0; ++i) {
          if (i >= mfn) continue;
          // rows >= 100 of fragment 6 read the next LDS image: their results are dropped
          const bf16x8 a = (ABL & 32) ? bf16x8{} : *(const bf16x8*)(xs + sw<XCH>((mfb + i) * 16 + fr, ks * 4 + fq));
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const bf16x8 w = ks < KH1 ? b1lo[j][ks] : b1hi[j][ks - KH1];
            if constexpr (ABL & 1) asm volatile("" ::"v"(a), "v"(w));
            else acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w, a, acc[i][j], 0, 0, 0);
          }
        }
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = (2 * wn + j) * 16 + fq * 4;        // this lane's 4 channels
        const f32x4 bias = *(const f32x4*)(p.b1 + n);
#pragma unroll
        for (int i = 0; i < MF0; ++i) {
          const int px = (mfb + i) * 16 + fr;
          if (i >= mfn || px >= HP) continue;
          const int gy = gy0 + px / HT, gx = gx0 + px % HT;
          const bool in = (unsigned)gy < (unsigned)p.H && (unsigned)gx < (unsigned)p.W;
          bf16x4 v;
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = f2bf(in ? fmaxf(acc[i][j][r] + bias[r], 0.f) : 0.f);
          if constexpr (ABL & 16) asm volatile("" ::"v"(v));
          else *(bf16x4*)(y1s + sw<8>(px, n >> 3) + (n & 7) * 2) = v;
        }
      }
    }
    lds_barrier();

    // ---- GEMM2: y2[64 px][64] = relu(conv3x3(y1) + b2); wave (wm, wn): pixel frags 2wm, 2wm+1,
    //      channel frags 2wn, 2wn+1; 18 k-steps (9 taps x 2 channel halves) in six
    //      register-resident groups, the next group (then GEMM3's weights) requested ahead
    {
      f32x4 acc[2][2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
      auto sixth = [&](bf16x8 (&b)[2][3], int g) __attribute__((always_inline)) {
#pragma unroll
        for (int t6 = 0; t6 < 3; ++t6) {
          const int ks = g * 3 + t6, tap = ks >> 1, h = ks & 1;
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            const int opx = (2 * wm + i) * 16 + fr;
            const int hp = ((opx >> 3) + tap / 3) * HT + (opx & 7) + tap % 3;
            const bf16x8 a = (ABL & 32) ? bf16x8{} : *(const bf16x8*)(y1s + sw<8>(hp, h * 4 + fq));
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              if constexpr (ABL & 1) asm volatile("" ::"v"(a), "v"(b[j][t6]));
              else acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j][t6], a, acc[i][j], 0, 0, 0);
            }
          }
        }
      };
      load_w2(b2b, 1);
      sixth(b2a, 0);
      load_w2(b2a, 2);
      sixth(b2b, 1);
      load_w2(b2b, 3);
      sixth(b2a, 2);
      load_w2(b2a, 4);
      sixth(b2b, 3);
      load_w2(b2b, 5);
      sixth(b2a, 4);
      load_w3();
      sixth(b2b, 5);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = (2 * wn + j) * 16 + fq * 4;
        const f32x4 bias = *(const f32x4*)(p.b2 + n);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int px = (2 * wm + i) * 16 + fr;
          bf16x4 v;
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = f2bf(fmaxf(acc[i][j][r] + bias[r], 0.f));
          if constexpr (ABL & 16) asm volatile("" ::"v"(v));
          else *(bf16x4*)(y2s + sw<8>(px, n >> 3) + (n & 7) * 2) = v;
        }
      }
    }
    lds_barrier();

    // ---- GEMM3: out[64 px][256] = relu(y2 . W3^T (+ x . Wp^T) + b3 (+ x)); wave w: channels 64w..64w+63,
    //      in two halves of 32 channels (accumulators of one half live at a time)
    bf16x4 o[4][4];                                      // lane -> pixel mf*16 + fr, channels n .. n+3
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      f32x4 acc[4][2];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS3; ++ks) {
#pragma unroll
        for (int mf = 0; mf < 4; ++mf) {
          const int px = mf * 16 + fr;
          bf16x8 a;
          if (ABL & 32) {
            a = bf16x8{};
          } else if (ks < 2) {
            a = *(const bf16x8*)(y2s + sw<8>(px, ks * 4 + fq));
          } else {                                      // projection shortcut: the x pixel under px
            const int hp = ((px >> 3) + 1) * HT + (px & 7) + 1;
            a = *(const bf16x8*)(xs + sw<XCH>(hp, (ks - 2) * 4 + fq));
          }
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            if constexpr (ABL & 1) asm volatile("" ::"v"(a), "v"(b3[ks][2 * hf + j]));
            else acc[mf][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b3[ks][2 * hf + j], a, acc[mf][j], 0, 0, 0);
          }
        }
      }
      // epilogue values in registers (the residual is read from the x image first)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = (wave * 4 + 2 * hf + j) * 16 + fq * 4;
        const f32x4 bias = *(const f32x4*)(p.b3 + n);
#pragma unroll
        for (int mf = 0; mf < 4; ++mf) {
          const int px = mf * 16 + fr;
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = acc[mf][j][r] + bias[r];
          if constexpr (!PROJ && !(ABL & 64)) {
            const int hp = ((px >> 3) + 1) * HT + (px & 7) + 1;
            const bf16x4 res = *(const bf16x4*)(xs + sw<XCH>(hp, n >> 3) + (n & 7) * 2);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] += bf2f(res[r]);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) o[mf][2 * hf + j][r] = f2bf(fmaxf(v[r], 0.f));
        }
      }
    }
    lds_barrier();                                       // every read of x / y2 is done: reuse LDS for the tile
    char* os = smem;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = (wave * 4 + j) * 16 + fq * 4;
#pragma unroll
      for (int mf = 0; mf < 4; ++mf) {
        const int px = mf * 16 + fr;
        if constexpr (ABL & 64) asm volatile("" ::"v"(o[mf][j]));
        else *(bf16x4*)(os + sw<32>(px, n >> 3) + (n & 7) * 2) = o[mf][j];
      }
    }
    lds_barrier();
    for (int i = tid; i < BT * BT * 32; i += 256) {
      const int px = i >> 5, c = i & 31;
      const int gy = ty * BT + (px >> 3), gx = tx * BT + (px & 7);
      const u32x4 v = *(const u32x4*)(os + sw<32>(px, c));
      if constexpr (ABL & 8) asm volatile("" ::"v"(v));
      else *(u32x4*)(p.out + (((size_t)img * p.H + gy) * p.W + gx) * CO + c * 8) = v;
    }
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
