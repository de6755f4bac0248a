// fp32 3x3 / stride-1 / pad-1 convolution by Winograd F(2x2, 3x3) on the fp32
// matrix cores (v_mfma_f32_16x16x4_f32), transforms fused: one launch reads
// the NHWC input and writes the NHWC output (BN folded, bias, ReLU).
//
// Why: at fp32 every ResNet 3x3 conv is matrix-bound (the fp32 MFMA runs at
// 1/16 of the bf16 rate) and the direct implicit-GEMM kernels (conv_f32g.hip)
// spend 76-86 us per layer at ~97 TF/s (tools/conv_bench_f32.py).  F(2x2, 3x3)
// computes each 2x2 output tile from a 4x4 input patch with 16 multiplies per
// (cin, cout) instead of 36: 2.25x less matrix work.  All arithmetic stays
// fp32 (the input / output transforms use only +/-1 coefficients, the weight
// transform's 1/2 factors are exact and done on the host in fp64), which is
// the algorithm cuDNN applies to float32 3x3 convs under TensorFlow -- the
// reference's Keras model (`/root/reference/test/test.py:13`, float32).
//
//   V_p[t][c] = (B^T d_t,c B)_p     (d = the 4x4 input patch of tile t, p = 0..15)
//   M_p[t][n] = sum_c V_p[t][c] U_p[c][n]          U = G g G^T  (host)
//   y_t[n]    = A^T M[t][n] A + bias[n]   (2x2 outputs)
//
// Block = NWM waves; wave w owns 16 tiles (the MFMA rows) x 16*FN output
// channels x all 16 positions (acc 64*FN VGPRs).  K walks the input channels
// in chunks of 16: MFMA step s of a chunk takes channel 4q+s from lane group q
// (the K permutation of conv_f32g.hip), so
//   * a lane's share of the input patch is 16 float4 loads (its tile, its 4
//     channels), transformed in registers -- no LDS, the A operand never exists
//     as a matrix;
//   * the transformed weights are host-packed in MFMA fragment order
//     ([chunk][n-frag][p][lane][4]) and streamed into an LDS ring by LDS-DMA,
//     one contiguous 16*FN KiB run per chunk per block, read back with
//     conflict-free lane-linear ds_read_b128 (one per (p, n-frag) per chunk).
// The accumulator layout puts all 16 positions of (tile, channel) in one lane,
// so the output transform is lane-local: no shuffle, no LDS round trip.
// Split-K (gridDim.z) writes the transformed partial outputs to fp32 slabs
// (linear, so A^T (sum M) A = sum A^T M A); splitk_reduce_f32 adds bias / ReLU.
#include "kernels.h"

namespace adapt {

namespace {

typedef __attribute__((address_space(3))) void lds_void_w;

__device__ __attribute__((aligned(64))) float g_wino_zero[64];

// two waves per SIMD (<= 256 VGPRs) up to FN = 2; FN = 3 keeps one (its 192 accumulators)
template <int NWM, int FN>
constexpr int wino_min_blocks() { return FN <= 2 ? (8 / NWM > 0 ? 8 / NWM : 1) : (4 / NWM > 0 ? 4 / NWM : 1); }

template <int NWM, int FN, int STAGES>
__global__ __launch_bounds__(NWM * 64, (wino_min_blocks<NWM, FN>())) void conv_wino_f32_kernel(WinoF32Params p) {
  constexpr int NT = NWM * 64;
  constexpr int BT = 16 * NWM;                       // tiles per block
  constexpr int PIECES = 16 * FN;                    // 1 KiB weight pieces per chunk
  constexpr int PPW = (PIECES + NWM - 1) / NWM;      // pieces per wave
  constexpr int SLOT = PIECES * 1024;
  __shared__ __attribute__((aligned(16))) char ring[STAGES * SLOT];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 15, q = lane >> 4;
  const int nf0 = blockIdx.y * FN;                   // first 16-channel output fragment
  const int NF = p.N / 16;
  const int KC = p.C / 16;                           // 16-channel chunks
  const int kper = (KC + p.ksplit - 1) / p.ksplit;
  const int kc0 = blockIdx.z * kper, kc1 = min(KC, kc0 + kper);

  // ---- this lane's tile (A row r of the wave) and its 4x4 input patch
  const int t = blockIdx.x * BT + wave * 16 + r;
  const int tpi = p.TH * p.TW;
  const bool tok = t < p.T;
  const int img = tok ? t / tpi : 0;
  const int tr = tok ? t - img * tpi : 0;
  const int ty = tr / p.TW, tx = tr - ty * p.TW;
  const int iy0 = 2 * ty - 1, ix0 = 2 * tx - 1;
  unsigned ok = 0;                                   // bit 4*dy + dx: patch pixel inside the image
#pragma unroll
  for (int dy = 0; dy < 4; ++dy)
#pragma unroll
    for (int dx = 0; dx < 4; ++dx)
      if (tok && (unsigned)(iy0 + dy) < (unsigned)p.H && (unsigned)(ix0 + dx) < (unsigned)p.W) ok |= 1u << (4 * dy + dx);
  const float* xb = p.x + (((ptrdiff_t)img * p.H + iy0) * p.W + ix0) * p.C + 4 * q;
  const ptrdiff_t rstride = (ptrdiff_t)p.W * p.C;

  // ---- weight pieces of chunk kc -> ring slot
  const float* ub = p.u + (size_t)nf0 * 16 * 256;    // 256 floats per piece
  const size_t uchunk = (size_t)NF * 16 * 256;
  auto issue_w = [&](int kc, int slot) {
    const float* src = ub + (size_t)kc * uchunk;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int pc = wave * PPW + i;
      if (PIECES % NWM == 0 || pc < PIECES)
        __builtin_amdgcn_global_load_lds((const void*)(src + pc * 256 + lane * 4),
                                         (lds_void_w*)(ring + slot * SLOT + pc * 1024), 16, 0, 0);
    }
  };

  f32x4 acc[16][FN];
#pragma unroll
  for (int i = 0; i < 16; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  if (kc0 < kc1) issue_w(kc0, 0);
  for (int kc = kc0; kc < kc1; ++kc) {
    const int slot = (kc - kc0) % STAGES;
    // this lane's patch, channels 16kc + 4q .. +3 (zero outside the image)
    f32x4 d[4][4];
#pragma unroll
    for (int dy = 0; dy < 4; ++dy)
#pragma unroll
      for (int dx = 0; dx < 4; ++dx) {
        const float* src = ((ok >> (4 * dy + dx)) & 1u) ? xb + dy * rstride + dx * p.C + kc * 16 : g_wino_zero;
        d[dy][dx] = *(const f32x4*)src;
      }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();                    // every wave's pieces of chunk kc are in; slot kc+1 is free
    asm volatile("" ::: "memory");
    if (kc + 1 < kc1) issue_w(kc + 1, (slot + 1) % STAGES);

    // B^T d: rows
#pragma unroll
    for (int dx = 0; dx < 4; ++dx) {
      const f32x4 a0 = d[0][dx], a1 = d[1][dx], a2 = d[2][dx], a3 = d[3][dx];
      d[0][dx] = a0 - a2;
      d[1][dx] = a1 + a2;
      d[2][dx] = a2 - a1;
      d[3][dx] = a1 - a3;
    }
    const char* sl = ring + slot * SLOT;
#pragma unroll
    for (int pa = 0; pa < 4; ++pa) {
      // (B^T d B)[pa][0..3] for this lane's 4 channels
      f32x4 v[4];
      v[0] = d[pa][0] - d[pa][2];
      v[1] = d[pa][1] + d[pa][2];
      v[2] = d[pa][2] - d[pa][1];
      v[3] = d[pa][1] - d[pa][3];
      f32x4 u[4][FN];
#pragma unroll
      for (int pb = 0; pb < 4; ++pb)
#pragma unroll
        for (int j = 0; j < FN; ++j) u[pb][j] = *(const f32x4*)(sl + ((j * 16 + pa * 4 + pb) * 64 + lane) * 16);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int pb = 0; pb < 4; ++pb)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[pa * 4 + pb][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(v[pb][s], u[pb][j][s], acc[pa * 4 + pb][j], 0, 0, 0);
    }
  }

  // ---- output transform A^T M A (lane-local) + bias / ReLU, or a split-K slab
  // acc[p][j][i] = M_p[tile 4q + i of the wave][channel 16 (nf0 + j) + r]
  const bool split = p.ksplit > 1;
  float* dst = split ? p.ws + (size_t)blockIdx.z * p.B * p.H * p.W * p.N : p.out;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int tt = blockIdx.x * BT + wave * 16 + 4 * q + i;
    if (tt >= p.T) continue;
    const int im = tt / tpi, rr = tt - im * tpi;
    const int oy = 2 * (rr / p.TW), ox = 2 * (rr - (rr / p.TW) * p.TW);
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = (nf0 + j) * 16 + r;
      float m[4][4];
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) m[a][b] = acc[a * 4 + b][j][i];
      float w0[4], w1[4];
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        w0[b] = m[0][b] + m[1][b] + m[2][b];
        w1[b] = m[1][b] - m[2][b] - m[3][b];
      }
      float y[2][2];
      y[0][0] = w0[0] + w0[1] + w0[2];
      y[0][1] = w0[1] - w0[2] - w0[3];
      y[1][0] = w1[0] + w1[1] + w1[2];
      y[1][1] = w1[1] - w1[2] - w1[3];
      const float bn = split ? 0.f : p.bias[n];
#pragma unroll
      for (int dy = 0; dy < 2; ++dy)
#pragma unroll
        for (int dx = 0; dx < 2; ++dx) {
          if (oy + dy >= p.H || ox + dx >= p.W) continue;
          const size_t o = (((size_t)im * p.H + oy + dy) * p.W + ox + dx) * p.N + n;
          float v = y[dy][dx] + bn;
          if (!split) {
            if (p.res) v += p.res[o];
            v = act_relu(v, p.relu);
          }
          dst[o] = v;
        }
    }
  }
}

template <int NWM, int FN, int STAGES>
hipError_t launch_wino(const WinoF32Params& p, hipStream_t s) {
  if (p.N % (16 * FN)) return hipErrorInvalidValue;
  const dim3 grid((p.T + 16 * NWM - 1) / (16 * NWM), p.N / (16 * FN), p.ksplit), block(NWM * 64);
  hipLaunchKernelGGL((conv_wino_f32_kernel<NWM, FN, STAGES>), grid, block, 0, s, p);
  return hipGetLastError();
}

}  // namespace

// Winograd cfg ids (ops/conv.py WINO_F32_CFGS mirrors them): id -> waves (16 tiles each), 16-channel
// output fragments per wave, LDS ring stages
#define ADAPT_WINO_CFGS(X) \
  X(80, 4, 2, 2)           \
  X(81, 4, 1, 2)           \
  X(82, 2, 2, 2)           \
  X(83, 8, 2, 2)           \
  X(84, 4, 3, 2)           \
  X(85, 2, 1, 2)

bool conv_wino_f32_ok(int cfg, int C, int N) {
  switch (cfg) {
#define X(id, NWM_, FN_, S_) case id: return C % 16 == 0 && N % (16 * FN_) == 0;
    ADAPT_WINO_CFGS(X)
#undef X
  }
  return false;
}

hipError_t conv_wino_f32_launch(const WinoF32Params& p, int cfg, hipStream_t s) {
  if (p.C % 16 || p.ksplit < 1 || p.T != p.B * p.TH * p.TW) return hipErrorInvalidValue;
  if (p.ksplit > 1 && !p.ws) return hipErrorInvalidValue;
  switch (cfg) {
#define X(id, NWM_, FN_, S_) case id: return launch_wino<NWM_, FN_, S_>(p, s);
    ADAPT_WINO_CFGS(X)
#undef X
  }
  return hipErrorInvalidValue;
}

}  // namespace adapt
