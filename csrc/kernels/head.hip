// Classifier head: GlobalAveragePooling2D -> Dense(+bias) -> softmax
// (`avg_pool` / `predictions` of the Keras ResNets; the reference runs them
// inside `model.predict`, src/node.py:177).
//
// The head is tiny (bs=32: 3.2 MB in, a 32 x 2048 x 1000 GEMM) but sat at
// ~20 us on the generic paths: the old GAP loop made each thread walk the 49
// pixels of one channel chunk with dependent loads, and the conv-kernel GEMM
// ran M = 32 rows through 64-row tiles with a K loop of 32 latency-bound
// steps plus a split-K reduce launch.  Here:
//
// * gap: a block takes (image, 256 channels); 8 pixel groups per channel chunk
//   issue all their loads before summing, LDS reduction of the 8 partials;
// * dense_partial: small-M GEMV on MFMA.  Block = 16 output columns x all M
//   (<= 32) rows x one K slice; the whole K slice of A and B is loaded up front
//   (one round trip), fp32 partials per K slice;
// * dense_finish: sum of the K-slice partials + bias (+ row softmax), one
//   block per row.
#include "kernels.h"

namespace adapt {

// ------------------------------------------------------------------ GAP
// block (image b, channel block of 32 chunks = 256 channels); 256 threads = 32 chunks x 8 pixel groups
// (bs=32 x 2048 channels: 256 blocks, one per CU)
constexpr int GAP_CH = 32, GAP_PG = 8;
__global__ __launch_bounds__(256) void gap2_kernel(const bf16* __restrict__ x, bf16* __restrict__ y,
                                                   float* __restrict__ y32, int HW, int C) {
  __shared__ float part[GAP_PG][GAP_CH][9];
  const int b = blockIdx.y;
  const int ch = threadIdx.x % GAP_CH, grp = threadIdx.x / GAP_CH;
  const int cc = blockIdx.x * GAP_CH + ch;              // 8-channel chunk
  const bool ok = cc * 8 < C;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (ok) {
    const bf16* base = x + (size_t)b * HW * C + cc * 8;
    constexpr int U = 4;
    for (int i0 = grp; i0 < HW; i0 += GAP_PG * U) {
      V8 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 + GAP_PG * u;
        v[u].u = i < HW ? *(const u32x4*)(base + (size_t)i * C) : (u32x4){0u, 0u, 0u, 0u};
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int t = 0; t < 8; ++t) s[t] += bf2f(v[u].e[t]);
    }
  }
#pragma unroll
  for (int t = 0; t < 8; ++t) part[grp][ch][t] = s[t];
  __syncthreads();
  if (grp != 0 || !ok) return;
  const float inv = 1.f / (float)HW;
  V8 o;
  float r[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    float a = 0.f;
#pragma unroll
    for (int q = 0; q < GAP_PG; ++q) a += part[q][ch][t];
    r[t] = a * inv;
    o.e[t] = f2bf(r[t]);
  }
  if (y) *(u32x4*)(y + (size_t)b * C + cc * 8) = o.u;
  if (y32) {
    float* d = y32 + (size_t)b * C + cc * 8;
#pragma unroll
    for (int t = 0; t < 8; ++t) d[t] = r[t];
  }
}

// ------------------------------------------------------ small-M dense (MFMA)
// x: [M][K] bf16 (M <= 32), w: [Npad][Kpad] bf16 (packed conv weights, k contiguous),
// part: [KS][M][N] fp32.  grid = (ceil(N/16), KS), one wave per block.
constexpr int DH_MAXK = 512;    // K slice per block (elements): 16 MFMA steps, 192 VGPRs of operands

__global__ __launch_bounds__(64) void dense_partial_kernel(const bf16* __restrict__ x, const bf16* __restrict__ w,
                                                           float* __restrict__ part, int M, int N, int K, int Kpad,
                                                           int kslice) {
  const int lane = threadIdx.x, fr = lane & 15, fq = lane >> 4;
  const int n0 = blockIdx.x * 16;
  const int k0 = blockIdx.y * kslice;
  const int k1 = min(K, k0 + kslice);
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  const bf16* wr = w + (size_t)(n0 + fr) * Kpad;        // B column n0+fr (packed rows are 256-aligned)
  const bf16* x0 = x + (size_t)fr * K;                  // A rows fr, fr+16
  const bf16* x1 = x + (size_t)(fr + 16) * K;
  const bool r0 = fr < M, r1 = fr + 16 < M;
  // all loads of the slice first (<= 32 steps x 3 x 16 B per lane), then the MFMAs
  constexpr int MAXS = DH_MAXK / 32;
  bf16x8 a0[MAXS], a1[MAXS], bv[MAXS];
  const int steps = (k1 - k0 + 31) / 32;
#pragma unroll
  for (int s = 0; s < MAXS; ++s) {
    const int k = k0 + s * 32 + fq * 8;
    const bool kin = s < steps && k < k1;
    V8 z;
    z.u = (u32x4){0u, 0u, 0u, 0u};
    a0[s] = (kin && r0) ? *(const bf16x8*)(x0 + k) : z.h;
    a1[s] = (kin && r1) ? *(const bf16x8*)(x1 + k) : z.h;
    bv[s] = kin ? *(const bf16x8*)(wr + k) : z.h;
  }
#pragma unroll
  for (int s = 0; s < MAXS; ++s) {
    acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[s], bv[s], acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[s], bv[s], acc1, 0, 0, 0);
  }
  // C fragment: row = 4*fq + r (+16 for acc1), col = n0 + fr
  float* pp = part + (size_t)blockIdx.y * M * N;
  const int n = n0 + fr;
  if (n < N) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = 4 * fq + r;
      if (m < M) pp[(size_t)m * N + n] = acc0[r];
      if (m + 16 < M) pp[(size_t)(m + 16) * N + n] = acc1[r];
    }
  }
}

// sum of the K-slice partials + bias -> logits (optional) and/or row softmax; one block per row
__global__ __launch_bounds__(256) void dense_finish_kernel(const float* __restrict__ part, const float* __restrict__ bias,
                                                           float* __restrict__ logits, float* __restrict__ probs,
                                                           int M, int N, int KS) {
  __shared__ float red[8];
  const int row = blockIdx.x;
  extern __shared__ float vals[];                         // N floats
  float mx = -INFINITY;
  for (int i = threadIdx.x; i < N; i += blockDim.x) {
    float v = bias ? bias[i] : 0.f;
    for (int s = 0; s < KS; ++s) v += part[((size_t)s * M + row) * N + i];
    vals[i] = v;
    if (logits) logits[(size_t)row * N + i] = v;
    mx = fmaxf(mx, v);
  }
  if (!probs) return;
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) red[wv] = mx;
  __syncthreads();
  mx = red[0];
  for (int i = 1; i < (int)(blockDim.x >> 6); ++i) mx = fmaxf(mx, red[i]);
  __syncthreads();
  float sum = 0.f;
  for (int i = threadIdx.x; i < N; i += blockDim.x) {
    const float e = __expf(vals[i] - mx);
    vals[i] = e;
    sum += e;
  }
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
  if (l == 0) red[wv] = sum;
  __syncthreads();
  sum = 0.f;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) sum += red[i];
  const float inv = 1.f / sum;
  for (int i = threadIdx.x; i < N; i += blockDim.x) probs[(size_t)row * N + i] = vals[i] * inv;
}

hipError_t gap(const bf16* x, bf16* y, float* y32, int B, int HW, int C, hipStream_t s) {
  dim3 grid((C / 8 + GAP_CH - 1) / GAP_CH, B);
  hipLaunchKernelGGL(gap2_kernel, grid, dim3(256), 0, s, x, y, y32, HW, C);
  return hipGetLastError();
}

int dense_small_kslices(int K) { return (K + DH_MAXK - 1) / DH_MAXK; }

// Register-resident finish for N <= 1024 (the ImageNet head): each thread owns up to 4 columns of the row,
// issues all KS x 4 partial loads before the first add, and keeps the logits in registers through the
// max / exp / sum passes (the generic kernel above round-trips them through LDS and loads serially).
__global__ __launch_bounds__(256) void dense_finish_reg_kernel(const float* __restrict__ part,
                                                               const float* __restrict__ bias,
                                                               float* __restrict__ logits, float* __restrict__ probs,
                                                               int M, int N, int KS) {
  __shared__ float red[4];
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  float v[4];
  bool ok[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int i = tid + 256 * j;
    ok[j] = i < N;
    v[j] = (ok[j] && bias) ? bias[i] : 0.f;
  }
  // four slices' loads in flight per round (the fp32 head has 16 slices; a loop of dependent
  // rounds left the finish latency-bound at 8 us); 16 slices: all of them in one round
  int sl = 0;
  if (KS == 16) {
    float t[16][4];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const float* pr = part + ((size_t)u * M + row) * N;
#pragma unroll
      for (int j = 0; j < 4; ++j) t[u][j] = ok[j] ? pr[tid + 256 * j] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 16; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] += t[u][j];
    sl = 16;
  }
  for (; sl + 4 <= KS; sl += 4) {
    float t[4][4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float* pr = part + ((size_t)(sl + u) * M + row) * N;
#pragma unroll
      for (int j = 0; j < 4; ++j) t[u][j] = ok[j] ? pr[tid + 256 * j] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] += t[u][j];
  }
  for (; sl < KS; ++sl) {
    const float* pr = part + ((size_t)sl * M + row) * N;
    float t[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) t[j] = ok[j] ? pr[tid + 256 * j] : 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] += t[j];
  }
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (!ok[j]) continue;
    if (logits) logits[(size_t)row * N + tid + 256 * j] = v[j];
    mx = fmaxf(mx, v[j]);
  }
  if (!probs) return;
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
  if (lane == 0) red[wv] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[j] = ok[j] ? __expf(v[j] - mx) : 0.f;
    sum += v[j];
  }
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
  if (lane == 0) red[wv] = sum;
  __syncthreads();
  const float inv = 1.f / (red[0] + red[1] + red[2] + red[3]);
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (ok[j]) probs[(size_t)row * N + tid + 256 * j] = v[j] * inv;
}

// fp32 classifier GEMM for M <= 32 rows (ResNet's 2048 -> 1000 head at the reference's precision): the
// generic fp32 conv GEMM ran it as 64x64 tiles split-K 8 plus a reduce and a softmax launch (~22 us at
// bs=32).  Here block (column group, K slice): 4 waves x 16 columns, both 16-row M fragments, the K
// slice in steps of 16 on v_mfma_f32_16x16x4_f32 (lane group q supplies k = 16h + 4q + s to step s for
// both operands, one float4 load each); fp32 partials [KS][M][N] go to the finish kernels above
// (bias, logits, softmax).  w: pack_conv_f32 layout [Npad][Kpad], zero-padded.
constexpr int DHF_KSL = 128;                 // K per slice
__global__ __launch_bounds__(256) void dense_partial_f32_kernel(const float* __restrict__ x,
                                                                const float* __restrict__ w, float* __restrict__ part,
                                                                int M, int N, int K, int Kpad) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r = lane & 15, q = lane >> 4;
  const int n = blockIdx.x * 64 + wv * 16 + r;
  const int k0 = blockIdx.y * DHF_KSL, k1 = min(Kpad, k0 + DHF_KSL);
  const float* wr = w + (size_t)n * Kpad + 4 * q;
  f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  if (k1 - k0 == DHF_KSL && k1 <= K) {
    // a whole slice (the ImageNet head: every slice): all 8 weight and 16 activation loads issued before the
    // first MFMA -- one memory latency per block instead of one per unrolled group of K steps
    constexpr int ST = DHF_KSL / 16;
    f32x4 b[ST], a[ST][2];
#pragma unroll
    for (int i = 0; i < ST; ++i) {
      b[i] = *(const f32x4*)(wr + k0 + 16 * i);
#pragma unroll
      for (int mf = 0; mf < 2; ++mf) {
        const int row = mf * 16 + r;
        a[i][mf] = row < M ? *(const f32x4*)(x + (size_t)row * K + k0 + 16 * i + 4 * q) : (f32x4){0.f, 0.f, 0.f, 0.f};
      }
    }
#pragma unroll
    for (int i = 0; i < ST; ++i)
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
        for (int mf = 0; mf < 2; ++mf)
          acc[mf] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][mf][s4], b[i][s4], acc[mf], 0, 0, 0);
  } else {
#pragma unroll 4
  for (int k = k0; k < k1; k += 16) {
    const f32x4 b = *(const f32x4*)(wr + k);
    f32x4 a[2];
#pragma unroll
    for (int mf = 0; mf < 2; ++mf) {
      const int row = mf * 16 + r;
      a[mf] = (row < M && k + 4 * q < K) ? *(const f32x4*)(x + (size_t)row * K + k + 4 * q)
                                         : (f32x4){0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
      for (int mf = 0; mf < 2; ++mf) acc[mf] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[mf][s4], b[s4], acc[mf], 0, 0, 0);
  }
  }
  // acc[mf][e] = C[row mf*16 + 4q + e][column n]
  if (n >= N) return;
  float* pr = part + (size_t)blockIdx.y * M * N;
#pragma unroll
  for (int mf = 0; mf < 2; ++mf)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = mf * 16 + 4 * q + e;
      if (row < M) pr[(size_t)row * N + n] = acc[mf][e];
    }
}

int dense_small_f32_kslices(int Kpad) { return (Kpad + DHF_KSL - 1) / DHF_KSL; }

hipError_t dense_small_f32(const float* x, const float* w, const float* bias, float* part, float* logits,
                           float* probs, int M, int N, int K, int Kpad, hipStream_t s) {
  if (M < 1 || M > 32 || K % 4 || Kpad % 16 || Kpad < K || N < 1) return hipErrorInvalidValue;
  const int ks = dense_small_f32_kslices(Kpad);
  hipLaunchKernelGGL(dense_partial_f32_kernel, dim3((N + 63) / 64, ks), dim3(256), 0, s, x, w, part, M, N, K, Kpad);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (N <= 1024)
    hipLaunchKernelGGL(dense_finish_reg_kernel, dim3(M), dim3(256), 0, s, part, bias, logits, probs, M, N, ks);
  else
    hipLaunchKernelGGL(dense_finish_kernel, dim3(M), dim3(256), (size_t)N * sizeof(float), s, part, bias, logits,
                       probs, M, N, ks);
  return hipGetLastError();
}

hipError_t dense_small(const bf16* x, const bf16* w, const float* bias, float* part, float* logits, float* probs,
                       int M, int N, int K, int Kpad, hipStream_t s) {
  if (M < 1 || M > 32 || K % 8 || N < 1) return hipErrorInvalidValue;
  const int ks = dense_small_kslices(K);
  dim3 grid((N + 15) / 16, ks);
  hipLaunchKernelGGL(dense_partial_kernel, grid, dim3(64), 0, s, x, w, part, M, N, K, Kpad, DH_MAXK);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (N <= 1024)
    hipLaunchKernelGGL(dense_finish_reg_kernel, dim3(M), dim3(256), 0, s, part, bias, logits, probs, M, N, ks);
  else
    hipLaunchKernelGGL(dense_finish_kernel, dim3(M), dim3(256), (size_t)N * sizeof(float), s, part, bias, logits,
                       probs, M, N, ks);
  return hipGetLastError();
}

}  // namespace adapt
