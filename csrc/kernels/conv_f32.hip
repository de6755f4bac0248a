// fp32 execution path: implicit-GEMM convolution / GEMM on the fp32 matrix
// cores (v_mfma_f32_16x16x4_f32) plus the fp32 pooling / element-wise kernels
// a ResNet slice needs.  This is the reference's precision: Keras runs the
// whole model in float32 (`src/node.py:177`, `test/local_infer.py:22`).
//
//   out[m][n] = act( sum_k X[m][k] * W[n][k] + bias[n] (+ res[m][n]) )
//
// m = (img, oh, ow) over the NHWC output, n = output channel, k = (kh, kw, ci)
// with ci innermost; weights packed [Npad][Kpad] fp32 (BN folded on the host).
//
// Tiling (BM x BN x 32 per block, 4 waves on a WM x WN grid, wave tile TM x TN):
// * the K permutation trick: an MFMA 16x16x4 takes k-slot q (q = lane / 16)
//   from every lane group; over the 4 MFMAs of one 16-wide K half, lane group q
//   supplies k = 4q + s at step s.  A and B use the same permutation, so the
//   sum is the plain dot product and each lane fetches ONE float4 per fragment
//   row per K half (ds_read_b128) instead of four scalar reads;
// * K tiles of 32 (two halves per barrier: twice the MFMA work between
//   barriers of the 16-wide v1, which left the loads' latency exposed);
// * LDS rows of 32 floats (128 B), float4 chunk index XOR-swizzled with
//   (row >> 1) & 7: the 16 rows a 16-lane group reads land on 16 distinct
//   16-byte slots of the 256-byte bank row;
// * register-prefetch double buffer: the next K tile is loaded from global
//   while the MFMAs of this one run, one barrier per K tile;
// * epilogue straight from the accumulators: for each of its 4 rows a 16-lane
//   group writes 16 consecutive floats (64 B) of the output row;
// * split-K: fp32 partial slabs + a reduce launch that applies the epilogue.
#include "kernels.h"
#include <algorithm>
#include <cstdint>
#include <initializer_list>

namespace adapt {

namespace {

constexpr int FBK = 32;          // fp32 elements per K tile (8 float4 chunks)
constexpr int FCH = FBK / 4;
constexpr int FNT = 256;

__device__ __forceinline__ int fswz(int r, int c) { return r * FBK + ((c ^ ((r >> 1) & 7)) << 2); }

// TAPK: Cin % FBK == 0, so a K tile never straddles a filter tap: the tap and
// its first channel are computed once per tile (wave-uniform), not per chunk
template <int BM, int BN, int WM, int WN, bool PURE, bool VEC, bool TAPK>
__global__ __launch_bounds__(FNT, 2) void conv_f32_kernel(ConvF32Params p) {
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16;
  constexpr int ACH = BM * FCH / FNT, BCH = BN * FCH / FNT;  // float4 chunks per thread per K tile
  static_assert(WM * WN == 4 && ACH >= 1 && BCH >= 1, "tile");
  __shared__ __attribute__((aligned(16))) float sa[2][BM * FBK];
  __shared__ __attribute__((aligned(16))) float sb[2][BN * FBK];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int tilesN = (p.N + BN - 1) / BN, tilesM = (p.M + BM - 1) / BM;
  const int tile = xcd_remap(blockIdx.x, tilesM * tilesN);
  const int m0 = (tile / tilesN) * BM, n0 = (tile % tilesN) * BN;
  const int ktiles = p.Kpad / FBK;
  const int kper = (ktiles + p.ksplit - 1) / p.ksplit;
  const int kt0 = blockIdx.y * kper, kt1 = min(ktiles, kt0 + kper);

  // per-thread A rows: chunk c of the tile = (row c / 4, float4 c % 4)
  int a_base[ACH], a_ih0[ACH], a_iw0[ACH];
  const int ohw = p.OH * p.OW;
#pragma unroll
  for (int i = 0; i < ACH; ++i) {
    const int m = m0 + (tid + i * FNT) / FCH;
    if (m < p.M) {
      if (PURE) {
        a_base[i] = m * p.Cin;
        a_ih0[i] = a_iw0[i] = 0;
      } else {
        const int img = m / ohw, r = m - img * ohw, oh = r / p.OW, ow = r - oh * p.OW;
        a_base[i] = img * p.H * p.W * p.Cin;
        a_ih0[i] = oh * p.stride - p.pad_t;
        a_iw0[i] = ow * p.stride - p.pad_l;
      }
    } else {
      a_base[i] = -1;
      a_ih0[i] = -(1 << 28);
      a_iw0[i] = 0;
    }
  }
  f32x4 ra[ACH], rb[BCH];
  const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};

  auto load = [&](int kt) {
    int t_ci0 = 0, t_kh = 0, t_kw = 0;
    if (TAPK) {
      const int kk0 = kt * FBK;
      const int tap = kk0 / p.Cin;
      t_ci0 = kk0 - tap * p.Cin;
      t_kh = tap / p.KW;
      t_kw = tap - t_kh * p.KW;
    }
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      const int c = (tid + i * FNT) % FCH;
      const int k = kt * FBK + c * 4;
      if (TAPK) {
        const int ih = a_ih0[i] + t_kh, iw = a_iw0[i] + t_kw;
        ra[i] = (a_base[i] >= 0 && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W)
                    ? *(const f32x4*)(p.x + a_base[i] + (ih * p.W + iw) * p.Cin + t_ci0 + c * 4) : z4;
        continue;
      }
      if (a_base[i] < 0 || k >= p.K) { ra[i] = z4; continue; }
      if (PURE) {
        ra[i] = *(const f32x4*)(p.x + a_base[i] + k);
      } else if (VEC) {                       // Cin % 4 == 0: 4 consecutive k share one tap
        const int tap = k / p.Cin, ci = k - tap * p.Cin, kh = tap / p.KW, kw = tap - kh * p.KW;
        const int ih = a_ih0[i] + kh, iw = a_iw0[i] + kw;
        ra[i] = ((unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W)
                    ? *(const f32x4*)(p.x + a_base[i] + (ih * p.W + iw) * p.Cin + ci) : z4;
      } else {                                // small Cin (the 3-channel image): element-wise gather
        f32x4 v = z4;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int kk = k + e;
          if (kk < p.K) {
            const int tap = kk / p.Cin, ci = kk - tap * p.Cin, kh = tap / p.KW, kw = tap - kh * p.KW;
            const int ih = a_ih0[i] + kh, iw = a_iw0[i] + kw;
            if ((unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W)
              v[e] = p.x[a_base[i] + (ih * p.W + iw) * p.Cin + ci];
          }
        }
        ra[i] = v;
      }
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int c = tid + i * FNT, row = c / FCH, ch = c % FCH;
      rb[i] = *(const f32x4*)(p.w + (size_t)(n0 + row) * p.Kpad + kt * FBK + ch * 4);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      const int c = tid + i * FNT;
      *(f32x4*)(&sa[buf][fswz(c / FCH, c % FCH)]) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int c = tid + i * FNT;
      *(f32x4*)(&sb[buf][fswz(c / FCH, c % FCH)]) = rb[i];
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = z4;
  const int fr = lane & 15, fq = lane >> 4;

  // the residual this lane adds in the epilogue, requested before the K loop so
  // its latency hides under the MFMAs (read one by one after the loop, each of
  // the FM*FN*4 loads was a serial round trip: the fp32 "_out" convs spent most
  // of their time there)
  const bool pre_res = p.res != nullptr && p.ksplit == 1;
  f32x4 rres[FM][FN];
  if (pre_res) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + wn * TN + j * 16 + fr;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * TM + i * 16 + fq * 4 + r;
          rres[i][j][r] = (n < p.N && m < p.M) ? p.res[(size_t)m * p.N + n] : 0.f;
        }
    }
  }

  if (kt0 < kt1) {
    load(kt0);
    store(0);
    __syncthreads();
    int buf = 0;
    for (int kt = kt0; kt < kt1; ++kt) {
      const bool more = kt + 1 < kt1;
      if (more) load(kt + 1);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        f32x4 af[FM], bfr[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) af[i] = *(const f32x4*)(&sa[buf][fswz(wm * TM + i * 16 + fr, h * 4 + fq)]);
#pragma unroll
        for (int j = 0; j < FN; ++j) bfr[j] = *(const f32x4*)(&sb[buf][fswz(wn * TN + j * 16 + fr, h * 4 + fq)]);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i][s], bfr[j][s], acc[i][j], 0, 0, 0);
      }
      if (more) store(buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
  }

  // epilogue from registers: acc[i][j][r] = C[row = wm*TM + i*16 + fq*4 + r][col = wn*TN + j*16 + fr]
  float* slab = p.ksplit > 1 ? p.ws + (size_t)blockIdx.y * p.M * p.N : nullptr;
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = n0 + wn * TN + j * 16 + fr;
    if (n >= p.N) continue;
    const float b = (slab == nullptr && p.bias) ? p.bias[n] : 0.f;
    const F32Dst d = f32_dst(p, n);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * TM + i * 16 + fq * 4 + r;
        if (m >= p.M) continue;
        const size_t o = (size_t)m * p.N + n;
        float v = acc[i][j][r];
        if (slab) {
          slab[o] = v;
          continue;
        }
        v += b;
        if (pre_res) v += rres[i][j][r];
        d.base[(size_t)m * d.ld + d.col] = act_relu(v, d.relu);
      }
  }
}

__global__ __launch_bounds__(256) void splitk_reduce_f32(ConvF32Params p) {
  const size_t total = (size_t)p.M * p.N;
  for (size_t o = blockIdx.x * (size_t)blockDim.x + threadIdx.x; o < total; o += (size_t)gridDim.x * blockDim.x) {
    float v = 0.f;
    for (int s = 0; s < p.ksplit; ++s) v += p.ws[(size_t)s * total + o];
    const int n = (int)(o % p.N);
    if (p.bias) v += p.bias[n];
    if (p.res) v += p.res[o];
    const F32Dst d = f32_dst(p, n);
    d.base[(o / p.N) * d.ld + d.col] = act_relu(v, d.relu);
  }
}

template <int BM, int BN, int WM, int WN>
hipError_t launch_f32(const ConvF32Params& p, bool pure, bool vec, hipStream_t s) {
  dim3 grid(((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN), p.ksplit), block(FNT);
  if (pure) hipLaunchKernelGGL((conv_f32_kernel<BM, BN, WM, WN, true, true, false>), grid, block, 0, s, p);
  else if (vec && p.Cin % FBK == 0)
    hipLaunchKernelGGL((conv_f32_kernel<BM, BN, WM, WN, false, true, true>), grid, block, 0, s, p);
  else if (vec) hipLaunchKernelGGL((conv_f32_kernel<BM, BN, WM, WN, false, true, false>), grid, block, 0, s, p);
  else hipLaunchKernelGGL((conv_f32_kernel<BM, BN, WM, WN, false, false, false>), grid, block, 0, s, p);
  return hipGetLastError();
}

}  // namespace

// fp32 tile configs (index -> BM, BN, WM, WN); ops/conv.py F32_TILES mirrors this
#define ADAPT_F32_CFGS(X) \
  X(0, 128, 128, 2, 2)    \
  X(1, 128, 64, 2, 2)     \
  X(2, 64, 128, 2, 2)     \
  X(3, 64, 64, 2, 2)      \
  X(4, 256, 64, 4, 1)     \
  X(5, 64, 256, 1, 4)

hipError_t conv_f32_forward(const float* x, const float* w, const float* bias, const float* res, float* out,
                            float* ws, int B, int H, int W, int Cin, int OH, int OW, int N, int KH, int KW,
                            int stride, int pad_t, int pad_l, int K, int Kpad, int relu, int ksplit, int cfg,
                            hipStream_t s, int* counters, float* out2, int n_split, int relu2) {
  ConvF32Params p{x, w, bias, res, out, ws, B, H, W, Cin, OH, OW, N, KH, KW, stride, pad_t, pad_l,
                  B * OH * OW, K, Kpad, relu, ksplit == 0 ? 1 : ksplit, counters, 0, out2, n_split, relu2};
  if (Kpad % FBK || (p.ksplit > 1 && ws == nullptr)) return hipErrorInvalidValue;
  if (n_split && (n_split % 4 || n_split >= N || !out2 || res || (cfg >= 80 && cfg < 300))) return hipErrorInvalidValue;
  if (cfg >= 300) return gemm_f32s_launch(p, cfg, s);   // big-tile 1x1 GEMM (gemm_f32s.hip)
  if (p.ksplit < 0 && cfg < 80) {
    // stream-K: v2 configs only
    int bm, bn, g;
    if (!conv_f32g_ok(cfg, Cin, N) || !conv_f32g_cfg_tile(cfg, &bm, &bn) || !ws || !counters)
      return hipErrorInvalidValue;
    conv_f32g_sk_plan(((p.M + bm - 1) / bm) * ((N + bn - 1) / bn), Kpad / FBK, -p.ksplit, &g, &p.sk_iters);
  }
  const bool pure = KH == 1 && KW == 1 && stride == 1 && pad_t == 0 && pad_l == 0 && H == OH && W == OW &&
                    Cin % 4 == 0;
  const bool vec = Cin % 4 == 0;
  hipError_t e = hipErrorInvalidValue;
  if (p.ksplit < 1 && cfg < 10) return hipErrorInvalidValue;
  switch (cfg) {
#define X(id, BM_, BN_, WM_, WN_) case id: e = launch_f32<BM_, BN_, WM_, WN_>(p, pure, vec, s); break;
    ADAPT_F32_CFGS(X)
#undef X
    default:
      if (cfg >= 200) return hipErrorInvalidValue;   // F(4x4): wino4s_forward (its own entry point)
      if (cfg >= 80) {
        // Winograd F(2x2, 3x3) (conv_wino_f32.hip): w is the transformed, fragment-packed weight tensor
        // ksplit <= -100: stream-K over (-ksplit - 100) x 256 blocks; -100 < ksplit < 0: split -ksplit
        // ways with the fixup fused into the kernel; both need ws + counters
        if (KH != 3 || KW != 3 || stride != 1 || pad_t != 1 || pad_l != 1 || OH != H || OW != W ||
            p.ksplit == 0 || p.ksplit == -1 || !conv_wino_f32_ok(cfg, Cin, N) ||
            (p.ksplit < 0 && (!ws || !counters)))
          return hipErrorInvalidValue;
        const int th = (H + 1) / 2, tw = (W + 1) / 2;
        const bool sk = p.ksplit <= -100;
        WinoF32Params wp{x, w, bias, res, out, ws, B, H, W, Cin, N, th, tw, B * th * tw, relu,
                         sk ? 1 : (p.ksplit < 0 ? -p.ksplit : p.ksplit), p.ksplit < 0 ? counters : nullptr, 0,
                         sk ? -p.ksplit - 100 : 0};
        if (sk) {
          int nw = 0, fn = 0;
          if (!conv_wino_f32_cfg(cfg, &nw, &fn)) return hipErrorInvalidValue;
          int G, iters, smax;
          conv_wino_sk_plan(((wp.T + 16 * nw - 1) / (16 * nw)) * (N / (16 * fn)), Cin / 16, wp.sk_mult, &G, &iters,
                            &smax);
          wp.sk_iters = iters;
        }
        e = conv_wino_f32_launch(wp, cfg, s);
        break;
      }
      // v2: LDS-DMA ring (conv_f32g.hip); tap-major walk needs Cin % 32 == 0
      if (!conv_f32g_ok(cfg, Cin, N)) return hipErrorInvalidValue;
      e = conv_f32g_launch(p, cfg, pure, s);
  }
  if (e != hipSuccess || p.ksplit <= 1) return e;
  size_t total = (size_t)p.M * p.N;
  int blocks = (int)((total + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(splitk_reduce_f32, dim3(blocks), dim3(256), 0, s, p);
  return hipGetLastError();
}

// ------------------------------------------------------------- fp32 layers
namespace {

__global__ __launch_bounds__(256) void maxpool_f32_kernel(const float* __restrict__ x, float* __restrict__ y, int B,
                                                          int H, int W, int C, int OH, int OW, int K, int S,
                                                          int pad_t, int pad_l, int pad_zero) {
  const int C4 = C / 4;
  const size_t total = (size_t)B * OH * OW * C4;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int c4 = (int)(i % C4);
    size_t r = i / C4;
    const int ow = (int)(r % OW);
    r /= OW;
    const int oh = (int)(r % OH);
    const int b = (int)(r / OH);
    f32x4 m = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    bool padded = false;
    for (int kh = 0; kh < K; ++kh) {
      const int ih = oh * S - pad_t + kh;
      for (int kw = 0; kw < K; ++kw) {
        const int iw = ow * S - pad_l + kw;
        if ((unsigned)ih >= (unsigned)H || (unsigned)iw >= (unsigned)W) {
          padded = true;
          continue;
        }
        const f32x4 v = *(const f32x4*)(x + (((size_t)b * H + ih) * W + iw) * C + c4 * 4);
        m[0] = fmaxf(m[0], v[0]); m[1] = fmaxf(m[1], v[1]); m[2] = fmaxf(m[2], v[2]); m[3] = fmaxf(m[3], v[3]);
      }
    }
    if (padded && pad_zero) {               // a ZeroPadding2D before the pool: the zeros take part
      m[0] = fmaxf(m[0], 0.f); m[1] = fmaxf(m[1], 0.f); m[2] = fmaxf(m[2], 0.f); m[3] = fmaxf(m[3], 0.f);
    }
    *(f32x4*)(y + i * 4) = m;
  }
}

// y[b][c] = mean over HW of x[b][hw][c]; one thread per (b, 4 channels)
// GAP over small maps (ResNet's 7x7x2048 head): one thread per (image, float4 channel chunk)
// walking all HW pixels made 64 blocks of 49 dependent loads (14 us at bs=32).  Here a block
// owns 64 float4 channel chunks of one image with GP = 4 threads per chunk: thread (g, c) sums
// pixels g, g + GP, ... of chunk c (independent loads), and the GP partials meet in LDS.
constexpr int GAP_CC = 64;                   // float4 channel chunks per block
constexpr int GAP_GP = 4;                    // pixel groups per chunk
__global__ __launch_bounds__(GAP_CC * GAP_GP) void gap_f32_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                                   int B, int HW, int C) {
  __shared__ f32x4 red[GAP_GP][GAP_CC];
  const int C4 = C / 4;
  const int cblocks = (C4 + GAP_CC - 1) / GAP_CC;
  const int b = blockIdx.x / cblocks, c4 = (blockIdx.x - b * cblocks) * GAP_CC + (threadIdx.x % GAP_CC);
  const int g = threadIdx.x / GAP_CC;
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  if (c4 < C4) {
    const float* p = x + (size_t)b * HW * C + c4 * 4;
#pragma unroll 4
    for (int t = g; t < HW; t += GAP_GP) s += *(const f32x4*)(p + (size_t)t * C);
  }
  red[g][threadIdx.x % GAP_CC] = s;
  __syncthreads();
  if (g == 0 && c4 < C4) {
#pragma unroll
    for (int k = 1; k < GAP_GP; ++k) s += red[k][threadIdx.x];
    *(f32x4*)(y + (size_t)b * C + c4 * 4) = s * (1.f / (float)HW);
  }
}

// GAP over large maps (the squeeze-excite pools of EfficientNet run over up to
// 112x112 pixels: one thread per channel chunk walking every pixel left most
// of the chip idle): pass 1, grid (S pixel slices, B); a block sums its slice
// for up to 256 float4 channel chunks (the other threads stride the pixels)
// and reduces in LDS; pass 2 adds the S partials and divides by HW.
__global__ __launch_bounds__(256) void gap_part_f32_kernel(const float* __restrict__ x, float* __restrict__ part,
                                                           int HW, int C, int S) {
  __shared__ f32x4 red[256];
  const int b = blockIdx.y, sl = blockIdx.x;
  const int C4 = C / 4;
  const int p0 = (int)((long long)HW * sl / S), p1 = (int)((long long)HW * (sl + 1) / S);
  for (int cg = 0; cg < C4; cg += 256) {
    const int nc = min(256, C4 - cg);
    const int lanes = 256 / nc;
    const int ch = threadIdx.x % nc, pl = threadIdx.x / nc;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if (pl < lanes) {
      const float* base = x + (size_t)b * HW * C + (size_t)(cg + ch) * 4;
      for (int q = p0 + pl; q < p1; q += lanes) acc += *(const f32x4*)(base + (size_t)q * C);
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x < nc) {
      f32x4 sum = {0.f, 0.f, 0.f, 0.f};
      for (int l = 0; l < lanes; ++l) sum += red[l * nc + threadIdx.x];
      *(f32x4*)(part + ((size_t)b * S + sl) * C + (size_t)(cg + threadIdx.x) * 4) = sum;
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void gap_finish_f32_kernel(const float* __restrict__ part, float* __restrict__ y,
                                                             int B, int HW, int C, int S) {
  const size_t total = (size_t)B * C;
  const float inv = 1.f / (float)HW;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const size_t b = i / C, c = i % C;
    float sum = 0.f;
    for (int sl = 0; sl < S; ++sl) sum += part[(b * S + sl) * C + c];
    y[i] = sum * inv;
  }
}

// elementwise fp32: mode 0 add(+act) a+b, 1 bn affine y = x*scale[c]+shift[c] (+act), 2 act only
__global__ __launch_bounds__(256) void eltwise_f32_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                          const float* __restrict__ scale,
                                                          const float* __restrict__ shift, float* __restrict__ y,
                                                          size_t n4, int C, int op, int relu) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    f32x4 v = *(const f32x4*)(a + i * 4);
    if (op == 0) {
      v += *(const f32x4*)(b + i * 4);
    } else if (op == 1) {
      const int c = (int)((i * 4) % C);
      v[0] = v[0] * scale[c] + shift[c];
      v[1] = v[1] * scale[c + 1] + shift[c + 1];
      v[2] = v[2] * scale[c + 2] + shift[c + 2];
      v[3] = v[3] * scale[c + 3] + shift[c + 3];
    }
    v[0] = act_relu(v[0], relu); v[1] = act_relu(v[1], relu);
    v[2] = act_relu(v[2], relu); v[3] = act_relu(v[3], relu);
    *(f32x4*)(y + i * 4) = v;
  }
}

// ---- the other families' layers (MobileNetV2 / EfficientNet / DenseNet / InceptionV3) in fp32:
// plain element-per-thread kernels over the true channel count (fp32 activations carry no padding)

// depthwise conv, multiplier 1, BN folded: y[b][oh][ow][c] = act(sum x * w[kh][kw][c] + bias[c])
template <bool GEN>
__global__ __launch_bounds__(256) void dwconv_f32_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                         const float* __restrict__ bias, float* __restrict__ y,
                                                         int B, int H, int W, int C, int OH, int OW, int KH, int KW,
                                                         int S, int pad_t, int pad_l, int act, float alpha) {
  const size_t total = (size_t)B * OH * OW * C;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    size_t r = i / C;
    const int ow = (int)(r % OW);
    r /= OW;
    const int oh = (int)(r % OH);
    const int b = (int)(r / OH);
    float acc = bias ? bias[c] : 0.f;
    for (int kh = 0; kh < KH; ++kh) {
      const int ih = oh * S - pad_t + kh;
      if ((unsigned)ih >= (unsigned)H) continue;
      for (int kw = 0; kw < KW; ++kw) {
        const int iw = ow * S - pad_l + kw;
        if ((unsigned)iw >= (unsigned)W) continue;
        acc = fmaf(x[(((size_t)b * H + ih) * W + iw) * C + c], w[(kh * KW + kw) * C + c], acc);
      }
    }
    y[i] = actx<GEN>(acc, act, alpha);
  }
}

// average pool, padding excluded from the count (Keras)
__global__ __launch_bounds__(256) void avgpool_f32_kernel(const float* __restrict__ x, float* __restrict__ y, int B,
                                                          int H, int W, int C, int OH, int OW, int KH, int KW, int S,
                                                          int pad_t, int pad_l) {
  const size_t total = (size_t)B * OH * OW * C;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    size_t r = i / C;
    const int ow = (int)(r % OW);
    r /= OW;
    const int oh = (int)(r % OH);
    const int b = (int)(r / OH);
    float acc = 0.f;
    int n = 0;
    for (int kh = 0; kh < KH; ++kh) {
      const int ih = oh * S - pad_t + kh;
      if ((unsigned)ih >= (unsigned)H) continue;
      for (int kw = 0; kw < KW; ++kw) {
        const int iw = ow * S - pad_l + kw;
        if ((unsigned)iw >= (unsigned)W) continue;
        acc += x[(((size_t)b * H + ih) * W + iw) * C + c];
        ++n;
      }
    }
    y[i] = n ? acc / (float)n : 0.f;
  }
}

// one input of a channel concat: y[p][off + c] = x[p][c]
__global__ __launch_bounds__(256) void concat_f32_kernel(const float* __restrict__ x, int Cx, float* __restrict__ y,
                                                         int Cy, int off, size_t pixels) {
  const size_t total = pixels * Cx;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const size_t p = i / Cx;
    y[p * Cy + off + (i - p * Cx)] = x[i];
  }
}

// y = act(a <op> b) (BinOp codes of layers.hip); b is a's shape or one [C] row per image (bcast_hw pixels)
template <bool GEN>
__global__ __launch_bounds__(256) void binary_f32_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                         float* __restrict__ y, size_t n, int C, int bcast_hw, int op,
                                                         int act) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    size_t bi = i;
    if (bcast_hw) {
      const size_t pix = i / C;
      bi = (pix / bcast_hw) * C + (i % C);
    }
    const float p = a[i], q = b[bi];
    float r;
    switch (op) {
      case 1: r = p - q; break;
      case 2: r = p * q; break;
      case 3: r = fmaxf(p, q); break;
      case 4: r = fminf(p, q); break;
      case 5: r = 0.5f * (p + q); break;
      default: r = p + q;
    }
    y[i] = actx<GEN>(r, act);
  }
}

// y = act(x * scale[c] + shift[c]) (scale null: y = act(x)); any channel count
template <bool GEN>
__global__ __launch_bounds__(256) void affine_act_f32_kernel(const float* __restrict__ x,
                                                             const float* __restrict__ scale,
                                                             const float* __restrict__ shift, float* __restrict__ y,
                                                             size_t n, int C, int act, float alpha) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    float v = x[i];
    if (scale) {
      const int c = (int)(i % C);
      v = v * scale[c] + shift[c];
    }
    y[i] = actx<GEN>(v, act, alpha);
  }
}

// ---- the same layers four channels per thread (every family's channel counts are multiples of 4): one
// 16-byte load / store per tap and 32-bit index math; the launchers take these whenever C % 4 == 0 and the
// tensor indexes in 32 bits, the scalar kernels above otherwise

template <bool GEN>
__device__ __forceinline__ f32x4 actx4(f32x4 v, int mode, float alpha = 0.3f) {
  v[0] = actx<GEN>(v[0], mode, alpha); v[1] = actx<GEN>(v[1], mode, alpha);
  v[2] = actx<GEN>(v[2], mode, alpha); v[3] = actx<GEN>(v[3], mode, alpha);
  return v;
}

template <bool GEN, int K>
__global__ __launch_bounds__(256) void dwconv_f32v_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                          const float* __restrict__ bias, float* __restrict__ y,
                                                          int B, int H, int W, int C, int OH, int OW, int KH, int KW,
                                                          int S, int pad_t, int pad_l, int act, float alpha) {
  if constexpr (K > 0) { KH = K; KW = K; }
  const int C4 = C >> 2;
  const unsigned total = (unsigned)B * OH * OW * C4;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int c4 = (int)(i % C4);
    unsigned r = i / C4;
    const int ow = (int)(r % OW);
    r /= OW;
    const int oh = (int)(r % OH);
    const int b = (int)(r / OH);
    f32x4 acc = bias ? *(const f32x4*)(bias + c4 * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
    const float* xb = x + (unsigned)b * H * W * C + c4 * 4;
#pragma unroll
    for (int kh = 0; kh < (K > 0 ? K : KH); ++kh) {
      const int ih = oh * S - pad_t + kh;
      if ((unsigned)ih >= (unsigned)H) continue;
#pragma unroll
      for (int kw = 0; kw < (K > 0 ? K : KW); ++kw) {
        const int iw = ow * S - pad_l + kw;
        if ((unsigned)iw >= (unsigned)W) continue;
        const f32x4 xv = *(const f32x4*)(xb + (unsigned)(ih * W + iw) * C);
        const f32x4 wv = *(const f32x4*)(w + (kh * KW + kw) * C + c4 * 4);
        acc += xv * wv;
      }
    }
    *(f32x4*)(y + i * 4) = actx4<GEN>(acc, act, alpha);
  }
}

__global__ __launch_bounds__(256) void avgpool_f32v_kernel(const float* __restrict__ x, float* __restrict__ y, int B,
                                                           int H, int W, int C, int OH, int OW, int KH, int KW, int S,
                                                           int pad_t, int pad_l) {
  const int C4 = C >> 2;
  const unsigned total = (unsigned)B * OH * OW * C4;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int c4 = (int)(i % C4);
    unsigned r = i / C4;
    const int ow = (int)(r % OW);
    r /= OW;
    const int oh = (int)(r % OH);
    const int b = (int)(r / OH);
    const int h0 = max(oh * S - pad_t, 0), h1 = min(oh * S - pad_t + KH, H);
    const int w0 = max(ow * S - pad_l, 0), w1 = min(ow * S - pad_l + KW, W);
    const float* xb = x + (unsigned)b * H * W * C + c4 * 4;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int ih = h0; ih < h1; ++ih)
      for (int iw = w0; iw < w1; ++iw) acc += *(const f32x4*)(xb + (unsigned)(ih * W + iw) * C);
    const int n = (h1 - h0) * (w1 - w0);
    *(f32x4*)(y + i * 4) = n > 0 ? acc * (1.f / (float)n) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
}

__global__ __launch_bounds__(256) void concat_f32v_kernel(const float* __restrict__ x, int Cx, float* __restrict__ y,
                                                          int Cy, int off, unsigned pixels) {
  const int C4 = Cx >> 2;
  const unsigned total = pixels * C4;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const unsigned p = i / C4;
    *(f32x4*)(y + p * Cy + off + (i - p * C4) * 4) = *(const f32x4*)(x + i * 4);
  }
}

template <bool GEN>
__global__ __launch_bounds__(256) void binary_f32v_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                          float* __restrict__ y, unsigned n4, int C, int bcast_hw,
                                                          int op, int act) {
  const int C4 = C >> 2;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x) {
    unsigned bi = i;
    if (bcast_hw) {
      const unsigned pix = i / C4;
      bi = (pix / bcast_hw) * C4 + (i - pix * C4);
    }
    const f32x4 p = *(const f32x4*)(a + i * 4), q = *(const f32x4*)(b + bi * 4);
    f32x4 r;
    switch (op) {
      case 1: r = p - q; break;
      case 2: r = p * q; break;
      case 3: for (int j = 0; j < 4; ++j) r[j] = fmaxf(p[j], q[j]); break;
      case 4: for (int j = 0; j < 4; ++j) r[j] = fminf(p[j], q[j]); break;
      case 5: r = 0.5f * (p + q); break;
      default: r = p + q;
    }
    *(f32x4*)(y + i * 4) = actx4<GEN>(r, act);
  }
}

template <bool GEN>
__global__ __launch_bounds__(256) void affine_act_f32v_kernel(const float* __restrict__ x,
                                                              const float* __restrict__ scale,
                                                              const float* __restrict__ shift, float* __restrict__ y,
                                                              unsigned n4, int C, int act, float alpha) {
  const int C4 = C >> 2;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x) {
    f32x4 v = *(const f32x4*)(x + i * 4);
    if (scale) {
      const int c = (int)(i % C4) * 4;
      v = v * *(const f32x4*)(scale + c) + *(const f32x4*)(shift + c);
    }
    *(f32x4*)(y + i * 4) = actx4<GEN>(v, act, alpha);
  }
}

// 16-byte paths need 16-byte aligned bases and a 32-bit index space
bool vec_ok(std::initializer_list<const void*> ps, size_t n) {
  if (n >= (size_t(1) << 31)) return false;
  for (const void* p : ps)
    if (reinterpret_cast<uintptr_t>(p) & 15) return false;
  return true;
}

__global__ __launch_bounds__(256) void pad_f32_kernel(const float* __restrict__ x, float* __restrict__ y, int B, int H,
                                                      int W, int C, int OH, int OW, int pad_t, int pad_l) {
  const size_t total = (size_t)B * OH * OW * C;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    size_t r = i / C;
    const int ow = (int)(r % OW);
    r /= OW;
    const int oh = (int)(r % OH);
    const int b = (int)(r / OH);
    const int ih = oh - pad_t, iw = ow - pad_l;
    y[i] = ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W) ? x[(((size_t)b * H + ih) * W + iw) * C + c]
                                                                       : 0.f;
  }
}

int grid_for(size_t n) {
  size_t b = (n + 255) / 256;
  return (int)(b > 8192 ? 8192 : (b ? b : 1));
}

}  // namespace

hipError_t maxpool_f32(const float* x, float* y, int B, int H, int W, int C, int OH, int OW, int K, int S, int pad_t,
                       int pad_l, int pad_zero, hipStream_t s) {
  if (C % 4) return hipErrorInvalidValue;
  hipLaunchKernelGGL(maxpool_f32_kernel, dim3(grid_for((size_t)B * OH * OW * C / 4)), dim3(256), 0, s, x, y, B, H, W,
                     C, OH, OW, K, S, pad_t, pad_l, pad_zero);
  return hipGetLastError();
}

hipError_t gap_f32(const float* x, float* y, int B, int HW, int C, hipStream_t s) {
  if (C % 4) return hipErrorInvalidValue;
  const int cblocks = (C / 4 + GAP_CC - 1) / GAP_CC;
  hipLaunchKernelGGL(gap_f32_kernel, dim3(B * cblocks), dim3(GAP_CC * GAP_GP), 0, s, x, y, B, HW, C);
  return hipGetLastError();
}

hipError_t gap_large_f32(const float* x, float* y, float* part, int B, int HW, int C, hipStream_t s) {
  if (C % 4) return hipErrorInvalidValue;
  const int S = gap_large_slices(B, HW);
  hipLaunchKernelGGL(gap_part_f32_kernel, dim3(S, B), dim3(256), 0, s, x, part, HW, C, S);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(gap_finish_f32_kernel, dim3(grid_for((size_t)B * C)), dim3(256), 0, s, part, y, B, HW, C, S);
  return hipGetLastError();
}

hipError_t eltwise_f32(const float* a, const float* b, const float* scale, const float* shift, float* y, size_t n,
                       int C, int op, int relu, hipStream_t s) {
  if (n % 4 || C % 4) return hipErrorInvalidValue;
  hipLaunchKernelGGL(eltwise_f32_kernel, dim3(grid_for(n / 4)), dim3(256), 0, s, a, b, scale, shift, y, n / 4, C, op,
                     relu);
  return hipGetLastError();
}

hipError_t pad_f32(const float* x, float* y, int B, int H, int W, int C, int OH, int OW, int pad_t, int pad_l,
                   hipStream_t s) {
  hipLaunchKernelGGL(pad_f32_kernel, dim3(grid_for((size_t)B * OH * OW * C)), dim3(256), 0, s, x, y, B, H, W, C, OH,
                     OW, pad_t, pad_l);
  return hipGetLastError();
}

hipError_t dwconv_f32(const float* x, const float* w, const float* bias, float* y, int B, int H, int W, int C, int OH,
                      int OW, int KH, int KW, int S, int pad_t, int pad_l, int act, float alpha, hipStream_t s) {
  const size_t n = (size_t)B * OH * OW * C;
  if (C % 4 == 0 && vec_ok({x, w, bias, y}, std::max(n, (size_t)B * H * W * C))) {
    const dim3 gv(grid_for(n / 4));
#define DWV(G, K)                                                                                                     \
  hipLaunchKernelGGL((dwconv_f32v_kernel<G, K>), gv, dim3(256), 0, s, x, w, bias, y, B, H, W, C, OH, OW, KH, KW, S, \
                     pad_t, pad_l, act, alpha)
    const int k = (KH == KW && (KH == 3 || KH == 5)) ? KH : 0;
    const bool gen = act > ACT_RELU6;
    if (k == 3) { if (gen) DWV(true, 3); else DWV(false, 3); }
    else if (k == 5) { if (gen) DWV(true, 5); else DWV(false, 5); }
    else { if (gen) DWV(true, 0); else DWV(false, 0); }
#undef DWV
    return hipGetLastError();
  }
  const dim3 g(grid_for(n));
  if (act > ACT_RELU6)
    hipLaunchKernelGGL(dwconv_f32_kernel<true>, g, dim3(256), 0, s, x, w, bias, y, B, H, W, C, OH, OW, KH, KW, S, pad_t,
                       pad_l, act, alpha);
  else
    hipLaunchKernelGGL(dwconv_f32_kernel<false>, g, dim3(256), 0, s, x, w, bias, y, B, H, W, C, OH, OW, KH, KW, S, pad_t,
                       pad_l, act, alpha);
  return hipGetLastError();
}

hipError_t avgpool_f32(const float* x, float* y, int B, int H, int W, int C, int OH, int OW, int KH, int KW, int S,
                       int pad_t, int pad_l, hipStream_t s) {
  const size_t n = (size_t)B * OH * OW * C;
  if (C % 4 == 0 && vec_ok({x, y}, std::max(n, (size_t)B * H * W * C))) {
    hipLaunchKernelGGL(avgpool_f32v_kernel, dim3(grid_for(n / 4)), dim3(256), 0, s, x, y, B, H, W, C, OH, OW, KH, KW, S,
                       pad_t, pad_l);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(avgpool_f32_kernel, dim3(grid_for(n)), dim3(256), 0, s, x, y, B, H, W, C,
                     OH, OW, KH, KW, S, pad_t, pad_l);
  return hipGetLastError();
}

hipError_t concat_f32(const float* x, int Cx, float* y, int Cy, int off, size_t pixels, hipStream_t s) {
  if (off + Cx > Cy) return hipErrorInvalidValue;
  if (Cx % 4 == 0 && Cy % 4 == 0 && off % 4 == 0 && vec_ok({x, y}, pixels * Cy)) {
    hipLaunchKernelGGL(concat_f32v_kernel, dim3(grid_for(pixels * Cx / 4)), dim3(256), 0, s, x, Cx, y, Cy, off,
                       (unsigned)pixels);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(concat_f32_kernel, dim3(grid_for(pixels * Cx)), dim3(256), 0, s, x, Cx, y, Cy, off, pixels);
  return hipGetLastError();
}

hipError_t binary_f32(const float* a, const float* b, float* y, size_t n, int C, int bcast_hw, int op, int act,
                      hipStream_t s) {
  if (C % 4 == 0 && n % 4 == 0 && vec_ok({a, b, y}, n)) {
    const dim3 gv(grid_for(n / 4));
    if (act > ACT_RELU6)
      hipLaunchKernelGGL(binary_f32v_kernel<true>, gv, dim3(256), 0, s, a, b, y, (unsigned)(n / 4), C, bcast_hw, op, act);
    else
      hipLaunchKernelGGL(binary_f32v_kernel<false>, gv, dim3(256), 0, s, a, b, y, (unsigned)(n / 4), C, bcast_hw, op,
                         act);
    return hipGetLastError();
  }
  if (act > ACT_RELU6)
    hipLaunchKernelGGL(binary_f32_kernel<true>, dim3(grid_for(n)), dim3(256), 0, s, a, b, y, n, C, bcast_hw, op, act);
  else
    hipLaunchKernelGGL(binary_f32_kernel<false>, dim3(grid_for(n)), dim3(256), 0, s, a, b, y, n, C, bcast_hw, op, act);
  return hipGetLastError();
}

hipError_t affine_act_f32(const float* x, const float* scale, const float* shift, float* y, size_t n, int C, int act,
                          float alpha, hipStream_t s) {
  if ((scale == nullptr) != (shift == nullptr)) return hipErrorInvalidValue;
  if (C % 4 == 0 && n % 4 == 0 && vec_ok({x, scale, shift, y}, n)) {
    const dim3 gv(grid_for(n / 4));
    if (act > ACT_RELU6)
      hipLaunchKernelGGL(affine_act_f32v_kernel<true>, gv, dim3(256), 0, s, x, scale, shift, y, (unsigned)(n / 4), C, act,
                         alpha);
    else
      hipLaunchKernelGGL(affine_act_f32v_kernel<false>, gv, dim3(256), 0, s, x, scale, shift, y, (unsigned)(n / 4), C,
                         act, alpha);
    return hipGetLastError();
  }
  if (act > ACT_RELU6)
    hipLaunchKernelGGL(affine_act_f32_kernel<true>, dim3(grid_for(n)), dim3(256), 0, s, x, scale, shift, y, n, C, act,
                       alpha);
  else
    hipLaunchKernelGGL(affine_act_f32_kernel<false>, dim3(grid_for(n)), dim3(256), 0, s, x, scale, shift, y, n, C, act,
                       alpha);
  return hipGetLastError();
}

}  // namespace adapt
