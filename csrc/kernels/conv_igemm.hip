// Implicit-GEMM convolution on MFMA (gfx950) with a fused epilogue.
//
//   out[m][n] = act( sum_k X[m][k] * W[n][k] + bias[n] (+ res[m][n]) )
//
//   m = (img, oh, ow) over the NHWC output, n = output channel,
//   k = (kh, kw, ci) with ci innermost (NHWC input, weights [Cout][KH][KW][Cin]).
//
// BN is folded into W/bias on the host (runtime/plan.py), so one launch
// covers the Keras conv -> bn [-> add] [-> relu] chain of a ResNet block
// (SURVEY §2.4).  Tiles: BM x BN x 64, 256 threads = 4 waves on a WM x WN
// grid, mfma_f32_16x16x32_bf16 (the faster bf16 shape on random data,
// MI355X_MICROARCH.md "DVFS give-back" (7)).  A/B tiles are staged through
// LDS with a register-prefetch double buffer (one barrier per K-tile) and an
// XOR chunk swizzle that makes the ds_read_b128 fragment reads conflict-free.
// The epilogue re-uses the stage LDS as an fp32 tile so bias/residual/ReLU
// are applied on coalesced 16-byte row segments.
//
// Split-K (ksplit > 1): each K-slice writes an fp32 partial slab
// ws[slice][M][N]; conv_splitk_reduce applies the epilogue.
#include <cstdlib>

#include "kernels.h"
#include "epilogue.h"

namespace adapt {



constexpr int BK = 64;            // bf16 elements per K-tile (8 x 16-byte chunks)
constexpr int NTHREADS = 256;

// byte offset of (row, 16B-chunk) inside a [rows][64] bf16 stage tile.
__device__ __forceinline__ int swz(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }

template <int BM, int BN, int WM, int WN, bool PURE_GEMM, bool OUT_F32>
__global__ __launch_bounds__(NTHREADS, 2) void conv_igemm_kernel(ConvParams p) {
  constexpr int TM = BM / WM, TN = BN / WN;       // wave tile
  constexpr int FM = TM / 16, FN = TN / 16;       // 16x16 MFMA fragments per wave
  constexpr int AROWS = BM / 32, BROWS = BN / 32; // rows loaded per thread per K-tile
  constexpr int STAGE_BYTES = (BM + BN) * BK * 2;
  constexpr int EPI_LD = BN + 4;                  // fp32 epilogue row stride (floats)
  constexpr int EPI_BYTES = BM * EPI_LD * 4;
  constexpr int LDS_BYTES = (2 * STAGE_BYTES > EPI_BYTES) ? 2 * STAGE_BYTES : EPI_BYTES;
  static_assert(WM * WN == 4, "4 waves");
  static_assert(TM % 16 == 0 && TN % 16 == 0, "wave tile");
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;

  const int tilesN = p.N / BN + ((p.N % BN) ? 1 : 0);
  const int tilesM = (p.M + BM - 1) / BM;
  const int nwg = tilesM * tilesN;
  const int tile = xcd_remap(blockIdx.x, nwg);
  const int tm = tile / tilesN, tn = tile % tilesN;
  const int m0 = tm * BM, n0 = tn * BN;

  // K range of this split-K slice
  const int ktiles_total = p.Kpad / BK;
  const int kt_per = (ktiles_total + p.ksplit - 1) / p.ksplit;
  const int kt0 = blockIdx.y * kt_per;
  const int kt1 = min(ktiles_total, kt0 + kt_per);

  // ---- per-thread A row bookkeeping (rows fixed for the whole K loop)
  const int lrow = tid >> 3;   // 0..31
  const int lch = tid & 7;     // 16B chunk within the 64-wide K tile
  int a_base[AROWS];           // element offset of image start (or of row for PURE_GEMM)
  int a_ih0[AROWS], a_iw0[AROWS];
  const int ohw = p.OH * p.OW;
#pragma unroll
  for (int i = 0; i < AROWS; ++i) {
    int m = m0 + lrow + 32 * i;
    if (PURE_GEMM) {
      a_base[i] = (m < p.M) ? m * p.Cin : -1;
      a_ih0[i] = a_iw0[i] = 0;
    } else {
      if (m < p.M) {
        int img = m / ohw;
        int r = m - img * ohw;
        int oh = r / p.OW;
        int ow = r - oh * p.OW;
        a_base[i] = img * p.H * p.W * p.Cin;
        a_ih0[i] = oh * p.stride - p.pad_t;
        a_iw0[i] = ow * p.stride - p.pad_l;
      } else {
        a_base[i] = 0;
        a_ih0[i] = -(1 << 28);
        a_iw0[i] = 0;
      }
    }
  }
  const bf16* wrow[BROWS];
#pragma unroll
  for (int i = 0; i < BROWS; ++i) wrow[i] = p.w + (size_t)(n0 + lrow + 32 * i) * p.Kpad + lch * 8;

  u32x4 ra[AROWS], rb[BROWS];
  const u32x4 zero4 = {0u, 0u, 0u, 0u};

  auto load_tile = [&](int kt) {
    const int k = kt * BK + lch * 8;
    if (PURE_GEMM) {
      const bool kok = k < p.K;
#pragma unroll
      for (int i = 0; i < AROWS; ++i) {
        ra[i] = (kok && a_base[i] >= 0) ? *(const u32x4*)(p.x + a_base[i] + k) : zero4;
      }
    } else {
      int tap = k / p.Cin;
      int ci = k - tap * p.Cin;
      int kh = tap / p.KW;
      int kw = tap - kh * p.KW;
      const bool kok = k < p.K;
#pragma unroll
      for (int i = 0; i < AROWS; ++i) {
        int ih = a_ih0[i] + kh, iw = a_iw0[i] + kw;
        bool ok = kok && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
        ra[i] = ok ? *(const u32x4*)(p.x + a_base[i] + (ih * p.W + iw) * p.Cin + ci) : zero4;
      }
    }
#pragma unroll
    for (int i = 0; i < BROWS; ++i) rb[i] = *(const u32x4*)(wrow[i] + (size_t)kt * BK);
  };
  auto store_tile = [&](int buf) {
    char* sa = smem + buf * STAGE_BYTES;
    char* sb = sa + BM * BK * 2;
#pragma unroll
    for (int i = 0; i < AROWS; ++i) *(u32x4*)(sa + swz(lrow + 32 * i, lch)) = ra[i];
#pragma unroll
    for (int i = 0; i < BROWS; ++i) *(u32x4*)(sb + swz(lrow + 32 * i, lch)) = rb[i];
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  EpiRes<BM, BN, NTHREADS> rpre;
  const bool use_pre = p.ksplit == 1 && p.res != nullptr;
  if (use_pre) rpre.prefetch(p, m0, n0, tid, p.M);
  if (kt0 < kt1) {
    load_tile(kt0);
    store_tile(0);
    __syncthreads();
    int buf = 0;
    for (int kt = kt0; kt < kt1; ++kt) {
      const bool more = kt + 1 < kt1;
      if (more) load_tile(kt + 1);
      const char* sa = smem + buf * STAGE_BYTES;
      const char* sb = sa + BM * BK * 2;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 af[FM], bfr[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i)
          af[i] = *(const bf16x8*)(sa + swz(wm * TM + i * 16 + fr, ks * 4 + fq));
#pragma unroll
        for (int j = 0; j < FN; ++j)
          bfr[j] = *(const bf16x8*)(sb + swz(wn * TN + j * 16 + fr, ks * 4 + fq));
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
      if (more) store_tile(buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
  }

  // ---- epilogue: fragments -> fp32 LDS tile -> coalesced 16B row segments
  float* epi = (float*)smem;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int col = wn * TN + j * 16 + fr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * TM + i * 16 + fq * 4 + r;
        epi[row * EPI_LD + col] = acc[i][j][r];
      }
    }
  __syncthreads();

  constexpr int CPR = BN / 8;                 // 8-wide chunks per row
  constexpr int NCH = BM * CPR;
  if (p.ksplit > 1) {
    float* slab = p.ws + (size_t)blockIdx.y * p.M * p.N;
    for (int c = tid; c < NCH; c += NTHREADS) {
      const int row = c / CPR, cc = c % CPR;
      const int m = m0 + row, n = n0 + cc * 8;
      if (m >= p.M || n >= p.N) continue;
      const float* e = epi + row * EPI_LD + cc * 8;
      f32x4 v0 = *(const f32x4*)e, v1 = *(const f32x4*)(e + 4);
      *(f32x4*)(slab + (size_t)m * p.N + n) = v0;
      *(f32x4*)(slab + (size_t)m * p.N + n + 4) = v1;
    }
    return;
  }
  fused_epilogue<BM, BN, NTHREADS, EPI_LD, OUT_F32>(p, epi, m0, n0, tid, p.M, &rpre, use_pre);
}

// split-K reduction + epilogue: out = act(sum_s ws[s] + bias (+res))
// KS > 0: the split count at compile time (every split's loads in flight at once) and 32-bit chunk math
// (host: chunks < 2^31); KS = 0: any split count
template <bool OUT_F32, int KS = 0>
__global__ __launch_bounds__(256) void conv_splitk_reduce(ConvParams p) {
  const size_t chunks = (size_t)p.M * (p.N / 8);
  for (size_t c = blockIdx.x * (size_t)blockDim.x + threadIdx.x; c < chunks; c += (size_t)gridDim.x * blockDim.x) {
    int m, n;
    if constexpr (KS > 0) {
      const unsigned n8 = (unsigned)(p.N / 8), cc = (unsigned)c;
      const unsigned mm = cc / n8;
      m = (int)mm;
      n = (int)(cc - mm * n8) * 8;
    } else {
      m = (int)(c / (p.N / 8));
      n = (int)(c % (p.N / 8)) * 8;
    }
    float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if constexpr (KS > 0) {
      f32x4 a[KS], b[KS];
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const float* src = p.ws + (size_t)s * p.M * p.N + (size_t)m * p.N + n;
        a[s] = *(const f32x4*)src;
        b[s] = *(const f32x4*)(src + 4);
      }
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        v[0] += a[s][0]; v[1] += a[s][1]; v[2] += a[s][2]; v[3] += a[s][3];
        v[4] += b[s][0]; v[5] += b[s][1]; v[6] += b[s][2]; v[7] += b[s][3];
      }
    } else {
      for (int s = 0; s < p.ksplit; ++s) {
        const float* src = p.ws + (size_t)s * p.M * p.N + (size_t)m * p.N + n;
        f32x4 a = *(const f32x4*)src, b = *(const f32x4*)(src + 4);
        v[0] += a[0]; v[1] += a[1]; v[2] += a[2]; v[3] += a[3];
        v[4] += b[0]; v[5] += b[1]; v[6] += b[2]; v[7] += b[3];
      }
    }
    if (p.bias) {
#pragma unroll
      for (int t = 0; t < 8; ++t) v[t] += p.bias[n + t];
    }
    if (p.res) {
      V8 r;
      r.u = *(const u32x4*)(p.res + (size_t)m * p.N + n);
#pragma unroll
      for (int t = 0; t < 8; ++t) v[t] += bf2f(r.e[t]);
    }
    const EpiDst d = epi_dst(p, n);
    if (d.relu) {
#pragma unroll
      for (int t = 0; t < 8; ++t) v[t] = act_relu(v[t], d.relu);
    }
    if (OUT_F32) {
      float* o = (float*)d.base + (size_t)m * d.ld + d.col;
#pragma unroll
      for (int t = 0; t < 8; ++t) o[t] = v[t];
    } else {
      V8 o;
#pragma unroll
      for (int t = 0; t < 8; ++t) o.e[t] = f2bf(v[t]);
      *(u32x4*)((bf16*)d.base + (size_t)m * d.ld + d.col) = o.u;
    }
  }
}

// ------------------------------------------------------------------ launch
// Tile configurations (index -> BM, BN, WM, WN).  Kept small and explicit so
// the host autotuner can time each for each conv problem.
#define ADAPT_CONV_CFGS(X)  \
  X(0, 128, 128, 2, 2)      \
  X(1, 128, 64, 2, 2)       \
  X(2, 64, 128, 2, 2)       \
  X(3, 64, 64, 2, 2)        \
  X(4, 256, 64, 4, 1)       \
  X(5, 32, 64, 1, 4)

int conv_num_cfgs() { return 6; }

void conv_cfg_tile(int cfg, int* bm, int* bn) {
  switch (cfg) {
#define X(id, BM_, BN_, WM_, WN_) case id: *bm = BM_; *bn = BN_; return;
    ADAPT_CONV_CFGS(X)
#undef X
  }
  if (!conv_glds_cfg_tile(cfg, bm, bn)) *bm = *bn = 0;
}

template <int BM, int BN, int WM, int WN>
static hipError_t launch_cfg(const ConvParams& p, hipStream_t s, bool pure, bool out_f32) {
  const int tilesM = (p.M + BM - 1) / BM;
  const int tilesN = (p.N + BN - 1) / BN;
  dim3 grid(tilesM * tilesN, p.ksplit), block(NTHREADS);
  if (pure) {
    if (out_f32) hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, true, true>), grid, block, 0, s, p);
    else hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, true, false>), grid, block, 0, s, p);
  } else {
    if (out_f32) hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, false, true>), grid, block, 0, s, p);
    else hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, false, false>), grid, block, 0, s, p);
  }
  return hipGetLastError();
}

hipError_t conv_forward(const ConvParams& p, int cfg, hipStream_t s, bool out_f32) {
  const bool pure = (p.KH == 1 && p.KW == 1 && p.stride == 1 && p.pad_t == 0 && p.pad_l == 0 &&
                     p.H == p.OH && p.W == p.OW);
  hipError_t e = hipErrorInvalidValue;
  if (p.ksplit == 0 || (p.ksplit < 0 && cfg < conv_num_cfgs())) return hipErrorInvalidValue;   // stream-K: v2 only
  switch (cfg) {
#define X(id, BM_, BN_, WM_, WN_) case id: e = launch_cfg<BM_, BN_, WM_, WN_>(p, s, pure, out_f32); break;
    ADAPT_CONV_CFGS(X)
#undef X
    default:
      if (cfg >= 40 && cfg < 53) return conv_halo_launch(p, cfg, s, out_f32);   // v3: 3x3 halo-patch kernel
      // v2 (LDS-DMA ring) configs walk K tap-major in 64-channel slices
      if (p.Cin % 64) return hipErrorInvalidValue;
      e = conv_glds_launch(p, cfg, s, pure, out_f32);
  }
  if (e != hipSuccess || p.ksplit <= 1) return e;
  const size_t chunks = (size_t)p.M * (p.N / 8);
  int blocks = (int)((chunks + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  const char* gk = getenv("ADAPT_SPLITK_GENERIC");            // A/B switch: the runtime-split kernel
  const bool small = chunks < 0x7fffffffu && !(gk && gk[0] == '1');
  if (small && p.ksplit == 2) {
    if (out_f32) hipLaunchKernelGGL((conv_splitk_reduce<true, 2>), dim3(blocks), dim3(256), 0, s, p);
    else hipLaunchKernelGGL((conv_splitk_reduce<false, 2>), dim3(blocks), dim3(256), 0, s, p);
  } else if (small && p.ksplit == 4) {
    if (out_f32) hipLaunchKernelGGL((conv_splitk_reduce<true, 4>), dim3(blocks), dim3(256), 0, s, p);
    else hipLaunchKernelGGL((conv_splitk_reduce<false, 4>), dim3(blocks), dim3(256), 0, s, p);
  } else if (out_f32) {
    hipLaunchKernelGGL((conv_splitk_reduce<true>), dim3(blocks), dim3(256), 0, s, p);
  } else {
    hipLaunchKernelGGL((conv_splitk_reduce<false>), dim3(blocks), dim3(256), 0, s, p);
  }
  return hipGetLastError();
}

}  // namespace adapt
