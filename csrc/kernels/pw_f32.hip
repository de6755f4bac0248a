// Persistent fp32 pointwise (1x1 / stride 1) conv with the filter slice resident in registers:
//
//   out = act(x . W + bias (+ res))      x [M][K], W [K][N], K in {64, 128, 256, 512, 1024}
//
// (also stride-s 1x1 convs, the input row of output pixel m being pixel (s oh, s ow), and merged
// sibling convs with a dual output split at a slice boundary)
//
// The fp32 tile GEMMs (conv_f32.hip / conv_f32g.hip) run ResNet's 1x1 convs at 43-51 % MFMA busy
// (profiles/r3/pmc/pmc_gemm1x1_f32.txt): at K = 128-512 a 64x64 tile has only 4-16 K steps, so every
// tile pays its ring fill, barriers and epilogue.  Here a block owns an N slice of NS = FPW x 128
// output channels for the whole launch: each of its 8 waves keeps FPW 16-channel fragments x all of
// K in VGPRs (FPW x K / 4 = 128 registers), and the block walks BM-pixel tiles of its slice, so the
// weights cross L2 -> VGPR once per block and the only per-tile traffic is the activation rows in
// (16-byte row-contiguous loads, prefetched one tile ahead into registers and staged in a swizzled
// LDS double buffer), the residual (16 bytes per lane, also a tile ahead, in registers) and the
// outputs (16 bytes per lane, straight from the accumulators).
// One barrier per tile.
//
// Transposed MFMA as in pw_pair_f32.hip: A = weight fragment, B = activation fragment
// (ds_read_b128 of a pixel row, lane group q supplying k = 16h + 4q + s to step s), D =
// [channel][pixel], so a lane's accumulator is 4 consecutive channels of one pixel.
#include <cstdlib>

#include "kernels.h"

namespace adapt {

namespace {

template <int NCH>
__device__ __forceinline__ int pswz32(int r, int c) {   // 16-byte chunk c of row r (NCH chunks per row)
  return r * (NCH * 16) + (((c & ~15) | ((c ^ r) & 15)) << 4);
}

}  // namespace

// KG > 1 (K = 1024): the 8 waves form KG groups that each hold the same channels over 1/KG of K;
// groups 1.. leave their partial sums in LDS and group 0 adds them in its epilogue.
template <int K, int FPW, int BM, int KG = 1>
__global__ __launch_bounds__(512, 1) void pw_f32_kernel(PwF32Params p) {
  constexpr int NT = 512, NWG = 8 / KG, NS = FPW * 16 * NWG;
  constexpr int KH = K / 16;                          // 16-wide K halves
  constexpr int KHG = KH / KG;                        // halves per K group
  constexpr int XCH = K / 4;                          // 16-byte chunks per pixel row
  constexpr int PF = BM / 16;
  constexpr int AB = BM * K * 4;
  constexpr int RED = (KG - 1) * BM * NS * 4;
  constexpr int XIT = (BM * XCH + NT - 1) / NT;
  static_assert(FPW * K / KG <= 512 && BM % 16 == 0 && 2 * AB + RED <= 160 * 1024 && KH % KG == 0, "pw shape");
  __shared__ __attribute__((aligned(16))) char abuf[2 * AB + (RED > 0 ? RED : 16)];
  float* const red = (float*)(abuf + 2 * AB);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kgi = wave / NWG, wg = wave - kgi * NWG;  // K group, wave within the group
  const int fr = lane & 15, fq = lane >> 4;
  const int nsl = p.N / NS;
  const int ntiles = (p.M + BM - 1) / BM;
  // slice-major block order: a slice's blocks are consecutive (one XCD shares its weights in L2)
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int per = gridDim.x / nsl;                    // blocks per slice (host: gridDim.x % nsl == 0)
  const int slice = logical / per, b0 = logical - slice * per;
  if (b0 >= ntiles) return;

  f32x4 wr[FPW][KHG];
  f32x4 bias[FPW];
#pragma unroll
  for (int j = 0; j < FPW; ++j) {
    const int gf = (slice * NWG + wg) * FPW + j;      // global 16-channel fragment
#pragma unroll
    for (int h = 0; h < KHG; ++h)
      wr[j][h] = *(const f32x4*)(p.w + ((size_t)(gf * KH + kgi * KHG + h) * 64 + lane) * 4);
    bias[j] = *(const f32x4*)(p.bias + gf * 16 + fq * 4);
  }

  // input row of output pixel m (stride-s 1x1: pixel (img, s oh, s ow) of the H x W input)
  const int ohw = p.OH * p.OW;
  auto xrow = [&](int m) __attribute__((always_inline)) {
    if (p.stride == 1) return m;
    const int img = m / ohw, r = m - img * ohw, oh = r / p.OW, ow = r - oh * p.OW;
    return (img * p.H + oh * p.stride) * p.W + ow * p.stride;
  };
  // dual output (merged sibling convs, n_split a multiple of the slice): one destination per block
  const bool second = p.n_split > 0 && slice * NS >= p.n_split;
  float* const dst = second ? p.out2 : p.out;
  const int ldo = p.n_split > 0 ? (second ? p.N - p.n_split : p.n_split) : p.N;
  const int cof = second ? p.n_split : 0;
  const int relu = second ? p.relu2 : p.relu;
  f32x4 rx[XIT];
  f32x4 rres[FPW][PF], nres[FPW][PF];                 // this tile's / the next tile's residual fragments
  const bool has_res = p.res != nullptr;
  auto load_next = [&](int t) __attribute__((always_inline)) {
#pragma unroll
    for (int it = 0; it < XIT; ++it) {
      const int i = tid + it * NT;
      const int px = i / XCH, c = i - px * XCH;
      const int m = min(t * BM + px, p.M - 1);
      if (XIT * NT == BM * XCH || i < BM * XCH) rx[it] = *(const f32x4*)(p.x + (size_t)xrow(m) * K + c * 4);
    }
    if (has_res && kgi == 0) {                        // the epilogue's residual, a tile ahead like x
#pragma unroll
      for (int i = 0; i < PF; ++i) {
        const int m = min(t * BM + i * 16 + fr, p.M - 1);
#pragma unroll
        for (int j = 0; j < FPW; ++j)
          nres[j][i] = *(const f32x4*)(p.res + (size_t)m * p.N + ((slice * NWG + wg) * FPW + j) * 16 + fq * 4);
      }
    }
  };
  auto stage_next = [&](int b) __attribute__((always_inline)) {
#pragma unroll
    for (int it = 0; it < XIT; ++it) {
      const int i = tid + it * NT;
      if (XIT * NT == BM * XCH || i < BM * XCH) *(f32x4*)(abuf + b * AB + pswz32<XCH>(i / XCH, i % XCH)) = rx[it];
    }
  };

  int t = b0;
  load_next(t);
  stage_next(0);
  __syncthreads();
  int buf = 0;
  for (; t < ntiles; t += per) {
    const int tn = t + per;
    const bool more = tn < ntiles;
    const int m0 = t * BM;
    if (has_res) {
#pragma unroll
      for (int j = 0; j < FPW; ++j)
#pragma unroll
        for (int i = 0; i < PF; ++i) rres[j][i] = nres[j][i];
    }
    if (more) load_next(tn);                          // in flight under this tile's MFMAs
    const char* a = abuf + buf * AB;
    f32x4 acc[FPW][PF];
#pragma unroll
    for (int j = 0; j < FPW; ++j)
#pragma unroll
      for (int i = 0; i < PF; ++i) acc[j][i] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int h = 0; h < KHG; ++h)
#pragma unroll
      for (int i = 0; i < PF; ++i) {
        const f32x4 xf = *(const f32x4*)(a + pswz32<XCH>(i * 16 + fr, (kgi * KHG + h) * 4 + fq));
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int j = 0; j < FPW; ++j)
            acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x4f32(wr[j][h][s], xf[s], acc[j][i], 0, 0, 0);
      }
    if constexpr (KG > 1) {                           // K groups 1.. -> LDS -> group 0
      if (kgi > 0) {
#pragma unroll
        for (int i = 0; i < PF; ++i)
#pragma unroll
          for (int j = 0; j < FPW; ++j)
            *(f32x4*)(red + (((kgi - 1) * BM + i * 16 + fr) * NS + (wg * FPW + j) * 16 + fq * 4)) = acc[j][i];
      }
      __syncthreads();
      if (kgi == 0) {
#pragma unroll
        for (int g = 1; g < KG; ++g)
#pragma unroll
          for (int i = 0; i < PF; ++i)
#pragma unroll
            for (int j = 0; j < FPW; ++j)
              acc[j][i] += *(const f32x4*)(red + (((g - 1) * BM + i * 16 + fr) * NS + (wg * FPW + j) * 16 + fq * 4));
      }
    }
    // epilogue (K group 0): acc[j][i][e] = out[pixel m0 + 16 i + fr][channel 16 gf + 4 fq + e]
#pragma unroll
    for (int i = 0; i < PF; ++i) {
      const int m = m0 + i * 16 + fr;
      if (m >= p.M || kgi > 0) continue;
#pragma unroll
      for (int j = 0; j < FPW; ++j) {
        const int ch = ((slice * NWG + wg) * FPW + j) * 16 + fq * 4;
        f32x4 v = acc[j][i] + bias[j];
        if (has_res) v += rres[j][i];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = act_relu(v[e], relu);
        *(f32x4*)(dst + (size_t)m * ldo + ch - cof) = v;
      }
    }
    if (more) stage_next(buf ^ 1);
    __syncthreads();                                  // next tile staged; this buffer's reads done
    buf ^= 1;
  }
}

// ---------------------------------------------------------------------------
// Streaming pointwise conv (bm codes 1 / 2 on the host, cfgs 122 / 123): the same math with no LDS
// and no block barrier.  Every wave is independent: it owns FPW 16-channel fragments x all of K in
// VGPRs (as above) and walks its own pixel tiles (slot, slot + nslots, ...), reading each tile's
// activation fragments straight from global memory into a ring of D float4 registers that is kept
// D K-steps ahead across tile boundaries, so the loads of tile t+1 stream in under the MFMAs of tile
// t.  pw_f32_kernel shares one LDS-staged tile between its 8 waves and pays a block barrier, the
// staging stores and an exposed epilogue per 16-pixel tile; the GEMM sweep put it at 61-80 % of
// the fp32 MFMA rate inside its loop plus ~6 us per launch (profiles/r4/gemm1x1_vs_k.log).  The
// waves that read one tile are the ncg channel groups of one slot; the XCD-aware block order keeps
// them on one XCD, so a tile crosses the fabric once per XCD.  FPW < 4 spreads each fragment over
// 4 / FPW accumulators by MFMA step, so every chain's consecutive MFMAs sit 4 apart.
//
// TAIL (bm codes 4 / 5, cfgs 125 / 126): the tile count rarely divides into the slots -- ResNet-50's
// 28x28 and 14x14 1x1 convs give every slot 6 tiles and an eighth of the slots a 7th, so 7/8 of the
// chip idles through the last tile round (`tools/pw_timeline.py`: waves with 7 tiles end 3.4 us after
// those with 6, one whole 4.6 us tile).  Here the slots walk `full` tiles each, then the `tail`
// left-over tiles are split by output fragment: the FPW waves of slots (ti x FPW + j) -- all holding
// the same filter slice as the tile's owner -- each run fragment j of tail tile ti over all of K and
// store it.  No partial sums, so no workspace, fence or counter (a K split needs all three and its
// chain of dependent round trips cost more than the tile it replaced: measured).
template <int KH, int FPW, int D, int J>
__device__ __forceinline__ void pw_tail_frag(const f32x4 (&wr)[FPW][KH], const float* xt, f32x4 (&acc)[4]) {
  f32x4 ring[D];
#pragma unroll
  for (int i = 0; i < D; ++i) ring[i] = *(const f32x4*)(xt + i * 16);
#pragma unroll
  for (int h = 0; h < KH; ++h) {
    const f32x4 xf = ring[h % D];
    if (h + D < KH) ring[h % D] = *(const f32x4*)(xt + (h + D) * 16);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int ss = 0; ss < 4; ++ss)       // four chains: a dependent 16x16x4 f32 MFMA waits 40 of 32 cycles
      acc[ss] = __builtin_amdgcn_mfma_f32_16x16x4f32(wr[J][h][ss], xf[ss], acc[ss], 0, 0, 0);
  }
}
template <int KH, int FPW, int D, int J = 0>
__device__ __forceinline__ void pw_tail_pick(int jj, const f32x4 (&wr)[FPW][KH], const float* xt, f32x4 (&acc)[4],
                                             const f32x4 (&bias)[FPW], f32x4& b) {
  if constexpr (J < FPW) {
    if (jj == J) {                                    // wave-uniform
      // the whole fragment's activations requested at once (the main ring is dead by now): one
      // fragment has only 4 MFMAs a K step, too few to hide a refill D steps ahead
      constexpr int TD = KH < 32 ? KH : 32;
      pw_tail_frag<KH, FPW, TD, J>(wr, xt, acc);
      b = bias[J];
    } else {
      pw_tail_pick<KH, FPW, D, J + 1>(jj, wr, xt, acc, bias, b);
    }
  }
}

// ACT >= 0: the activation mode at compile time (single-output launches; the runtime mode costs a max, a
// min and two selects per output element, ~25 % of the VALU work of a tile); -1: p.relu / p.relu2 at run time
template <int K, int FPW, int D, int OCC, bool TAIL = false, int ACT = -1>
__global__ __launch_bounds__(256, OCC) void pw_stream_f32_kernel(PwF32Params p, int ncg, int nslots, int full,
                                                                 int tail) {
  constexpr int KH = K / 16;
  // accumulator chains per fragment, taken by MFMA step ss: consecutive MFMAs into one chain sit >= 4
  // MFMAs apart (a dependent 16x16x4 f32 MFMA would wait 40 cycles past its 32 issue cycles -- the FPW = 1
  // twins used to chain all four steps of a K step back to back: 8.8 us a tile instead of 4.6)
  constexpr int NA = FPW >= 4 ? 1 : 4 / FPW;
  static_assert(KH % D == 0, "ring depth must divide the K steps");
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int gw = xcd_remap(blockIdx.x, gridDim.x) * 4 + wave;
  if (gw >= ncg * nslots) return;                     // wave-uniform
  const int cg = gw % ncg, slot = gw / ncg;
  const int fr = lane & 15, fq = lane >> 4;
  const int ntiles = (p.M + 15) / 16;
  if (slot >= ntiles) return;

  // per-wave stamps (p.dbg, tools/pw_timeline.py): [0] shader clock at start, [1] wall clock at start,
  // [2] HW_ID, [3] XCC_ID, [4] weights + first ring landed, [5..12] end of tiles 0..7, [13] shader clock
  // and [14] wall clock after the last stores, [15] tiles walked
  unsigned long long* const dbg = p.dbg ? p.dbg + 16 * gw : nullptr;
  const bool stamp = dbg && lane == 0;
  if (stamp) {
    dbg[0] = __builtin_amdgcn_s_memtime();
    dbg[1] = __builtin_amdgcn_s_memrealtime();
    dbg[2] = (unsigned)__builtin_amdgcn_s_getreg(0xF804);       // HW_ID
    dbg[3] = (unsigned)__builtin_amdgcn_s_getreg(0x7814);       // XCC_ID
  }
  f32x4 wr[FPW][KH];
  f32x4 bias[FPW];
#pragma unroll
  for (int j = 0; j < FPW; ++j) {
    const int gf = cg * FPW + j;
#pragma unroll
    for (int h = 0; h < KH; ++h) wr[j][h] = *(const f32x4*)(p.w + ((size_t)(gf * KH + h) * 64 + lane) * 4);
    bias[j] = *(const f32x4*)(p.bias + gf * 16 + fq * 4);
  }
  const bool second = p.n_split > 0 && cg * FPW * 16 >= p.n_split;
  float* const dst = second ? p.out2 : p.out;
  const int ldo = p.n_split > 0 ? (second ? p.N - p.n_split : p.n_split) : p.N;
  const int cof = second ? p.n_split : 0;
  const int relu = second ? p.relu2 : p.relu;
  const bool has_res = p.res != nullptr;
  const int ohw = p.OH * p.OW;
  auto xptr = [&](int t, int h) __attribute__((always_inline)) {
    int m = min(t * 16 + fr, p.M - 1);
    if (p.stride != 1) {
      const int img = m / ohw, r = m - img * ohw, oh = r / p.OW, ow = r - oh * p.OW;
      m = (img * p.H + oh * p.stride) * p.W + ow * p.stride;
    }
    return p.x + (size_t)m * K + h * 16 + fq * 4;
  };

  const int lim = TAIL ? full * nslots : ntiles;      // TAIL: the host guarantees full >= 1
  int t = slot;
  f32x4 ring[D];
  const float* xb = xptr(t, 0);
#pragma unroll
  for (int i = 0; i < D; ++i) ring[i] = *(const f32x4*)(xb + i * 16);
  if (dbg) {                                          // measurement only: wait for the prologue's loads
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) dbg[4] = __builtin_amdgcn_s_memtime();
  }
  int nt = 0;
  while (true) {
    const int tn = t + nslots;
    const bool more = tn < lim;
    const float* xn = xptr(more ? tn : t, 0);         // the last tile re-reads its own (valid) rows
    const int m = t * 16 + fr;
    f32x4 res[FPW];
    if (has_res) {
#pragma unroll
      for (int j = 0; j < FPW; ++j)
        res[j] = *(const f32x4*)(p.res + (size_t)min(m, p.M - 1) * p.N + (cg * FPW + j) * 16 + fq * 4);
    }
    f32x4 acc[NA][FPW];
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
      for (int j = 0; j < FPW; ++j) acc[a][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int h = 0; h < KH; ++h) {
      const f32x4 xf = ring[h % D];
      ring[h % D] = h + D < KH ? *(const f32x4*)(xb + (h + D) * 16) : *(const f32x4*)(xn + (h + D - KH) * 16);
      // keep the refill D steps ahead of its use (the scheduler otherwise sinks it next to the use)
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ss = 0; ss < 4; ++ss)
#pragma unroll
        for (int j = 0; j < FPW; ++j)
          acc[ss % NA][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(wr[j][h][ss], xf[ss], acc[ss % NA][j], 0, 0, 0);
    }
    if (m < p.M) {
#pragma unroll
      for (int j = 0; j < FPW; ++j) {
        f32x4 v = acc[0][j] + bias[j];
#pragma unroll
        for (int a = 1; a < NA; ++a) v += acc[a][j];
        if (has_res) v += res[j];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = act_relu(v[e], ACT >= 0 ? ACT : relu);
        *(f32x4*)(dst + (size_t)m * ldo + (cg * FPW + j) * 16 + fq * 4 - cof) = v;
      }
    }
    if (stamp) dbg[5 + min(nt, 7)] = __builtin_amdgcn_s_memtime();
    ++nt;
    if (!more) break;
    t = tn;
    xb = xn;
  }
  if (dbg) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) {
      dbg[13] = __builtin_amdgcn_s_memtime();
      dbg[14] = __builtin_amdgcn_s_memrealtime();
      dbg[15] = nt;
    }
  }
  if constexpr (TAIL && FPW > 1) {
    const int ti = slot / FPW, jj = slot - ti * FPW;
    if (ti >= tail) return;                           // wave-uniform
    const int tt = lim + ti;
    f32x4 acc[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) acc[a] = (f32x4){0.f, 0.f, 0.f, 0.f};
    f32x4 b;
    pw_tail_pick<KH, FPW, D>(jj, wr, xptr(tt, 0), acc, bias, b);
    const int m = tt * 16 + fr;
    const int col = (cg * FPW + jj) * 16 + fq * 4;
    f32x4 v = acc[0] + b;
    v += acc[1];
    v += acc[2];
    v += acc[3];
    if (has_res) v += *(const f32x4*)(p.res + (size_t)min(m, p.M - 1) * p.N + col);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = act_relu(v[e], ACT >= 0 ? ACT : relu);
    if (m < p.M) *(f32x4*)(dst + (size_t)m * ldo + col - cof) = v;
    if (dbg) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) {
        dbg[13] = __builtin_amdgcn_s_memtime();
        dbg[14] = __builtin_amdgcn_s_memrealtime();
        dbg[15] = nt + 100;                           // tiles walked + 100: this wave ran a tail fragment
      }
    }
  }
}

// (K, FPW, D, OCC): weights FPW x K / 4 VGPRs; OCC 2 where they leave room for a second wave per SIMD
#define ADAPT_PW_STREAM_CFGS(X) \
  X(64, 4, 4, 2)                \
  X(128, 4, 8, 2)               \
  X(256, 2, 8, 2)               \
  X(256, 4, 8, 1)               \
  X(512, 1, 8, 2)               \
  X(512, 2, 8, 1)               \
  X(1024, 1, 8, 1)

// deep-ring twins of the one-wave-per-SIMD instances (bm code 3, cfg 124): with a single wave per SIMD
// nothing covers a late activation load but the ring, and these have the VGPRs for 16 K-steps of lead
#define ADAPT_PW_STREAM_DEEP_CFGS(X) \
  X(256, 4, 16, 1)                  \
  X(512, 2, 16, 1)                  \
  X(1024, 1, 16, 1)

static int pw_stream_pick(int K, int N, int n_split, int wide) {
  // wide (bm code 2): the largest built FPW; else the one that keeps two waves per SIMD
  int best = 0;
#define X(K_, F_, D_, O_)                                                                    \
  if (K == K_ && N % (F_ * 16) == 0 && n_split % (F_ * 16) == 0 && (wide ? 1 : O_ == 2 || K_ == 1024)) \
    best = best > F_ ? best : F_;
  ADAPT_PW_STREAM_CFGS(X)
#undef X
  return best;
}

// (K, FPW, BM, KG) instances: FPW x K / KG <= 512 resident weight floats per lane (<= 128 VGPRs)
#define ADAPT_PW_F32_CFGS(X) \
  X(64, 2, 16, 1)            \
  X(64, 2, 32, 1)            \
  X(128, 4, 16, 1)           \
  X(128, 4, 32, 1)           \
  X(256, 2, 16, 1)           \
  X(256, 2, 32, 1)           \
  X(256, 1, 16, 1)           \
  X(512, 1, 16, 1)           \
  X(512, 1, 32, 1)           \
  X(1024, 1, 16, 2)

static int pw_f32_kg(int K) { return K == 1024 ? 2 : 1; }
static bool pw_f32_has(int K, int fpw, int bm) {
#define X(K_, F_, B_, G_) if (K == K_ && fpw == F_ && bm == B_) return true;
  ADAPT_PW_F32_CFGS(X)
#undef X
  return false;
}
// fragments per wave for (K, N, bm): the widest built instance whose slice (FPW x 16 x waves per
// K group channels) divides N, and (dual output) the first output's width; 0: none
static int pw_f32_pick(int K, int N, int n_split, int bm) {
  for (int fpw = 4; fpw >= 1; fpw >>= 1) {
    const int ns = fpw * 16 * (8 / pw_f32_kg(K));
    if (pw_f32_has(K, fpw, bm) && N % ns == 0 && n_split % ns == 0) return fpw;
  }
  return 0;
}
static int pw_stream_deep_pick(int K, int N, int n_split) {
  int best = 0;
#define X(K_, F_, D_, O_) \
  if (K == K_ && N % (F_ * 16) == 0 && n_split % (F_ * 16) == 0) best = best > F_ ? best : F_;
  ADAPT_PW_STREAM_DEEP_CFGS(X)
#undef X
  return best;
}
int pw_f32_fpw(int K, int N, int n_split, int bm) {
  if (bm == 3) return pw_stream_deep_pick(K, N, n_split);
  if (bm == 4 || bm == 5) return pw_stream_pick(K, N, n_split, bm == 5);
  return bm <= 2 ? pw_stream_pick(K, N, n_split, bm == 2) : pw_f32_pick(K, N, n_split, bm);
}

// a channel-split tail launch fits: whole rounds first, and tail x FPW waves to split the rest
static bool pw_tail_fits(int fpw, int ntiles, int nslots) {
  const int full = ntiles / nslots, tail = ntiles - full * nslots;
  return fpw > 1 && full >= 1 && tail >= 1 && tail * fpw <= nslots;
}

static unsigned long long* g_pw_dbg = nullptr;
void pw_set_debug(unsigned long long* buf) { g_pw_dbg = buf; }

template <int K, int F, int D, int O, bool TAIL>
static hipError_t pw_stream_launch(const PwF32Params& p_, int ncg, int ntiles, hipStream_t s) {
  PwF32Params p = p_;
  p.dbg = g_pw_dbg;
  int nslots = (1024 * O) / ncg;                      // ~O waves per SIMD over the chip
  if (nslots < 1) nslots = 1;
  if (nslots > ntiles) nslots = ntiles;
  const int blocks = (ncg * nslots + 3) / 4;
  const char* ag = getenv("ADAPT_PW_ACT_GENERIC");             // A/B switch: the run-time activation mode
  if (p.n_split == 0 && p.relu == 1 && !(ag && ag[0] == '1')) {
    if constexpr (!TAIL) {
      hipLaunchKernelGGL((pw_stream_f32_kernel<K, F, D, O, false, 1>), dim3(blocks), dim3(256), 0, s, p, ncg,
                         nslots, 0, 0);
      return hipGetLastError();
    } else if constexpr (F > 1) {
      const int full = ntiles / nslots, tail = ntiles - full * nslots;
      if (pw_tail_fits(F, ntiles, nslots)) {
        hipLaunchKernelGGL((pw_stream_f32_kernel<K, F, D, O, true, 1>), dim3(blocks), dim3(256), 0, s, p, ncg,
                           nslots, full, tail);
        return hipGetLastError();
      }
      return hipErrorInvalidValue;
    }
  }
  if constexpr (!TAIL) {
    hipLaunchKernelGGL((pw_stream_f32_kernel<K, F, D, O>), dim3(blocks), dim3(256), 0, s, p, ncg, nslots, 0, 0);
    return hipGetLastError();
  } else {
    const int full = ntiles / nslots, tail = ntiles - full * nslots;
    if constexpr (F > 1) {
      if (pw_tail_fits(F, ntiles, nslots)) {
        hipLaunchKernelGGL((pw_stream_f32_kernel<K, F, D, O, true>), dim3(blocks), dim3(256), 0, s, p, ncg, nslots,
                           full, tail);
        return hipGetLastError();
      }
    }
  }
  return hipErrorInvalidValue;
}

void pw_f32_tail_plan(int M, int K, int N, int n_split, int bm, int* tail_tiles, int* parts) {
  *tail_tiles = *parts = 0;
  const int fpw = pw_f32_fpw(K, N, n_split, bm);
  if (!fpw || (bm != 4 && bm != 5)) return;
  const int ncg = N / (16 * fpw), ntiles = (M + 15) / 16;
  int o = 0;
#define X(K_, F_, D_, O_) if (K == K_ && fpw == F_) o = O_;
  ADAPT_PW_STREAM_CFGS(X)
#undef X
  int nslots = (1024 * o) / ncg;
  if (nslots < 1) nslots = 1;
  if (nslots > ntiles) nslots = ntiles;
  if (!pw_tail_fits(fpw, ntiles, nslots)) return;
  *tail_tiles = ntiles % nslots;
  *parts = fpw;
}

bool pw_f32_supported(int K, int N, int bm) { return pw_f32_fpw(K, N, 0, bm) > 0; }

static hipError_t pw_stream_f32_forward(const PwF32Params& p, int mode, hipStream_t s) {
  const int fpw = pw_f32_fpw(p.K, p.N, p.n_split, mode);
  if (!fpw) return hipErrorInvalidValue;
  const int ncg = p.N / (16 * fpw);
  const int ntiles = (p.M + 15) / 16;
  if (mode == 3) {
#define X(K_, F_, D_, O_) \
  if (p.K == K_ && fpw == F_) return pw_stream_launch<K_, F_, D_, O_, false>(p, ncg, ntiles, s);
    ADAPT_PW_STREAM_DEEP_CFGS(X)
#undef X
    return hipErrorInvalidValue;
  }
#define X(K_, F_, D_, O_)                                                                          \
  if (p.K == K_ && fpw == F_)                                                                      \
    return mode >= 4 ? pw_stream_launch<K_, F_, D_, O_, true>(p, ncg, ntiles, s)                   \
                     : pw_stream_launch<K_, F_, D_, O_, false>(p, ncg, ntiles, s);
  ADAPT_PW_STREAM_CFGS(X)
#undef X
  return hipErrorInvalidValue;
}

hipError_t pw_f32_forward(const PwF32Params& p, int bm, hipStream_t s) {
  if (bm >= 1 && bm <= 5) {
    if (p.M < 1 || p.stride < 1 || (p.n_split && (!p.out2 || p.res)) || p.M != p.B * p.OH * p.OW ||
        (p.stride == 1 && (p.H != p.OH || p.W != p.OW)))
      return hipErrorInvalidValue;
    return pw_stream_f32_forward(p, bm, s);
  }
  const int fpw = pw_f32_pick(p.K, p.N, p.n_split, bm);
  if (!fpw || p.M < 1 || p.stride < 1 || (p.n_split && (!p.out2 || p.res)) ||
      p.M != p.B * p.OH * p.OW || (p.stride == 1 && (p.H != p.OH || p.W != p.OW)))
    return hipErrorInvalidValue;
  const int nsl = p.N / (fpw * 16 * (8 / pw_f32_kg(p.K)));
  const int ntiles = (p.M + bm - 1) / bm;
  int per = 256 / nsl;                                // ~one block per CU over all slices
  if (per < 1) per = 1;
  if (per > ntiles) per = ntiles;
#define X(K_, F_, B_, G_)                                                                              \
  if (p.K == K_ && fpw == F_ && bm == B_) {                                                            \
    hipLaunchKernelGGL((pw_f32_kernel<K_, F_, B_, G_>), dim3(per * nsl), dim3(512), 0, s, p);          \
    return hipGetLastError();                                                                          \
  }
  ADAPT_PW_F32_CFGS(X)
#undef X
  return hipErrorInvalidValue;
}

}  // namespace adapt
