// ResNet stem: fp32 image -> [7x7/s2 conv + folded BN + ReLU] -> [3x3/s2 max-pool]
// in ONE launch (SURVEY §2.4 rows conv1_pad/conv1_conv/conv1_bn/conv1_relu/
// pool1_pad/pool1_pool; the reference runs these as six Keras layers inside
// `model.predict`, src/node.py:177).
//
// Why a dedicated kernel: the generic implicit-GEMM path needs Cin % 8, so the
// 3-channel image is first packed to 8 channels (K = 7*7*8 = 392 -> 448, 3x the
// real K = 147) and the 51 MB conv1 output makes a round trip through HBM for
// the max-pool.  Here:
//
// * the block stages the fp32 input rows it needs into LDS as bf16 with the
//   channel dim padded to 4, so one filter row (kw = 0..7 x 4 ch) is 64
//   contiguous bytes and K = 7 rows x 32 = 224 (one 16x16x32 MFMA k-step per
//   filter row, the kw = 7 / c = 3 slots carry zero weights);
// * A fragments are single 16-byte ds_read_b128 (stride 2 -> 2 pixel columns
//   = 16 B between neighbouring output pixels: conflict-free);
// * the 64-output-channel weight panel (7 x 4 fragments) lives in VGPRs for the
//   whole block;
// * conv outputs (bias + ReLU, rounded to bf16 exactly like the unfused path)
//   stay in LDS and the block emits the max-pooled rows directly.  One pool
//   row needs conv rows 2p-1..2p+1: the row shared with the neighbouring
//   block is recomputed (cheap: the stem is memory-bound).
#include "kernels.h"

namespace adapt {
namespace {

constexpr int ST_NT = 256;              // 4 waves
constexpr int ST_OWMAX = 112;           // widest conv row a block stages (224-px input)
constexpr int ST_PWC = 2 * ST_OWMAX + 8;  // patch columns (kw up to 7 past 2*ow)
constexpr int ST_CROWS_POOL = 3, ST_CROWS_CONV = 2;
constexpr int ST_PROWS = 2 * (ST_CROWS_POOL - 1) + 7;   // 11 input rows
constexpr int ST_K = 224;               // 7 filter rows x (8 kw x 4 ch)
static_assert(ST_PWC <= ST_NT, "one thread per patch column");

struct __attribute__((aligned(8))) bf16x4s {
  bf16 v[4];
};

// staged conv output: [pixel][64 ch] bf16 = 8 chunks of 16 B per pixel, chunk
// index XOR-swizzled by (pixel >> 1) so the C^T fragment stores (16 pixels x
// one chunk) spread over all 64 banks
__device__ __forceinline__ int stage_off(int row, int pix, int chunk) {
  return ((row * ST_OWMAX + pix) * 8 + (chunk ^ ((pix >> 1) & 7))) * 8;   // in bf16 elements
}

// Input pixels by buffer load: an out-of-range offset (outside the image, or channel >= C) reads 0 with
// no branch.  A plain `ok ? px[c] : 0` load compiles to a branch around every load with a vmcnt(0)
// behind it, so each of a thread's ~20-76 loads was its own round trip.
__device__ __forceinline__ float stem_ld(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t stem_rsrc(const float* xi, int H, int W, int C) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)xi, (short)0, H * W * C * 4, 0x00020000);
}

}  // namespace

template <bool POOL>
__global__ __launch_bounds__(ST_NT, 2) void stem_kernel(const float* __restrict__ x, const bf16* __restrict__ w,
                                                        const float* __restrict__ bias, bf16* __restrict__ out,
                                                        int H, int W, int C, int OH, int OW, int pad_t, int pad_l,
                                                        int PH, int PW, int pool_pad) {
  __shared__ __attribute__((aligned(16))) bf16 patch[ST_PROWS * ST_PWC * 4];          // 20.4 KB
  __shared__ __attribute__((aligned(16))) bf16 stage[ST_CROWS_POOL * ST_OWMAX * 64];  // 43 KB

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // 1-D grid, XCD-aware: the row blocks of one image (which share 7 of their 11
  // input rows with their neighbours) run on the same XCD and hit its L2
  constexpr int CROWS = POOL ? ST_CROWS_POOL : ST_CROWS_CONV;
  const int rows_per_img = POOL ? PH : (OH + CROWS - 1) / CROWS;
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int img = logical / rows_per_img;
  const int t = logical - img * rows_per_img;
  constexpr int PROWS = 2 * (CROWS - 1) + 7;
  const int r0 = POOL ? 2 * t - pool_pad : CROWS * t;    // first conv row of this block
  const int ih0 = 2 * r0 - pad_t;                          // input row of patch row 0
  const int tpr = (OW + 15) >> 4;                          // 16-pixel m-tiles per conv row
  const int pwc = 2 * tpr * 16 + 8;                        // patch columns in use

  // ---- weight panel -> VGPRs (7 k-steps x 4 n-tiles of 16 columns)
  const int fr = lane & 15, fq = lane >> 4;
  bf16x8 bw[7][4];
#pragma unroll
  for (int s = 0; s < 7; ++s)
#pragma unroll
    for (int n = 0; n < 4; ++n) bw[s][n] = *(const bf16x8*)(w + (size_t)(n * 16 + fr) * ST_K + s * 32 + fq * 8);

  // ---- stage input rows: fp32 NHWC (C <= 4) -> bf16 [row][col][4], zero outside the image.
  // Thread j owns patch column j for every row (no index division); all of its
  // loads are issued before the first conversion so the round trips overlap.
  const float* xi = x + (size_t)img * H * W * C;
  {
    const int j = tid, iw = j - pad_l;
    const bool colok = j < pwc && (unsigned)iw < (unsigned)W;
    const __amdgpu_buffer_rsrc_t xr = stem_rsrc(xi, H, W, C);
    float pv[PROWS][4];
#pragma unroll
    for (int i = 0; i < PROWS; ++i) {
      const int ih = ih0 + i;
      const bool ok = colok && (unsigned)ih < (unsigned)H;
      const int off = ((ih * W + iw) * C) * 4;
#pragma unroll
      for (int c = 0; c < 4; ++c) pv[i][c] = stem_ld(xr, ok && c < C ? off + 4 * c : 0x7fffffff);
    }
    if (j < pwc) {
#pragma unroll
      for (int i = 0; i < PROWS; ++i) {
        bf16x4s v;
#pragma unroll
        for (int c = 0; c < 4; ++c) v.v[c] = f2bf(pv[i][c]);
        *(bf16x4s*)(patch + (i * ST_PWC + j) * 4) = v;
      }
    }
  }
  __syncthreads();

  // ---- conv: each wave takes m-tiles round-robin; one tile = 16 pixels x 64 channels.
  // The MFMA computes the transposed tile (weights as the A operand) so each
  // lane ends up with 4 consecutive channels of one pixel: one 8-byte LDS
  // store per 16-channel group instead of four 2-byte ones.
  float b4[4][4];
#pragma unroll
  for (int n = 0; n < 4; ++n)
#pragma unroll
    for (int r = 0; r < 4; ++r) b4[n][r] = bias[n * 16 + 4 * fq + r];
  const int ntiles = CROWS * tpr;
  for (int mt = wave; mt < ntiles; mt += ST_NT / 64) {
    const int rr = mt / tpr, c0 = (mt - rr * tpr) * 16;
    f32x4 acc[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[n] = (f32x4){0.f, 0.f, 0.f, 0.f};
    const int ow = c0 + fr;
#pragma unroll
    for (int s = 0; s < 7; ++s) {
      // k = s*32 + 8*fq + e  ->  filter row s, kw = 2*fq + e/4, c = e%4
      const bf16x8 a = *(const bf16x8*)(patch + ((2 * rr + s) * ST_PWC + 2 * ow + 2 * fq) * 4);
#pragma unroll
      for (int n = 0; n < 4; ++n) acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[s][n], a, acc[n], 0, 0, 0);
    }
    // C^T fragment: channel = 16*n + 4*fq + r, pixel = c0 + fr
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      bf16x4s v;
#pragma unroll
      for (int r = 0; r < 4; ++r) v.v[r] = f2bf(fmaxf(acc[n][r] + b4[n][r], 0.f));
      *(bf16x4s*)(stage + stage_off(rr, ow, 2 * n + (fq >> 1)) + 4 * (fq & 1)) = v;
    }
  }
  __syncthreads();

  if (!POOL) {
    // conv rows -> global, 16 B per lane
    for (int idx = tid; idx < CROWS * OW * 8; idx += ST_NT) {
      const int ch8 = idx & 7, pix = idx >> 3;
      const int rr = pix / OW, ow = pix - rr * OW;
      const int oh = r0 + rr;
      if (oh >= OH) continue;
      *(u32x4*)(out + (((size_t)img * OH + oh) * OW + ow) * 64 + ch8 * 8) =
          *(const u32x4*)(stage + stage_off(rr, ow, ch8));
    }
    return;
  }
  // ---- 3x3/s2 max-pool of the staged conv rows: pool row t.  Post-ReLU values
  // are >= 0, so the zero padding of pool1_pad is the 0 the max starts from.
  for (int idx = tid; idx < PW * 8; idx += ST_NT) {
    const int ch8 = idx & 7, pw = idx >> 3;
    float m[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) m[e] = 0.f;
#pragma unroll
    for (int dr = 0; dr < 3; ++dr) {
      const int oh = r0 + dr;
      if ((unsigned)oh >= (unsigned)OH) continue;
#pragma unroll
      for (int dc = 0; dc < 3; ++dc) {
        const int ow = 2 * pw - pool_pad + dc;
        if ((unsigned)ow >= (unsigned)OW) continue;
        V8 v;
        v.u = *(const u32x4*)(stage + stage_off(dr, ow, ch8));
#pragma unroll
        for (int e = 0; e < 8; ++e) m[e] = fmaxf(m[e], bf2f(v.e[e]));
      }
    }
    V8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o.e[e] = f2bf(m[e]);
    *(u32x4*)(out + (((size_t)img * PH + t) * PW + pw) * 64 + ch8 * 8) = o.u;
  }
}

// ---- v2 pooled stem: one block per (image, group of S2_SP pool rows) ------------
//
// v1 (stem_kernel<true>) recomputes 3 conv rows per pool row (1.5x the conv
// work) and re-stages 11 input rows per 2 new conv rows: 1792 blocks of 4
// waves, 52.9 us at bs=32 (profiles/stem_bench.txt; PMC: VALU-heavy staging,
// waits).  v2 walks S2_SP pool rows per block with a 3-row ring of conv rows
// in LDS: each step computes conv rows 2t, 2t+1 once (only the block's first
// pool row also computes row 2t-1) and emits pool row t from rows 2t-1..2t+1.
// The (4*S2_SP+7)-row input patch is staged once.  224x224 at bs=32: 8 row
// groups x 32 images = 256 blocks, one per CU; 7 waves = the 14 16-pixel conv
// tiles of a two-row step, two per wave.
namespace {
constexpr int S2_SP = 7;                                   // pool rows per block
constexpr int ST_V1_MAX_BLOCKS = 448;                      // auto: v1 up to this many pool-row blocks (B<=8 at 224)
constexpr int S2_WAVES = 7;
constexpr int S2_NT = S2_WAVES * 64;
constexpr int S2_PROWS = 4 * S2_SP + 7;                    // input rows of a block's patch (35)
constexpr int S2_ROWS0 = 11;                              // patch rows the first step needs
constexpr int S2_ITEMS0 = (S2_ROWS0 * ST_PWC + S2_NT - 1) / S2_NT;
constexpr int S2_ITEMS1 = (4 * ST_PWC + S2_NT - 1) / S2_NT;  // 4 new input rows per later step
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
union P8 {                                                 // 8 bf16 as 16 B or as 4 packed u16 pairs
  u32x4 u;
  u16x2 h[4];
};
}  // namespace

// fp32 NHWC patch rows [row0, row0 + nrows) -> registers (loads only; `put_rows` converts + stores)
template <int ITEMS, int NT = S2_NT>
__device__ __forceinline__ void get_rows(float (&pv)[ITEMS][4], const float* __restrict__ xi, int tid, int row0,
                                         int nrows, int row_end, int ih0, int H, int W, int C, int pwc, int pad_l) {
  const __amdgpu_buffer_rsrc_t xr = stem_rsrc(xi, H, W, C);
#pragma unroll
  for (int k = 0; k < ITEMS; ++k) {
    const int idx = tid + k * NT;
    const int i = row0 + idx / ST_PWC, j = idx % ST_PWC;
    const int ih = ih0 + i, iw = j - pad_l;
    const bool ok = idx < nrows * ST_PWC && i < row_end && j < pwc && (unsigned)ih < (unsigned)H &&
                    (unsigned)iw < (unsigned)W;
    const int off = ((ih * W + iw) * C) * 4;
#pragma unroll
    for (int c = 0; c < 4; ++c) pv[k][c] = stem_ld(xr, ok && c < C ? off + 4 * c : 0x7fffffff);
  }
}
template <int ITEMS>
__device__ __forceinline__ void put_rows(const float (&pv)[ITEMS][4], bf16* patch, int tid, int row0, int nrows) {
#pragma unroll
  for (int k = 0; k < ITEMS; ++k) {
    const int idx = tid + k * S2_NT;
    if (idx < nrows * ST_PWC && row0 * ST_PWC + idx < S2_PROWS * ST_PWC) {
      bf16x4s v;
#pragma unroll
      for (int c = 0; c < 4; ++c) v.v[c] = f2bf(pv[k][c]);
      *(bf16x4s*)(patch + (row0 * ST_PWC + idx) * 4) = v;
    }
  }
}

// patch items [k0, k0 + N) of a block's whole patch -> LDS, rows [rlo, rhi) only (k compile-time: no
// register indexing; the compiler waits only for the loads of the items it stores)
template <int K0, int N, int ITEMS, int NT = S2_NT>
__device__ __forceinline__ void put_items(const float (&pv)[ITEMS][4], bf16* patch, int tid, int rlo, int rhi) {
#pragma unroll
  for (int k = K0; k < K0 + N; ++k) {
    const int idx = tid + k * NT;
    if (idx >= rlo * ST_PWC && idx < rhi * ST_PWC) {
      bf16x4s v;
#pragma unroll
      for (int c = 0; c < 4; ++c) v.v[c] = f2bf(pv[k][c]);
      *(bf16x4s*)(patch + idx * 4) = v;
    }
  }
}

// ALL (v3): the block's whole (4*S2_SP+7)-row patch is requested in the prologue -- 19 items of 4 floats
// per thread in flight at once -- and the first step's 11 rows go to LDS as soon as they land; the
// other rows are stored during the first step's MFMAs.  v2 requested 4 rows a step, one step ahead,
// and paid a global-load round trip per step (29 us at bs=32, profiles/r4/r4s: ~4 us a step for
// ~0.75 us of MFMAs).
constexpr int S2_ITEMS_ALL = (S2_PROWS * ST_PWC + S2_NT - 1) / S2_NT;   // 19
constexpr int S2_ITEMS_A = (S2_ROWS0 * ST_PWC + S2_NT - 1) / S2_NT;     // items holding rows 0..10

template <bool ALL>
__global__ __launch_bounds__(S2_NT, 1) void stem_pool_v2_kernel(const float* __restrict__ x,
                                                                const bf16* __restrict__ w,
                                                                const float* __restrict__ bias,
                                                                bf16* __restrict__ out, int H, int W, int C, int OH,
                                                                int OW, int pad_t, int pad_l, int PH, int PW,
                                                                int pool_pad, int groups) {
  __shared__ __attribute__((aligned(16))) bf16 patch[S2_PROWS * ST_PWC * 4];        // 63.4 KiB
  __shared__ __attribute__((aligned(16))) bf16 ring[ST_CROWS_POOL * ST_OWMAX * 64];  // 42 KiB

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int img = logical / groups;
  const int t0 = (logical - img * groups) * S2_SP;
  const int t1 = min(PH, t0 + S2_SP);                      // pool rows [t0, t1)
  const int r_first = 2 * t0 - pool_pad;                   // first conv row (may be -1)
  const int ih0 = 2 * r_first - pad_t;                     // input row of patch row 0
  const int row_end = 4 * (t1 - t0) + 7;                   // patch rows in use (2R+5 for R = 2(t1-t0)+1 conv rows)
  const int tpr = (OW + 15) >> 4;
  const int pwc = 2 * tpr * 16 + 8;
  const float* xi = x + (size_t)img * H * W * C;

  // first step's 11 input rows (v3: the whole patch): loads in flight while the weight panel loads
  float pall[ALL ? S2_ITEMS_ALL : 1][4];
  if constexpr (ALL) {
    get_rows<S2_ITEMS_ALL>(pall, xi, tid, 0, row_end, row_end, ih0, H, W, C, pwc, pad_l);
  } else {
    float pv0[S2_ITEMS0][4];
    get_rows<S2_ITEMS0>(pv0, xi, tid, 0, S2_ROWS0, row_end, ih0, H, W, C, pwc, pad_l);
    put_rows<S2_ITEMS0>(pv0, patch, tid, 0, S2_ROWS0);
  }
  const int fr = lane & 15, fq = lane >> 4;
  bf16x8 bw[7][4];
#pragma unroll
  for (int s = 0; s < 7; ++s)
#pragma unroll
    for (int n = 0; n < 4; ++n) bw[s][n] = *(const bf16x8*)(w + (size_t)(n * 16 + fr) * ST_K + s * 32 + fq * 8);
  float b4[4][4];
#pragma unroll
  for (int n = 0; n < 4; ++n)
#pragma unroll
    for (int r = 0; r < 4; ++r) b4[n][r] = bias[n * 16 + 4 * fq + r];
  if constexpr (ALL) put_items<0, S2_ITEMS_A>(pall, patch, tid, 0, S2_ROWS0);
  __syncthreads();

  auto step = [&](const int t, auto first) __attribute__((always_inline)) {
    // v2: the NEXT step's 4 input rows, issued now, landed in LDS after this step's MFMAs
    const int nrow0 = 4 * (t - t0) + S2_ROWS0;
    float pv[S2_ITEMS1][4];
    const bool more = !ALL && t + 1 < t1;
    if (more) get_rows<S2_ITEMS1>(pv, xi, tid, nrow0, 4, row_end, ih0, H, W, C, pwc, pad_l);
    // conv rows of this step: 2t-pp+1 .. 2t-pp+2, plus 2t-pp on the block's first step
    const int ra = 2 * t - pool_pad + (t == t0 ? 0 : 1);
    const int nr = 2 * t - pool_pad + 3 - ra;
    const int ntiles = nr * tpr;
    for (int mt = wave; mt < ntiles; mt += S2_WAVES) {
      const int q = mt / tpr;
      const int r = ra + q;
      if (r < 0 || r >= OH) continue;                      // wave-uniform
      const int c0 = (mt - q * tpr) * 16;
      const int prow = 2 * (r - r_first);
      f32x4 acc[4];
#pragma unroll
      for (int n = 0; n < 4; ++n) acc[n] = (f32x4){0.f, 0.f, 0.f, 0.f};
      const int ow = c0 + fr;
#pragma unroll
      for (int s = 0; s < 7; ++s) {
        const bf16x8 a = *(const bf16x8*)(patch + ((prow + s) * ST_PWC + 2 * ow + 2 * fq) * 4);
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[s][n], a, acc[n], 0, 0, 0);
      }
      const int slot = r % ST_CROWS_POOL;
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        bf16x4s v;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float y = acc[n][e] + b4[n][e];
          v.v[e] = f2bf(y > 0.f ? y : 0.f);               // +0 for y <= 0: staged values are non-negative bit patterns
        }
        *(bf16x4s*)(ring + stage_off(slot, ow, 2 * n + (fq >> 1)) + 4 * (fq & 1)) = v;
      }
    }
    if (more) put_rows<S2_ITEMS1>(pv, patch, tid, nrow0, 4);
    if constexpr (ALL && decltype(first)::value)     // v3: the rest of the patch, landed under the MFMAs
      put_items<S2_ITEMS_A - 1, S2_ITEMS_ALL - S2_ITEMS_A + 1>(pall, patch, tid, S2_ROWS0, row_end);
    __syncthreads();
    // pool row t from conv rows 2t-pp .. 2t-pp+2.  Non-negative bf16 values order
    // like their u16 bit patterns: packed integer max, 2 values per instruction;
    // the zero padding is the 0 the max starts from.
    for (int idx = tid; idx < PW * 8; idx += S2_NT) {
      const int ch8 = idx & 7, pw = idx >> 3;
      P8 m;
#pragma unroll
      for (int e = 0; e < 4; ++e) m.h[e] = (u16x2){0, 0};
#pragma unroll
      for (int dr = 0; dr < 3; ++dr) {
        const int oh = 2 * t - pool_pad + dr;
        if ((unsigned)oh >= (unsigned)OH) continue;
        const int slot = oh % ST_CROWS_POOL;
#pragma unroll
        for (int dc = 0; dc < 3; ++dc) {
          const int ow = 2 * pw - pool_pad + dc;
          if ((unsigned)ow >= (unsigned)OW) continue;
          P8 v;
          v.u = *(const u32x4*)(ring + stage_off(slot, ow, ch8));
#pragma unroll
          for (int e = 0; e < 4; ++e) m.h[e] = __builtin_elementwise_max(m.h[e], v.h[e]);
        }
      }
      *(u32x4*)(out + (((size_t)img * PH + t) * PW + pw) * 64 + ch8 * 8) = m.u;
    }
    __syncthreads();                                       // ring slots of rows 2t-pp, 2t-pp+1 are free
  };
  // the first step peeled (straight-line), so v3's remaining patch stores wait only for their own loads
  step(t0, std::integral_constant<bool, true>{});
  for (int t = t0 + 1; t < t1; ++t) step(t, std::integral_constant<bool, false>{});
}

// ---- v4 pooled stem: software-pipelined conv / pool, 8 waves -------------------------------------------
//
// v3 (26 us at bs=32, profiles/r4/stem_bf16) alternates "conv 2 rows | barrier | pool 1 row | barrier" with
// 7 waves: MFMA busy 0.21, 37 % of LDS cycles lost to bank conflicts, 2 of the 4 SIMDs carrying 2 waves
// and 2 carrying 1 or 2.  v4:
// * one barrier per step: step k computes conv rows 2k+1, 2k+2 of the block into a 6-row ring while
//   the same waves pool row k-1 from rows 2k-2..2k, finished the step before (the two row sets never
//   share a ring slot);
// * 8 waves = 2 per SIMD: one wave's pool reads / stores hide behind its SIMD partner's MFMAs;
// * ring rows stored as pixel pairs (256 B = all 64 banks) with the 16-byte unit index XOR-swizzled by
//   pair & 15: the MFMA epilogue's 16 lanes (8 aligned pairs x 2 pixels, one channel chunk) and the
//   pool's 16 lanes (16 consecutive pool columns = 16 consecutive pairs, one chunk; the lane order is
//   pool column fastest) both hit 16 distinct bank groups.
namespace {
constexpr int S4_SP = 7;                                   // pool rows per block
constexpr int S4_WAVES = 8;
constexpr int S4_NT = S4_WAVES * 64;
constexpr int S4_RING = 6;
constexpr int S4_PAIRS = ST_OWMAX / 2;
constexpr int S4_PROWS = 4 * S4_SP + 7;
constexpr int S4_ITEMS = (S4_PROWS * ST_PWC + S4_NT - 1) / S4_NT;     // 16
constexpr int S4_ITEMS_A = (S2_ROWS0 * ST_PWC + S4_NT - 1) / S4_NT;   // items holding rows 0..10 (5)
static_assert(S4_PROWS * ST_PWC * 8 + S4_RING * S4_PAIRS * 256 <= 160 * 1024, "v4 LDS");

// barrier for LDS hand-offs only: __syncthreads() also waits for every outstanding global store (its
// workgroup-scope release), which put the pool rows' HBM write latency (~1.8 us) into every v4 step
__device__ __forceinline__ void s4_lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

struct F3 {
  float a, b, c;
};
// 3-channel images: one 12-byte load per patch item (consecutive lanes = consecutive pixels, fully
// coalesced) instead of one 4-byte buffer load per channel; items outside the image read pixel 0 and
// are zeroed after the load, so no load sits behind a branch
template <int ITEMS, int NT>
__device__ __forceinline__ void get_rows3(float (&pv)[ITEMS][4], const float* __restrict__ xi, int tid, int row_end,
                                          int ih0, int H, int W, int pwc, int pad_l) {
  F3 v[ITEMS];
  bool ok[ITEMS];
#pragma unroll
  for (int k = 0; k < ITEMS; ++k) {
    const int idx = tid + k * NT;
    const int i = idx / ST_PWC, j = idx - i * ST_PWC;
    const int ih = ih0 + i, iw = j - pad_l;
    ok[k] = i < row_end && j < pwc && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
    v[k] = *(const F3*)(xi + (ok[k] ? (ih * W + iw) * 3 : 0));
  }
#pragma unroll
  for (int k = 0; k < ITEMS; ++k) {
    pv[k][0] = ok[k] ? v[k].a : 0.f;
    pv[k][1] = ok[k] ? v[k].b : 0.f;
    pv[k][2] = ok[k] ? v[k].c : 0.f;
    pv[k][3] = 0.f;
  }
}

// bf16 element offset of 16-byte channel chunk `chunk` of conv pixel `ow` in ring slot `slot`
__device__ __forceinline__ int ring4_off(int slot, int ow, int chunk) {
  const int pair = ow >> 1;
  const int u = (((ow & 1) << 3) | chunk) ^ (pair & 15);
  return ((slot * S4_PAIRS + pair) * 16 + u) * 8;
}
}  // namespace

// EXP (tools/stem_timeline.py --exp, outputs wrong by design): 1 no MFMAs in the steps, 2 no pool in the
// steps, 4 no ring stores in the steps, 8 no A-fragment reads in the steps
// NH: 16-channel groups per wave.  4 = every wave computes all 64 channels of its tiles (v4).  2 (v5): waves
// 0-3 take channels 0-31 and waves 4-7 channels 32-63 of every tile, so each wave loads half the weight
// panel and the 28 half-tiles of a step split 7 / 7 / 7 / 7 over the SIMDs (v4: 4 / 4 / 3 / 3 tiles).
// WL (v6): the 28 KB weight panel is loaded once per block (3.5 16-byte loads a thread) and staged in the
// not-yet-used ring area with a 232-element row pitch (conflict-free fragment reads), instead of every wave
// loading the whole panel from L2 (229 KB per CU, >= 1.7 us at the 64 B/clk L1 path)
template <bool C3, int EXP = 0, int NH = 4, bool WL = false>
__global__ __launch_bounds__(S4_NT, 1) void stem_pool_v4_kernel(const float* __restrict__ x, const bf16* __restrict__ w,
                                                                const float* __restrict__ bias, bf16* __restrict__ out,
                                                                int H, int W, int C, int OH, int OW, int pad_t,
                                                                int pad_l, int PH, int PW, int pool_pad, int groups,
                                                                unsigned long long* dbg_all) {
  __shared__ __attribute__((aligned(16))) bf16 patch[S4_PROWS * ST_PWC * 4];       // 63.4 KiB
  __shared__ __attribute__((aligned(16))) bf16 ring[S4_RING * S4_PAIRS * 16 * 8];  // 84 KiB

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int img = logical / groups;
  const int t0 = (logical - img * groups) * S4_SP;
  const int t1 = min(PH, t0 + S4_SP);                      // pool rows [t0, t1)
  const int r_first = 2 * t0 - pool_pad;                   // conv row of ring row 0 (may be -1)
  const int ih0 = 2 * r_first - pad_t;                     // input row of patch row 0
  const int row_end = 4 * (t1 - t0) + 7;
  const int tpr = (OW + 15) >> 4;
  const int pwc = 2 * tpr * 16 + 8;
  const float* xi = x + (size_t)img * H * W * C;
  // measurement only (tools/stem_timeline.py): per wave, shader clock at start / patch rows 0-10 in LDS /
  // step 0 done / steps done / end, wall clock at start and end
  unsigned long long* const dbg = dbg_all ? dbg_all + 8 * (wave + S4_WAVES * blockIdx.x) : nullptr;
  auto stamp = [&](int i) {
    if (dbg != nullptr && lane == 0) dbg[i] = __builtin_amdgcn_s_memtime();
  };
  stamp(0);
  if (dbg && lane == 0) dbg[6] = __builtin_amdgcn_s_memrealtime();

  // weights and bias first: loads return in order, so step 0 then waits only for them and patch rows 0-10
  const int fr = lane & 15, fq = lane >> 4;
  static_assert(NH == 4 || NH == 2, "whole or half channel panel per wave");
  constexpr int TSTRIDE = NH == 4 ? S4_WAVES : 4;          // tile index stride between a wave's tiles
  const int hsel = NH == 4 ? 0 : (wave >> 2);              // channel half (NH = 2)
  const int nb = hsel * NH;                                // first 16-channel group of this wave
  const int tfirst = NH == 4 ? wave : (((wave & 3) + 2 * hsel) & 3);
  bf16x8 bw[7][NH];
  constexpr int WPITCH = ST_K + 8;                         // staged row pitch (bf16): 464 B, 16 rows on 16 bank groups
  constexpr int WCH = 64 * ST_K / 8;                       // 16-byte chunks of the panel (1792)
  constexpr int WIT = (WCH + S4_NT - 1) / S4_NT;
  u32x4 wst[WL ? WIT : 1];
  if constexpr (WL) {
#pragma unroll
    for (int k = 0; k < WIT; ++k) {
      const int i = tid + k * S4_NT;
      if (i < WCH) wst[k] = ((const u32x4*)w)[i];
    }
  } else {
#pragma unroll
    for (int s = 0; s < 7; ++s)
#pragma unroll
      for (int n = 0; n < NH; ++n)
        bw[s][n] = *(const bf16x8*)(w + (size_t)((nb + n) * 16 + fr) * ST_K + s * 32 + fq * 8);
  }
  float b4[NH][4];
#pragma unroll
  for (int n = 0; n < NH; ++n)
#pragma unroll
    for (int r = 0; r < 4; ++r) b4[n][r] = bias[(nb + n) * 16 + 4 * fq + r];
  float pall[S4_ITEMS][4];
  if constexpr (C3)
    get_rows3<S4_ITEMS, S4_NT>(pall, xi, tid, row_end, ih0, H, W, pwc, pad_l);
  else
    get_rows<S4_ITEMS, S4_NT>(pall, xi, tid, 0, row_end, row_end, ih0, H, W, C, pwc, pad_l);
  if constexpr (WL) {
    // the panel's loads were issued before the patch's: these stores wait for them only
#pragma unroll
    for (int k = 0; k < WIT; ++k) {
      const int i = tid + k * S4_NT;
      if (i < WCH) *(u32x4*)(ring + (i / (ST_K / 8)) * WPITCH + (i % (ST_K / 8)) * 8) = wst[k];
    }
    s4_lds_barrier();
#pragma unroll
    for (int s = 0; s < 7; ++s)
#pragma unroll
      for (int n = 0; n < NH; ++n)
        bw[s][n] = *(const bf16x8*)(ring + ((nb + n) * 16 + fr) * WPITCH + s * 32 + fq * 8);
  }
  put_items<0, S4_ITEMS_A, S4_ITEMS, S4_NT>(pall, patch, tid, 0, S2_ROWS0);
  s4_lds_barrier();                                        // (WL: every wave's panel reads are done: the ring is free)
  stamp(1);

  // one 16-pixel x 64-channel conv tile: geometry / A-fragment reads / MFMAs / bias + ReLU into the ring.
  // ReLU after the bf16 rounding as a packed signed max with 0: the same bits as rounding max(y, 0)
  // (a value <= 0 rounds to a bf16 <= 0, including -0, which the integer max sends to +0)
  struct Tile {
    bool ok;
    int slot;                                              // ring slot base (bf16 elements)
    const bf16* pa;
    int col[NH];                                           // per 16-channel group: offset within the slot
  };
  auto tile_cols = [&](Tile& g, const int ow) __attribute__((always_inline)) {
#pragma unroll
    for (int n = 0; n < NH; ++n) g.col[n] = ring4_off(0, ow, 2 * (nb + n) + (fq >> 1)) + 4 * (fq & 1);
  };
  auto tile_geo = [&](const int mt, const int rel0, const int ntiles) __attribute__((always_inline)) {
    Tile g;
    const int q = mt / tpr;
    const int rel = rel0 + q, r = r_first + rel;
    g.ok = mt < ntiles && r >= 0 && r < OH;               // wave-uniform; the pool never reads skipped rows
    const int ow = (mt - q * tpr) * 16 + fr;
    g.slot = (rel % S4_RING) * (S4_PAIRS * 128);
    g.pa = patch + ((2 * rel) * ST_PWC + 2 * ow + 2 * fq) * 4;
    tile_cols(g, ow);
    return g;
  };
  auto tile_read = [&](const Tile& g, bf16x8 (&a)[7]) __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < 7; ++s) a[s] = *(const bf16x8*)(g.pa + s * ST_PWC * 4);
  };
  auto tile_mfma = [&](const bf16x8 (&a)[7], f32x4 (&acc)[NH]) __attribute__((always_inline)) {
#pragma unroll
    for (int n = 0; n < NH; ++n) acc[n] = (f32x4){0.f, 0.f, 0.f, 0.f};
    // (pinning the 4-MFMA groups in order with sched_barrier: no change, 10.37 vs 10.2 us of steps)
#pragma unroll
    for (int s = 0; s < 7; ++s)
#pragma unroll
      for (int n = 0; n < NH; ++n) acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[s][n], a[s], acc[n], 0, 0, 0);
  };
  // packed: v_pk_add_f32 (bias) + v_cvt_pk_bf16_f32 + v_pk_max_i16 per channel pair (the scalar form
  // compiled to one cvt per value plus a v_perm per pair)
  auto tile_store = [&](const Tile& g, const f32x4 (&acc)[NH]) __attribute__((always_inline)) {
#pragma unroll
    for (int n = 0; n < NH; ++n) {
      s16x2 h[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const f32x2 y = (f32x2){acc[n][2 * i], acc[n][2 * i + 1]} + (f32x2){b4[n][2 * i], b4[n][2 * i + 1]};
        h[i] = __builtin_elementwise_max(__builtin_bit_cast(s16x2, __builtin_convertvector(y, bf16x2v)),
                                         (s16x2){0, 0});
      }
      u32x2 w2 = {__builtin_bit_cast(unsigned, h[0]), __builtin_bit_cast(unsigned, h[1])};
      *(u32x2*)(ring + g.slot + g.col[n]) = w2;
    }
  };
  // the three phases of a tile with the measurement switches (EXP applies inside the step loop only)
  auto t_read = [&](const Tile& g, bf16x8 (&a)[7], auto in_steps) __attribute__((always_inline)) {
    if constexpr (decltype(in_steps)::value && (EXP & 8)) {
#pragma unroll
      for (int s = 0; s < 7; ++s) a[s] = bw[s][0];
    } else {
      tile_read(g, a);
    }
  };
  auto t_mfma = [&](const bf16x8 (&a)[7], f32x4 (&acc)[NH], auto in_steps) __attribute__((always_inline)) {
    if constexpr (decltype(in_steps)::value && (EXP & 1)) {
#pragma unroll
      for (int n = 0; n < NH; ++n) acc[n] = (f32x4){(float)a[0][0], (float)a[6][7], 0.f, 0.f};
    } else {
      tile_mfma(a, acc);
    }
  };
  auto t_store = [&](const Tile& g, const f32x4 (&acc)[NH], auto in_steps) __attribute__((always_inline)) {
    if constexpr (decltype(in_steps)::value && (EXP & 4)) {
      if (acc[0][0] == 12345.f && acc[NH - 1][1] == 1.f) ring[fr] = bf16(acc[0][0]);   // keep acc live
    } else {
      tile_store(g, acc);
    }
  };
  auto tile_run = [&](const Tile& g) __attribute__((always_inline)) {
    constexpr std::integral_constant<bool, false> no{};
    bf16x8 a[7];
    f32x4 acc[NH];
    t_read(g, a, no);
    t_mfma(a, acc, no);
    t_store(g, acc, no);
  };
  // conv rows [rel0, rel0 + nr) of the block (ring row index rel = conv row - r_first) -> ring
  auto conv_rows = [&](const int rel0, const int nr) __attribute__((always_inline)) {
    const int ntiles = nr * tpr;
    for (int mt = tfirst; mt < ntiles; mt += TSTRIDE) {
      const Tile g = tile_geo(mt, rel0, ntiles);
      if (g.ok) tile_run(g);
    }
  };
  // pool row t from conv rows 2t-pp .. 2t-pp+2 (non-negative bf16: packed integer max; the zero padding
  // is the 0 the max starts from).  A thread owns one item (chunk, pool column) for every row, pool
  // column fastest across lanes (PW * 8 <= 512 threads: host check), its three ring column offsets
  // hoisted.  Window positions outside the conv output are clamped to the nearest row / column, which is
  // inside the same window: a duplicate cannot change a max, and all nine reads issue without a branch.
  const bool pool_item = tid < PW * 8;
  const int pch8 = tid / PW, ppw = tid - pch8 * PW;
  int pcol[3];
#pragma unroll
  for (int dc = 0; dc < 3; ++dc) pcol[dc] = ring4_off(0, min(max(2 * ppw - pool_pad + dc, 0), OW - 1), pch8);
  bf16* const pout = out + ((size_t)img * PH * PW + ppw) * 64 + pch8 * 8;
  auto pool_read = [&](const int t, P8 (&v)[9]) __attribute__((always_inline)) {
    int rb[3];
#pragma unroll
    for (int dr = 0; dr < 3; ++dr) {
      const int oh = min(max(2 * t - pool_pad + dr, 0), OH - 1);
      rb[dr] = ((oh - r_first) % S4_RING) * (S4_PAIRS * 128);
    }
#pragma unroll
    for (int dr = 0; dr < 3; ++dr)
#pragma unroll
      for (int dc = 0; dc < 3; ++dc) v[3 * dr + dc].u = *(const u32x4*)(ring + rb[dr] + pcol[dc]);
  };
  auto pool_finish = [&](const int t, const P8 (&v)[9]) __attribute__((always_inline)) {
    P8 m = v[0];
#pragma unroll
    for (int i = 1; i < 9; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) m.h[e] = __builtin_elementwise_max(m.h[e], v[i].h[e]);
    *(u32x4*)(pout + (size_t)t * PW * 64) = m.u;
  };
  auto pool_row = [&](const int t) __attribute__((always_inline)) {
    if (!pool_item) return;
    P8 v[9];
    pool_read(t, v);
    pool_finish(t, v);
  };

  // step 0: conv rows 0..2; the rest of the patch lands under its MFMAs (step 1 reads patch rows <= 14)
  conv_rows(0, 3);
  put_items<S4_ITEMS_A - 1, S4_ITEMS - S4_ITEMS_A + 1, S4_ITEMS, S4_NT>(pall, patch, tid, S2_ROWS0, row_end);
  s4_lds_barrier();
  stamp(2);
  const int P = t1 - t0;
  // step k: conv rows 2k+1, 2k+2 and pool row k-1 from rows 2k-2 .. 2k (ring slots disjoint).  A wave's
  // (at most two) tiles sit at the same place of every step's row pair: their column geometry is computed
  // once.  (Interleaving a wave's pool reads / second tile's reads under its first tile's MFMAs by hand
  // measured slower: 22.4 vs 21.6 us.)
  {
    constexpr int TPW = NH == 4 ? 2 : 4;                   // most tiles a wave takes of a step's 14
    const int ntl = 2 * tpr;
    Tile g[TPW];
    int q[TPW];
    bool has[TPW];
    const bf16* p0[TPW];
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
      const int mt = tfirst + TSTRIDE * i;
      g[i] = tile_geo(mt, 0, ntl);
      q[i] = mt / tpr;
      has[i] = mt < ntl;
      p0[i] = g[i].pa - (2 * q[i]) * ST_PWC * 4;           // tile_geo(., 0, .) put rel = q in pa
    }
    for (int k = 1; k < P; ++k) {
      // (both tiles' MFMAs before both epilogues measured slower: 11.5 vs 10.2 us of steps)
      constexpr std::integral_constant<bool, true> yes{};
      const int t = t0 + k - 1;
#pragma unroll
      for (int i = 0; i < TPW; ++i) {
        const int rel = 2 * k + 1 + q[i];
        g[i].ok = has[i] && r_first + rel < OH;            // rel >= 3: never above the image
        g[i].slot = (rel % S4_RING) * (S4_PAIRS * 128);
        g[i].pa = p0[i] + (2 * rel) * ST_PWC * 4;
        if (g[i].ok) {
          bf16x8 a[7];
          f32x4 c[NH];
          t_read(g[i], a, yes);
          t_mfma(a, c, yes);
          t_store(g[i], c, yes);
        }
      }
      if (pool_item && !(EXP & 2)) pool_row(t);
      s4_lds_barrier();
    }
  }
  stamp(3);
  pool_row(t1 - 1);
  if (dbg) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stamp(4);
    if (lane == 0) dbg[7] = __builtin_amdgcn_s_memrealtime();
  }
}

static unsigned long long* g_stem_dbg = nullptr;
static int g_stem_exp = 0;
void stem_set_debug(unsigned long long* buf, int exp) {
  g_stem_dbg = buf;
  g_stem_exp = exp;
}

hipError_t stem_forward(const float* x, const bf16* w, const float* bias, bf16* out, int B, int H, int W, int C,
                        int OH, int OW, int pad_t, int pad_l, int pool, int PH, int PW, int pool_pad,
                        hipStream_t s) {
  if (C < 1 || C > 4 || OW < 1 || OW > ST_OWMAX || OH < 1 || B < 1) return hipErrorInvalidValue;
  if (pool) {
    if (PH < 1 || PW < 1 || PH > (OH + 2 * pool_pad - 3) / 2 + 1 || PW > (OW + 2 * pool_pad - 3) / 2 + 1)
      return hipErrorInvalidValue;
    // v2 walks S2_SP pool rows per block, so a small batch launches only a few
    // dozen blocks (8 at B=1): there the one-pool-row-per-block v1 grid fills more
    // CUs and wins.  ADAPT_STEM_V1=1 / =0 forces v1 / v2 (A/B switch).
    const int groups = (PH + S2_SP - 1) / S2_SP;
    // ADAPT_STEM_V1=1 / =0 / =3 / =4 / =6: v1 / v2 / v3 (v3: the row-group kernel with the whole patch
    // requested up front) / v4 (8 waves, pool of step k-1 beside the conv of step k) / v6 (v4 with the weight
    // panel loaded once per block, 3-channel images).  v5 / v7 (each wave on half the channels) and the v4
    // ablation builds were measurement variants (profiles/r5/stem_bf16_v4.md) and are no longer built.
    const char* v1 = getenv("ADAPT_STEM_V1");
    // default: v1 for small batches, above it v6 for 3-channel images (18.4 us vs v5's 20.4, v4's 21.1 and v3's
    // 26.1 at bs=32, profiles/r5/stem_bf16_v4.md), else v4
    const char ver = v1 && v1[0] ? v1[0]
                                 : (PH * B <= ST_V1_MAX_BLOCKS ? '1' : (PW * 8 <= S4_NT ? (C == 3 ? '6' : '4') : '3'));
    if (ver == '5' || ver == '7') return hipErrorInvalidValue;
    if (ver == '4' || ver == '6') {
      if (PW * 8 > S4_NT) return hipErrorInvalidValue;
      const int g4 = (PH + S4_SP - 1) / S4_SP;
      if (C == 3 && ver == '6') {
        hipLaunchKernelGGL(HIP_KERNEL_NAME(stem_pool_v4_kernel<true, 0, 4, true>), dim3(g4 * B), dim3(S4_NT), 0, s, x, w,
                           bias, out, H, W, C, OH, OW, pad_t, pad_l, PH, PW, pool_pad, g4, g_stem_dbg);
      } else if (C == 3) {
        hipLaunchKernelGGL(HIP_KERNEL_NAME(stem_pool_v4_kernel<true, 0>), dim3(g4 * B), dim3(S4_NT), 0, s, x, w, bias,
                           out, H, W, C, OH, OW, pad_t, pad_l, PH, PW, pool_pad, g4, g_stem_dbg);
      } else {
        hipLaunchKernelGGL(stem_pool_v4_kernel<false>, dim3(g4 * B), dim3(S4_NT), 0, s, x, w, bias, out, H, W, C, OH,
                           OW, pad_t, pad_l, PH, PW, pool_pad, g4, g_stem_dbg);
      }
      return hipGetLastError();
    }
    if (ver != '1') {
      if (ver == '3')
        hipLaunchKernelGGL(stem_pool_v2_kernel<true>, dim3(groups * B), dim3(S2_NT), 0, s, x, w, bias, out, H, W, C,
                           OH, OW, pad_t, pad_l, PH, PW, pool_pad, groups);
      else
        hipLaunchKernelGGL(stem_pool_v2_kernel<false>, dim3(groups * B), dim3(S2_NT), 0, s, x, w, bias, out, H, W, C,
                           OH, OW, pad_t, pad_l, PH, PW, pool_pad, groups);
      return hipGetLastError();
    }
    dim3 grid(PH * B);
    hipLaunchKernelGGL(stem_kernel<true>, grid, dim3(ST_NT), 0, s, x, w, bias, out, H, W, C, OH, OW, pad_t, pad_l,
                       PH, PW, pool_pad);
  } else {
    dim3 grid((OH + ST_CROWS_CONV - 1) / ST_CROWS_CONV * B);
    hipLaunchKernelGGL(stem_kernel<false>, grid, dim3(ST_NT), 0, s, x, w, bias, out, H, W, C, OH, OW, pad_t, pad_l,
                       0, 0, 0);
  }
  return hipGetLastError();
}

}  // namespace adapt
