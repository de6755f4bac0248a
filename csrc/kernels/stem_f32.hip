// fp32 ResNet stem in one launch: fp32 image -> 7x7/s2 conv (+folded BN, ReLU)
// -> 3x3/s2 max-pool, on the fp32 matrix cores (v_mfma_f32_16x16x4_f32).  The
// reference runs these as six Keras float32 layers inside `model.predict`
// (src/node.py:177; SURVEY §2.4 rows conv1_pad .. pool1_pool).
//
// The generic fp32 conv gathers the 3-channel image element by element and
// writes the 103 MB conv1 output for a separate max-pool: 169 + 29 us at bs=32
// (profiles/r2/fp32/r50_fp32_bs32_steps_r2r.json).  Here (the bf16 stem v2
// design, stem.hip, carried to fp32):
//
// * one block per (image, group of SF_SP pool rows); each step computes the two
//   new conv rows a pool row needs (three on the first step) into a 3-row LDS
//   ring and emits the pool row from it, so the conv output never leaves LDS;
// * input rows live in a 16-row LDS ring with the 3 channels packed
//   ([col][c]): the 21 (kw, c) taps of one filter row are 21 consecutive floats.
//   K is ordered so that every MFMA is real work: taps 0..19 of a filter row are
//   five float4 reads (35 K slots of 4 for the 7 rows), tap 20 of rows 0..3 is
//   a 4-row gather in the 36th slot and tap 20 of rows 4..6 is one more MFMA
//   (element 0 of the 37th slot): 37 MFMAs per 16 px x 16 ch tile for K = 147
//   (a 24-tap row layout needs 44, a 4-channel layout 56);
// * a step's 2 x 7 pixel tiles x 4 channel tiles are 56 (16 px x 16 ch) units,
//   7 per wave on 8 waves; a wave always works on the same 16 channels, so its
//   A operand (the weights: 9 float4 + 1 float per lane) stays in VGPRs;
// * the next step's 4 input rows are loaded into registers before this step's
//   MFMAs and land in LDS after them;
// * each unit keeps two accumulators (even / odd K halves): two independent
//   MFMA chains instead of one 37-long dependent chain.
#include "kernels.h"

namespace adapt {
namespace {

constexpr int SF_SP = 7;                     // pool rows per block
constexpr int SF_WAVES = 8;
constexpr int SF_NT = SF_WAVES * 64;
constexpr int SF_OWMAX = 112;
constexpr int SF_COLS = 2 * SF_OWMAX + 8;    // patch columns (input col + pad_l)
constexpr int SF_OFF = 4;                    // row origin: even, so 6*ow + j + OFF stays 8-byte aligned
constexpr int SF_ROWLEN = 704;               // >= SF_OFF + SF_COLS * 3, 16-byte multiple
constexpr int SF_RING = 16;                  // input-row ring
constexpr int SF_K = 160;                    // packed weight row: 9 full halves of 16 + element 0 of 4 slots
constexpr int SF_KH = 9;                     // full K halves (4 MFMAs each); one single MFMA follows
static_assert(SF_OFF + SF_COLS * 3 <= SF_ROWLEN, "row length");

typedef float f32x2 __attribute__((ext_vector_type(2)));

// conv ring [3][112 px][16 chunks of 4 ch], chunk XOR-swizzled by the pixel so
// the 16 pixels of a C^T fragment store spread over the banks
__device__ __forceinline__ int cring_off(int slot, int px, int chunk) {
  return ((slot * SF_OWMAX + px) * 16 + (chunk ^ (px & 15))) * 4;
}

// one unit's B operand: 8 K halves, the gathered half 8, element 0 of the last MFMA
struct StemB {
  f32x4 h[SF_KH - 1];
  f32x4 g8;
  float g9;
};

}  // namespace

constexpr int SF_TPR = SF_OWMAX / 16;        // variant 2: pixel tiles of a 112-wide conv row

// V = 0: one unit (16 px x 16 ch) at a time; 1: units software-pipelined; 2: each wave of a pair
// takes a whole conv row per step, its 7 tiles unrolled with every LDS address a per-row base plus
// an immediate (OW = 112 only)
// the step barriers hand off LDS only (patch rows, conv ring): __syncthreads() would also wait for the pool
// rows' global stores still in flight (its workgroup-scope release), an HBM write round trip per step
__device__ __forceinline__ void sf_lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int V>
__global__ __launch_bounds__(SF_NT, 1) void stem_pool_f32_kernel(const float* __restrict__ x,
                                                                 const float* __restrict__ w,
                                                                 const float* __restrict__ bias,
                                                                 float* __restrict__ out, int H, int W, int OH,
                                                                 int OW, int pad_t, int pad_l, int PH, int PW,
                                                                 int pool_pad, int groups) {
  __shared__ __attribute__((aligned(16))) float patch[SF_RING * SF_ROWLEN];     // 44 KiB
  __shared__ __attribute__((aligned(16))) float cring[3 * SF_OWMAX * 64];       // 84 KiB

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int img = logical / groups;
  const int t0 = (logical - img * groups) * SF_SP;
  const int t1 = min(PH, t0 + SF_SP);
  const int tpr = (OW + 15) >> 4;
  const float* xi = x + (size_t)img * H * W * 3;
  const int c4row = W * 3 / 4;               // float4 chunks of one image row (W % 4 == 0)

  // zero the whole patch once: pad columns are never written again, rows outside
  // the image are written as zeros by the staging below
  for (int i = tid; i < SF_RING * SF_ROWLEN / 4; i += SF_NT) *(f32x4*)(patch + i * 4) = (f32x4){0.f, 0.f, 0.f, 0.f};

  // input rows [ih_lo, ih_lo + n): loads to registers / stores to their ring slots
  constexpr int MAXC = (11 * (SF_OWMAX * 2 * 3 / 4) + SF_NT - 1) / SF_NT;   // chunks per thread, 11 rows
  auto get_rows = [&](f32x4 (&v)[MAXC], int ih_lo, int n) {
#pragma unroll
    for (int k = 0; k < MAXC; ++k) {
      const int idx = tid + k * SF_NT;
      const int r = idx / c4row, c = idx - r * c4row;
      const int ih = ih_lo + r;
      v[k] = (f32x4){0.f, 0.f, 0.f, 0.f};
      if (r < n && (unsigned)ih < (unsigned)H) v[k] = *(const f32x4*)(xi + (size_t)ih * W * 3 + c * 4);
    }
  };
  auto put_rows = [&](const f32x4 (&v)[MAXC], int ih_lo, int n) {
#pragma unroll
    for (int k = 0; k < MAXC; ++k) {
      const int idx = tid + k * SF_NT;
      const int r = idx / c4row, c = idx - r * c4row;
      if (r >= n) continue;
      float* row = patch + ((ih_lo + r + 4 * SF_RING) % SF_RING) * SF_ROWLEN + SF_OFF + pad_l * 3 + c * 4;
      row[0] = v[k][0]; row[1] = v[k][1]; row[2] = v[k][2]; row[3] = v[k][3];
    }
  };

  const int r_first = 2 * t0 - pool_pad;     // first conv row (may be -1)
  // first step: conv rows r_first .. r_first+2 need input rows 2*r_first-pad_t .. +10
  __syncthreads();
  {
    f32x4 v0[MAXC];
    get_rows(v0, 2 * r_first - pad_t, 11);
    put_rows(v0, 2 * r_first - pad_t, 11);
  }
  // weights of this wave's 16 channels: A operand, lane = (channel fr, k group fq)
  const int fr = lane & 15, fq = lane >> 4;
  const int ct = wave & 3;
  f32x4 wa[SF_KH];
#pragma unroll
  for (int h = 0; h < SF_KH; ++h) wa[h] = *(const f32x4*)(w + (size_t)(ct * 16 + fr) * SF_K + h * 16 + fq * 4);
  float wa9 = w[(size_t)(ct * 16 + fr) * SF_K + SF_KH * 16 + fq * 4];
  f32x4 b4 = *(const f32x4*)(bias + ct * 16 + fq * 4);
  // per-lane k layout: slot p = 4h + fq (h < 8) is filter row p / 5, taps 4 (p % 5) .. +3;
  // half 8: slots 32..34 likewise (row 6), slot 35 (fq = 3) is tap 20 of rows 0..3;
  // the last MFMA: lane fq supplies tap 20 of row 4 + fq (fq = 3: zero weight, row 4 read)
  int koff[SF_KH - 1];
#pragma unroll
  for (int h = 0; h < SF_KH - 1; ++h) {
    const int p = 4 * h + fq;
    koff[h] = (p / 5) * 0x10000 + 4 * (p % 5);                  // (filter row, first tap) packed
  }
  const bool g8 = fq == 3;
  const int j8 = g8 ? 20 : 4 * (fq + 2);                        // half 8: tap of element 0
  const int r9 = fq < 3 ? 4 + fq : 4;                           // last MFMA: filter row
  // the weights must have landed before the step loop: otherwise the wait-count pass, which cannot
  // tell the first unit from the others, puts vmcnt waits for them between the MFMAs of every unit,
  // and those also wait for the next step's input rows (issued just before the units).  The empty
  // asm consumes and redefines each register, so the loads complete here and cannot sink below.
#pragma unroll
  for (int h = 0; h < SF_KH; ++h) asm volatile("" : "+v"(wa[h]));
  asm volatile("" : "+v"(wa9));
  asm volatile("" : "+v"(b4));
  __syncthreads();

  for (int t = t0; t < t1; ++t) {
    const bool first = t == t0;
    const int ra = first ? r_first : 2 * t - pool_pad + 1;     // first conv row this step computes
    const int nr = first ? 3 : 2;
    // the next step's 4 input rows, in flight during this step's MFMAs
    const bool more = t + 1 < t1;
    // step t+1 computes conv rows ra' = 2(t+1) - pp + 1 and ra' + 1, which need input rows
    // 2ra' - pad_t .. 2ra' - pad_t + 8; rows up to 2ra' - pad_t + 4 are staged already
    const int nxt_lo = 2 * (2 * (t + 1) - pool_pad + 1) - pad_t + 5;
    f32x4 pv[MAXC];
    if (more) get_rows(pv, nxt_lo, 4);
    const int units = nr * tpr;                                 // pixel tiles this step (x 4 channel tiles)
    // unit u: conv row ra + u / tpr, pixels c0 .. c0+15 (ragged last tile: clamp the read, skip the store)
    auto load_unit = [&](int u, StemB& b) {
      const int q = u / tpr;
      const int r = ra + q;
      const int c0 = (u - q * tpr) * 16;
      const int ow = min(c0 + fr, OW - 1);
      // ring row of filter row s: (2r - pad_t + s) mod 16, with the sum + 64 > 0, so a mask, not a signed %
      const unsigned rb = (unsigned)(2 * r - pad_t + 4 * SF_RING);
      const float* pcol = patch + SF_OFF + 6 * ow;
#pragma unroll
      for (int h = 0; h < SF_KH - 1; ++h) {
        const int sr = koff[h] >> 16, j = koff[h] & 0xffff;
        const float* src = pcol + ((rb + sr) & (SF_RING - 1)) * SF_ROWLEN + j;
        const f32x2 lo = *(const f32x2*)src, hi = *(const f32x2*)(src + 2);
        b.h[h] = (f32x4){lo[0], lo[1], hi[0], hi[1]};
      }
      // half 8: lanes fq < 3 read taps j8 .. j8+3 of row 6, lane group 3 gathers tap 20 of rows 0..3
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int sr = g8 ? e : 6;
        b.g8[e] = pcol[((rb + sr) & (SF_RING - 1)) * SF_ROWLEN + j8 + (g8 ? 0 : e)];
      }
      b.g9 = pcol[((rb + r9) & (SF_RING - 1)) * SF_ROWLEN + 20];
    };
    // 37 MFMAs; the even / odd K halves alternate MFMA by MFMA: two independent chains back to back
    // instead of runs of four dependent MFMAs (40-cycle dependent latency vs 32-cycle issue)
    auto run_unit = [&](int u, const StemB& b) {
      f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int h = 0; h < SF_KH - 1; h += 2)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[h][e], b.h[h][e], acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[h + 1][e], b.h[h + 1][e], acc1, 0, 0, 0);
        }
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[8][0], b.g8[0], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[8][1], b.g8[1], acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[8][2], b.g8[2], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[8][3], b.g8[3], acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(wa9, b.g9, acc0, 0, 0, 0);
      // C^T fragment: channel = 16ct + 4fq + e, pixel = c0 + fr; rows outside the image are
      // computed (their ring reads are in bounds) and dropped here
      const int q = u / tpr;
      const int r = ra + q;
      const int c0 = (u - q * tpr) * 16;
      if (r >= 0 && r < OH && c0 + fr < OW) {
        f32x4 y = acc0 + acc1 + b4;
        y[0] = fmaxf(y[0], 0.f); y[1] = fmaxf(y[1], 0.f); y[2] = fmaxf(y[2], 0.f); y[3] = fmaxf(y[3], 0.f);
        *(f32x4*)(cring + cring_off((r + 3) % 3, c0 + fr, ct * 4 + fq)) = y;
      }
    };
    const int u0 = wave >> 2;                                   // this wave's units: u0, u0 + 2, ...
    if constexpr (V >= 2) {
      // The unit loops spend ~150 VALU per unit (8 ring-row addresses, the gather, the unit's
      // geometry, the ring store address: 7.9k VALU per wave for 1.9k MFMAs, profiles/r4/pmc_stem_r4j.txt),
      // and the two waves of a SIMD reach that VALU phase together.  A whole row has one ring base
      // per K half; its tiles are 96 floats apart in the patch and 1024 apart in the conv ring.
      if (first) {                                              // the extra first row, split 4 / 3
        for (int u = u0; u < tpr; u += 2) {
          StemB b;
          load_unit(u, b);
          run_unit(u, b);
        }
      }
      const int r = ra + (first ? 1 : 0) + u0;
      if (r >= 0 && r < OH) {                                   // wave-uniform
        const int rb = 2 * r - pad_t + 4 * SF_RING;
        const int pbase = SF_OFF + 6 * fr;
        int ah[SF_KH - 1], ag[4];
#pragma unroll
        for (int h = 0; h < SF_KH - 1; ++h)
          ah[h] = pbase + ((rb + (koff[h] >> 16)) & (SF_RING - 1)) * SF_ROWLEN + (koff[h] & 0xffff);
#pragma unroll
        for (int e = 0; e < 4; ++e) ag[e] = pbase + ((rb + (g8 ? e : 6)) & (SF_RING - 1)) * SF_ROWLEN + j8 + (g8 ? 0 : e);
        const int a9 = pbase + ((rb + r9) & (SF_RING - 1)) * SF_ROWLEN + 20;
        float* cdst = cring + cring_off((r + 3) % 3, fr, ct * 4 + fq);
#pragma unroll
        for (int c = 0; c < SF_TPR; ++c) {
          const int po = c * 96;                                // 16 pixels x 6 floats
          f32x4 acc0 = b4, acc1 = {0.f, 0.f, 0.f, 0.f};
          f32x4 bh[SF_KH - 1];
#pragma unroll
          for (int h = 0; h < SF_KH - 1; ++h) {
            const f32x2 lo = *(const f32x2*)(patch + ah[h] + po), hi = *(const f32x2*)(patch + ah[h] + po + 2);
            bh[h] = (f32x4){lo[0], lo[1], hi[0], hi[1]};
          }
          f32x4 b8;
#pragma unroll
          for (int e = 0; e < 4; ++e) b8[e] = patch[ag[e] + po];
          const float b9 = patch[a9 + po];
#pragma unroll
          for (int h = 0; h < SF_KH - 1; h += 2)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[h][e], bh[h][e], acc0, 0, 0, 0);
              acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[h + 1][e], bh[h + 1][e], acc1, 0, 0, 0);
            }
          acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[8][0], b8[0], acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[8][1], b8[1], acc1, 0, 0, 0);
          acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[8][2], b8[2], acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[8][3], b8[3], acc1, 0, 0, 0);
          acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(wa9, b9, acc0, 0, 0, 0);
          f32x4 y = acc0 + acc1;
          y[0] = fmaxf(y[0], 0.f); y[1] = fmaxf(y[1], 0.f); y[2] = fmaxf(y[2], 0.f); y[3] = fmaxf(y[3], 0.f);
          *(f32x4*)(cdst + c * 1024) = y;
        }
      }
    } else if constexpr (V == 0) {
      for (int u = u0; u < units; u += 2) {
        StemB b;
        load_unit(u, b);
        run_unit(u, b);
      }
    } else {
      // software-pipelined: the next unit's B operand (21 LDS reads) is in flight under this unit's
      // 37 MFMAs.  Unpipelined, the two waves of a SIMD leave every step's barrier in lockstep and
      // wait on their LDS reads at the same time, so the matrix core idled between units (MFMA busy
      // 0.50, profiles/r4/roofline_r50_fp32_bs32.txt).  Out-of-range prefetches re-read the last unit.
      const int last = units - 1 - ((units - 1 - u0) & 1);
      StemB ba, bb;
      load_unit(u0, ba);
      for (int u = u0; u < units; u += 4) {
        load_unit(min(u + 2, last), bb);
        __builtin_amdgcn_sched_barrier(0);
        run_unit(u, ba);
        load_unit(min(u + 4, last), ba);
        __builtin_amdgcn_sched_barrier(0);
        if (u + 2 < units) run_unit(u + 2, bb);
      }
    }
    if (more) put_rows(pv, nxt_lo, 4);
    sf_lds_barrier();
    // pool row t from conv rows 2t-pp .. 2t-pp+2; post-ReLU values are >= 0, so the
    // zero padding is the 0 the max starts from
    // (all 9 reads unconditional, out-of-image taps clamped and masked to 0, so they issue back to back)
    for (int idx = tid; idx < PW * 16; idx += SF_NT) {
      const int ch = idx & 15, pw = idx >> 4;
      f32x4 v[3][3];
#pragma unroll
      for (int dr = 0; dr < 3; ++dr) {
        const int oh = 2 * t - pool_pad + dr;
        const int ohc = min(max(oh, 0), OH - 1);
#pragma unroll
        for (int dc = 0; dc < 3; ++dc) {
          const int oc = 2 * pw - pool_pad + dc;
          const int occ = min(max(oc, 0), OW - 1);
          v[dr][dc] = *(const f32x4*)(cring + cring_off((ohc + 3) % 3, occ, ch));
        }
      }
      f32x4 m = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int dr = 0; dr < 3; ++dr) {
        const int oh = 2 * t - pool_pad + dr;
#pragma unroll
        for (int dc = 0; dc < 3; ++dc) {
          const int oc = 2 * pw - pool_pad + dc;
          if ((unsigned)oh >= (unsigned)OH || (unsigned)oc >= (unsigned)OW) continue;
          m[0] = fmaxf(m[0], v[dr][dc][0]); m[1] = fmaxf(m[1], v[dr][dc][1]);
          m[2] = fmaxf(m[2], v[dr][dc][2]); m[3] = fmaxf(m[3], v[dr][dc][3]);
        }
      }
      *(f32x4*)(out + (((size_t)img * PH + t) * PW + pw) * 64 + ch * 4) = m;
    }
    sf_lds_barrier();                                           // ring slots of rows 2t-pp, 2t-pp+1 are free
  }
}

// ---------------------------------------------------------------- variant 5
// Variant 2's whole-row conv with the max-pool split in two and taken off the step's critical path
// (variant 2 spends a pool phase between two barriers every step, with no MFMA in flight on the CU):
// * horizontal, in the conv epilogue: a tile's C^T fragment holds 16 consecutive pixels in the 16 lanes
//   of a DPP row, so the 3-wide / stride-2 max at the even pixels is two row shifts (lane 0's left
//   neighbour is lane 15 of the row's previous tile: a row rotate of that tile's result); the half-width
//   row (56 x 64) goes to a 5-row LDS ring;
// * vertical: pool row t - 1 (3 ring reads per output instead of 9) runs in step t next to step t's conv
//   rows, so a step has one barrier and the MFMA bursts of consecutive steps are back to back.
// The first step's extra conv row is split at tile 3 / 4 between the wave sets, the second set recomputing
// tile 3 for its carry (4 tiles each).
constexpr int SF_HP = SF_OWMAX / 2;          // half-width (horizontally pooled) row
constexpr int SF_HR = 5;                     // ring rows: pool t - 1 reads 2t-3 .. 2t-1 while step t writes 2t, 2t+1

namespace {
__device__ __forceinline__ int hring_off(int slot, int pc, int chunk) {
  return ((slot * SF_HP + pc) * 16 + (chunk ^ (pc & 15))) * 4;
}

// row shifts of the 16-lane DPP rows, per component.  Inline asm: through __builtin_amdgcn_update_dpp /
// mov_dpp the compiler (ROCm 7.2) folded the four components' moves into the first one's and fed that to
// all four maxes.  The s_nop 1 covers the VALU-write -> DPP-read hazard inside the statement.  Source lanes
// outside the row leave the destination undefined; those lanes' results are never used.
#define ADAPT_SF_DPP(NAME, CTRL)                                                                          \
  __device__ __forceinline__ f32x4 NAME(f32x4 v) {                                                        \
    f32x4 r;                                                                                              \
    asm volatile("s_nop 1\n\tv_mov_b32_dpp %0, %4 " CTRL " row_mask:0xf bank_mask:0xf\n\t"              \
                 "v_mov_b32_dpp %1, %5 " CTRL " row_mask:0xf bank_mask:0xf\n\t"                            \
                 "v_mov_b32_dpp %2, %6 " CTRL " row_mask:0xf bank_mask:0xf\n\t"                            \
                 "v_mov_b32_dpp %3, %7 " CTRL " row_mask:0xf bank_mask:0xf"                                 \
                 : "=&v"(r.x), "=&v"(r.y), "=&v"(r.z), "=&v"(r.w)                                        \
                 : "v"(v.x), "v"(v.y), "v"(v.z), "v"(v.w));                                               \
    return r;                                                                                             \
  }
ADAPT_SF_DPP(sf_shl1, "row_shl:1")           // lane i <- lane i + 1 of its row of 16
ADAPT_SF_DPP(sf_shr1, "row_shr:1")           // lane i <- lane i - 1
ADAPT_SF_DPP(sf_ror1, "row_ror:1")           // lane i <- lane (i - 1) mod 16
#undef ADAPT_SF_DPP

__device__ __forceinline__ f32x4 max4(f32x4 a, f32x4 b) {
  return (f32x4){fmaxf(a[0], b[0]), fmaxf(a[1], b[1]), fmaxf(a[2], b[2]), fmaxf(a[3], b[3])};
}
}  // namespace

// PIPE (variant 6): a whole row's tiles with the next tile's 21 LDS operand reads issued ahead of this tile's
// 37 MFMAs (two operand sets, alternating over the unrolled tiles), so the read latency hides under the MFMA
// burst instead of sitting in front of it (the two waves of a SIMD reach each tile start together)
template <bool PIPE>
__global__ __launch_bounds__(SF_NT, 1) void stem_hpool_f32_kernel(const float* __restrict__ x,
                                                                  const float* __restrict__ w,
                                                                  const float* __restrict__ bias,
                                                                  float* __restrict__ out, int H, int W, int OH,
                                                                  int pad_t, int pad_l, int PH, int groups) {
  __shared__ __attribute__((aligned(16))) float patch[SF_RING * SF_ROWLEN];     // 44 KiB
  __shared__ __attribute__((aligned(16))) float hring[SF_HR * SF_HP * 64];      // 70 KiB
  constexpr int PW = SF_HP;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int img = logical / groups;
  const int t0 = (logical - img * groups) * SF_SP;
  const int t1 = min(PH, t0 + SF_SP);
  const float* xi = x + (size_t)img * H * W * 3;
  const int c4row = W * 3 / 4;

  for (int i = tid; i < SF_RING * SF_ROWLEN / 4; i += SF_NT) *(f32x4*)(patch + i * 4) = (f32x4){0.f, 0.f, 0.f, 0.f};

  constexpr int MAXC = (11 * (SF_OWMAX * 2 * 3 / 4) + SF_NT - 1) / SF_NT;
  auto get_rows = [&](f32x4 (&v)[MAXC], int ih_lo, int n) {
#pragma unroll
    for (int k = 0; k < MAXC; ++k) {
      const int idx = tid + k * SF_NT;
      const int r = idx / c4row, c = idx - r * c4row;
      const int ih = ih_lo + r;
      v[k] = (f32x4){0.f, 0.f, 0.f, 0.f};
      if (r < n && (unsigned)ih < (unsigned)H) v[k] = *(const f32x4*)(xi + (size_t)ih * W * 3 + c * 4);
    }
  };
  auto put_rows = [&](const f32x4 (&v)[MAXC], int ih_lo, int n) {
#pragma unroll
    for (int k = 0; k < MAXC; ++k) {
      const int idx = tid + k * SF_NT;
      const int r = idx / c4row, c = idx - r * c4row;
      if (r >= n) continue;
      float* row = patch + ((ih_lo + r + 4 * SF_RING) % SF_RING) * SF_ROWLEN + SF_OFF + pad_l * 3 + c * 4;
      row[0] = v[k][0]; row[1] = v[k][1]; row[2] = v[k][2]; row[3] = v[k][3];
    }
  };

  const int r_first = 2 * t0 - 1;            // pool_pad 1: the first step's conv rows r_first .. r_first + 2
  __syncthreads();
  {
    f32x4 v0[MAXC];
    get_rows(v0, 2 * r_first - pad_t, 11);
    put_rows(v0, 2 * r_first - pad_t, 11);
  }
  const int fr = lane & 15, fq = lane >> 4;
  const int ct = wave & 3;
  f32x4 wa[SF_KH];
#pragma unroll
  for (int h = 0; h < SF_KH; ++h) wa[h] = *(const f32x4*)(w + (size_t)(ct * 16 + fr) * SF_K + h * 16 + fq * 4);
  float wa9 = w[(size_t)(ct * 16 + fr) * SF_K + SF_KH * 16 + fq * 4];
  f32x4 b4 = *(const f32x4*)(bias + ct * 16 + fq * 4);
  int koff[SF_KH - 1];
#pragma unroll
  for (int h = 0; h < SF_KH - 1; ++h) {
    const int p = 4 * h + fq;
    koff[h] = (p / 5) * 0x10000 + 4 * (p % 5);
  }
  const bool g8 = fq == 3;
  const int j8 = g8 ? 20 : 4 * (fq + 2);
  const int r9 = fq < 3 ? 4 + fq : 4;
#pragma unroll
  for (int h = 0; h < SF_KH; ++h) asm volatile("" : "+v"(wa[h]));
  asm volatile("" : "+v"(wa9));
  asm volatile("" : "+v"(b4));
  __syncthreads();

  // conv row r, tiles cb .. ce - 1 (wave-uniform), for this wave's 16 channels; the half-width pooled
  // values of tiles >= st go to the ring
  auto conv_row = [&](int r, int cb, int ce, int st) {
    if (r < 0 || r >= OH) return;
    const int rb = 2 * r - pad_t + 4 * SF_RING;
    const int pbase = SF_OFF + 6 * fr;
    int ah[SF_KH - 1], ag[4];
#pragma unroll
    for (int h = 0; h < SF_KH - 1; ++h)
      ah[h] = pbase + ((rb + (koff[h] >> 16)) & (SF_RING - 1)) * SF_ROWLEN + (koff[h] & 0xffff);
#pragma unroll
    for (int e = 0; e < 4; ++e) ag[e] = pbase + ((rb + (g8 ? e : 6)) & (SF_RING - 1)) * SF_ROWLEN + j8 + (g8 ? 0 : e);
    const int a9 = pbase + ((rb + r9) & (SF_RING - 1)) * SF_ROWLEN + 20;
    const int slot = r % SF_HR;
    const bool even = (fr & 1) == 0;
    f32x4 prev = {0.f, 0.f, 0.f, 0.f};
    if constexpr (PIPE) {
      if (cb == 0 && ce == SF_TPR && st == 0) {           // a whole row (wave-uniform)
        // the 8 float4 halves are read a tile ahead; the gathered half and the last element (5 reads, used by
        // the tile's last 5 MFMAs) are read at the tile's start
        struct Ops {
          f32x4 h[SF_KH - 1];
        };
        auto load = [&](int c, Ops& o) __attribute__((always_inline)) {
          const int po = c * 96;
#pragma unroll
          for (int h = 0; h < SF_KH - 1; ++h) {
            const f32x2 lo = *(const f32x2*)(patch + ah[h] + po), hi = *(const f32x2*)(patch + ah[h] + po + 2);
            o.h[h] = (f32x4){lo[0], lo[1], hi[0], hi[1]};
          }
        };
        Ops oa, ob;
        load(0, oa);
#pragma unroll
        for (int c = 0; c < SF_TPR; ++c) {
          Ops& cur = (c & 1) ? ob : oa;
          Ops& nxt = (c & 1) ? oa : ob;
          f32x4 g8;
#pragma unroll
          for (int e = 0; e < 4; ++e) g8[e] = patch[ag[e] + c * 96];
          const float g9 = patch[a9 + c * 96];
          if (c + 1 < SF_TPR) load(c + 1, nxt);
          __builtin_amdgcn_sched_barrier(0);
          f32x4 acc0 = b4, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int h = 0; h < SF_KH - 1; h += 2)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[h][e], cur.h[h][e], acc0, 0, 0, 0);
              acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[h + 1][e], cur.h[h + 1][e], acc1, 0, 0, 0);
            }
          acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[8][0], g8[0], acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[8][1], g8[1], acc1, 0, 0, 0);
          acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[8][2], g8[2], acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[8][3], g8[3], acc1, 0, 0, 0);
          acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(wa9, g9, acc0, 0, 0, 0);
          f32x4 y = max4(acc0 + acc1, (f32x4){0.f, 0.f, 0.f, 0.f});
          const f32x4 rgt = sf_shl1(y), lsh = sf_shr1(y), lro = sf_ror1(prev);
          const f32x4 lft = fr == 0 ? lro : lsh;
          if (even) *(f32x4*)(hring + hring_off(slot, 8 * c + (fr >> 1), ct * 4 + fq)) = max4(max4(lft, y), rgt);
          prev = y;
        }
        return;
      }
    }
#pragma unroll
    for (int c = 0; c < SF_TPR; ++c) {
      if (c < cb || c >= ce) continue;
      const int po = c * 96;
      f32x4 acc0 = b4, acc1 = {0.f, 0.f, 0.f, 0.f};
      f32x4 bh[SF_KH - 1];
#pragma unroll
      for (int h = 0; h < SF_KH - 1; ++h) {
        const f32x2 lo = *(const f32x2*)(patch + ah[h] + po), hi = *(const f32x2*)(patch + ah[h] + po + 2);
        bh[h] = (f32x4){lo[0], lo[1], hi[0], hi[1]};
      }
      f32x4 b8;
#pragma unroll
      for (int e = 0; e < 4; ++e) b8[e] = patch[ag[e] + po];
      const float b9 = patch[a9 + po];
#pragma unroll
      for (int h = 0; h < SF_KH - 1; h += 2)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[h][e], bh[h][e], acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[h + 1][e], bh[h + 1][e], acc1, 0, 0, 0);
        }
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[8][0], b8[0], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[8][1], b8[1], acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[8][2], b8[2], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[8][3], b8[3], acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(wa9, b9, acc0, 0, 0, 0);
      f32x4 y = acc0 + acc1;
      y = max4(y, (f32x4){0.f, 0.f, 0.f, 0.f});
      // post-ReLU values are >= 0, so the pad column left of the image is the 0 the carry starts from
      const f32x4 rgt = sf_shl1(y), lsh = sf_shr1(y), lro = sf_ror1(prev);
      const f32x4 lft = fr == 0 ? lro : lsh;
      if (c >= st && even) *(f32x4*)(hring + hring_off(slot, 8 * c + (fr >> 1), ct * 4 + fq)) = max4(max4(lft, y), rgt);
      prev = y;
    }
  };
  // pool row tp from the half-width rows 2tp - 1 .. 2tp + 1 (rows outside the map are skipped: the max of
  // post-ReLU values starts from 0)
  auto pool_row = [&](int tp) {
    for (int idx = tid; idx < PW * 16; idx += SF_NT) {
      const int ch = idx & 15, pc = idx >> 4;
      f32x4 m = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int dr = 0; dr < 3; ++dr) {
        const int oh = 2 * tp - 1 + dr;
        if ((unsigned)oh < (unsigned)OH) m = max4(m, *(const f32x4*)(hring + hring_off(oh % SF_HR, pc, ch)));
      }
      *(f32x4*)(out + (((size_t)img * PH + tp) * PW + pc) * 64 + ch * 4) = m;
    }
  };

  const int set = wave >> 2;                 // wave sets: 4 waves (one per channel tile) each
  for (int t = t0; t < t1; ++t) {
    const bool first = t == t0, more = t + 1 < t1;
    const int nxt_lo = 2 * (2 * (t + 1)) - pad_t + 5;
    f32x4 pv[MAXC];
    if (more) get_rows(pv, nxt_lo, 4);
    if (!first) pool_row(t - 1);
    if (first) {
      conv_row(r_first, set ? 3 : 0, set ? SF_TPR : 4, set ? 4 : 0);
      conv_row(r_first + 1 + set, 0, SF_TPR, 0);
    } else {
      conv_row(2 * t + set, 0, SF_TPR, 0);
    }
    if (more) put_rows(pv, nxt_lo, 4);
    sf_lds_barrier();
  }
  pool_row(t1 - 1);
}

// weights [64][160] fp32 in the slot order above (ops/conv.py pack_stem_f32); image NHWC, C = 3
bool stem_f32_supported(int C, int W, int OW, int pool_pad) {
  return C == 3 && W % 4 == 0 && OW >= 1 && OW <= SF_OWMAX && 2 * OW + 8 <= SF_COLS && pool_pad == 1;
}

hipError_t stem_f32_forward(const float* x, const float* w, const float* bias, float* out, int B, int H, int W, int C,
                            int OH, int OW, int pad_t, int pad_l, int PH, int PW, int pool_pad, hipStream_t s,
                            int variant) {
  if (!stem_f32_supported(C, W, OW, pool_pad) || pad_l != 3 || variant < 0 || variant > 6 || variant == 3 ||
      variant == 4 || B < 1 || PH < 1 || PW < 1 || PH > (OH + 2 * pool_pad - 3) / 2 + 1 ||
      PW > (OW + 2 * pool_pad - 3) / 2 + 1 || W + pad_l > SF_COLS)
    return hipErrorInvalidValue;
  const int groups = (PH + SF_SP - 1) / SF_SP;
  if (variant >= 2 && (OW != 16 * SF_TPR || (variant >= 5 && PW != SF_HP))) variant = 1;   // 112-wide rows only
  if (variant == 0)
    hipLaunchKernelGGL(stem_pool_f32_kernel<0>, dim3(groups * B), dim3(SF_NT), 0, s, x, w, bias, out, H, W, OH, OW,
                       pad_t, pad_l, PH, PW, pool_pad, groups);
  else if (variant == 1)
    hipLaunchKernelGGL(stem_pool_f32_kernel<1>, dim3(groups * B), dim3(SF_NT), 0, s, x, w, bias, out, H, W, OH, OW,
                       pad_t, pad_l, PH, PW, pool_pad, groups);
  else if (variant == 2)
    hipLaunchKernelGGL(stem_pool_f32_kernel<2>, dim3(groups * B), dim3(SF_NT), 0, s, x, w, bias, out, H, W, OH, OW,
                       pad_t, pad_l, PH, PW, pool_pad, groups);
  else if (variant == 6)
    hipLaunchKernelGGL(stem_hpool_f32_kernel<true>, dim3(groups * B), dim3(SF_NT), 0, s, x, w, bias, out, H, W, OH,
                       pad_t, pad_l, PH, groups);
  else
    hipLaunchKernelGGL(stem_hpool_f32_kernel<false>, dim3(groups * B), dim3(SF_NT), 0, s, x, w, bias, out, H, W, OH,
                       pad_t, pad_l, PH, groups);
  return hipGetLastError();
}

}  // namespace adapt
