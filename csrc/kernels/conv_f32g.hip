// fp32 implicit-GEMM convolution, v2: LDS-DMA (global_load_lds) multi-stage
// ring on the fp32 matrix cores (v_mfma_f32_16x16x4_f32).  The reference's
// precision: Keras runs the model in float32 (`src/node.py:177`,
// `test/local_infer.py:22`).
//
//   out[m][n] = act( sum_k X[m][k] * W[n][k] + bias[n] (+ res[m][n]) )
//
// Why a second fp32 kernel: the v1 kernel (conv_f32.hip) stages its tiles
// through registers with a double buffer and 4 waves per block; rocprofv3 put
// its waves in waits 55-64 % of their cycles with the matrix pipe busy 38-50 %
// (profiles/r2/fp32/pmc_fp32_conv_kernels.txt).  The fp32 MFMA runs at 1/16 of
// the bf16 rate, so every ResNet conv is compute-bound at the matrix pipe and
// the only job of the memory side is to never make it wait:
//
// * K tiles of 32 floats = 128-byte LDS rows, the same geometry as the bf16
//   ring (conv_glds.hip: 64 bf16 per row), so the same XOR chunk swizzle makes
//   the 16-row fragment reads conflict-free and one 1 KiB LDS-DMA piece is
//   8 rows x 128 B;
// * STAGES-deep ring, STAGES-1 tiles in flight (counted vmcnt, one barrier per
//   tile); a 128x128 tile's K step is 4096 MFMA cycles per wave, so three tiles
//   in flight cover any HBM / Infinity-Cache latency;
// * the k permutation of v1: lane group q supplies k = 16h + 4q + s to MFMA step
//   s of half h for both operands, so every fragment is one ds_read_b128;
// * tap-major K walk: Cin % 32 == 0, so a K tile never straddles a filter tap
//   and each row's source pointer moves by a wave-uniform tap offset;
// * KG = 2: two K-groups of waves, group g runs half g of every K tile; the
//   block has twice the waves (two per SIMD) at the same per-wave sub-tile, and
//   the partial sums meet in the fp32 epilogue tile;
// * fused epilogue from an LDS fp32 tile: 16-byte row segments, bias,
//   residual (prefetched before the K loop when it fits the registers), ReLU.
#include "kernels.h"

#include <type_traits>

namespace adapt {

typedef __attribute__((address_space(3))) void lds_void_f32;
void conv_f32g_sk_plan(int tiles, int kt, int mult, int* grid, int* iters);

namespace {
constexpr int GBK = 32;          // floats per K tile (one 128-byte LDS row)

__device__ __forceinline__ int fswz2(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }

template <int N> __device__ __forceinline__ void fwait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int BM, int BN, int STAGES>
struct F32gShape {
  static constexpr int STAGE_BYTES = (BM + BN) * 128;
  static constexpr int EPI_LD = BN + 4;
  static constexpr int EPI_BYTES = BM * EPI_LD * 4;
  static constexpr int LDS_BYTES = (STAGES * STAGE_BYTES > EPI_BYTES) ? STAGES * STAGE_BYTES : EPI_BYTES;
};

// stream-K bookkeeping of one (tile, K-range) segment; slot < 0: whole K range
struct F32Seg {
  int slot;      // this segment's fp32 partial slot in p.ws
  int nseg;      // segments covering the tile
  int seg;       // this segment's index among them (summation order)
  int g_first;   // first block covering the tile
};

__device__ __forceinline__ int f32_sk_slot(int g, int tile, int kt, int iters) {
  // a block's first segment uses slot 2g, its last (when it started in an earlier tile) 2g+1
  return 2 * g + ((long long)g * iters >= (long long)tile * kt ? 0 : 1);
}

constexpr int F32_CPOL_SC1 = 16;   // gfx950 cache policy: sc1 (write-through L2, bypass L1)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t f32_ws_rsrc(const float* base) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, 0x7fffffff, 0x00020000);
}

template <int BM, int BN, int WM, int WN, int STAGES, bool PURE, int KG, bool PIPE>
__device__ __forceinline__ void f32g_tile(const ConvF32Params& p, const float* __restrict__ zero, char* smem,
                                          int tile, int kt0, int kt1, int split_idx, const F32Seg& sk) {
  using S = F32gShape<BM, BN, STAGES>;
  constexpr int NW = WM * WN;                 // compute waves per K-group
  constexpr int NWA = NW * KG;                // all waves (every wave issues pieces)
  constexpr int NT = NWA * 64;
  constexpr int NH = 2 / KG;                  // 16-wide K halves per wave per K tile
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16;
  constexpr int A_INS = BM / (8 * NWA), B_INS = BN / (8 * NWA);
  constexpr int LPW = A_INS + B_INS;
  constexpr int TILE_A = BM * 128, STAGE_BYTES = S::STAGE_BYTES, EPI_LD = S::EPI_LD;
  static_assert(A_INS * 8 * NWA == BM && B_INS * 8 * NWA == BN, "waves / tile split");
  static_assert(STAGES >= 2 && S::LDS_BYTES <= 160 * 1024, "stages");
  static_assert((STAGES - (PIPE ? 1 : 2)) * LPW <= 63, "vmcnt range");

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kg = KG > 1 ? wave / NW : 0;
  const int wsub = wave % NW;
  const int wm = wsub / WN, wn = wsub % WN;

  const int tilesN = (p.N + BN - 1) / BN;
  const int m0 = (tile / tilesN) * BM, n0 = (tile % tilesN) * BN;
  const int nk = kt1 > kt0 ? kt1 - kt0 : 0;

  // ---- per-lane source bookkeeping (rows fixed over the K loop)
  const int lrow = lane >> 3, pchunk = lane & 7;
  const float* a_ptr[A_INS];
  int a_ih0[A_INS], a_iw0[A_INS];
  const int ohw = p.OH * p.OW;
#pragma unroll
  for (int i = 0; i < A_INS; ++i) {
    const int r = (wave * A_INS + i) * 8 + lrow;
    const int m = m0 + r;
    const int c = pchunk ^ ((r >> 1) & 7);            // logical 4-float chunk this lane fetches
    a_ih0[i] = a_iw0[i] = 0;
    a_ptr[i] = nullptr;
    if (m < p.M) {
      if (PURE) {
        a_ptr[i] = p.x + (size_t)m * p.Cin + c * 4;
      } else {
        const int img = m / ohw, rr = m - img * ohw, oh = rr / p.OW, ow = rr - oh * p.OW;
        a_ih0[i] = oh * p.stride - p.pad_t;
        a_iw0[i] = ow * p.stride - p.pad_l;
        a_ptr[i] = p.x + ((size_t)img * p.H * p.W + (ptrdiff_t)a_ih0[i] * p.W + a_iw0[i]) * p.Cin + c * 4;
      }
    }
  }
  const float* b_src[B_INS];
#pragma unroll
  for (int i = 0; i < B_INS; ++i) {
    const int r = (wave * B_INS + i) * 8 + lrow;
    b_src[i] = p.w + (size_t)(n0 + r) * p.Kpad + (pchunk ^ ((r >> 1) & 7)) * 4;
  }
  const int cpt = p.Cin / GBK;                // 32-channel slices per tap
  int ck = kt0;
  int c_kh = 0, c_kw = 0, c_cc = 0;
  if (!PURE) {
    const int tap = ck / cpt;
    c_cc = ck - tap * cpt;
    c_kh = tap / p.KW;
    c_kw = tap - c_kh * p.KW;
  }
  unsigned a_ok = 0;
  ptrdiff_t tap_off = 0;
  auto tap_update = [&]() {
    tap_off = ((ptrdiff_t)c_kh * p.W + c_kw) * p.Cin;
    a_ok = 0;
#pragma unroll
    for (int i = 0; i < A_INS; ++i) {
      const int ih = a_ih0[i] + c_kh, iw = a_iw0[i] + c_kw;
      if (a_ptr[i] != nullptr && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W) a_ok |= 1u << i;
    }
  };
  if (!PURE) tap_update();

  // branch-free issue of the next K tile into ring slot `slot`; tiles past the
  // block's K range fetch the zero page so the wait count stays a constant
  auto issue = [&](int slot) {
    char* sa = smem + slot * STAGE_BYTES;
    char* sb = sa + TILE_A;
    const bool live = ck < kt1;
#pragma unroll
    for (int i = 0; i < A_INS; ++i) {
      const float* src;
      if (PURE) src = (live && a_ptr[i] != nullptr) ? a_ptr[i] + (size_t)ck * GBK : zero;
      else src = (live && ((a_ok >> i) & 1u)) ? a_ptr[i] + tap_off + c_cc * GBK : zero;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void_f32*)(sa + (wave * A_INS + i) * 1024), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < B_INS; ++i) {
      const float* src = live ? b_src[i] + (size_t)ck * GBK : zero;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void_f32*)(sb + (wave * B_INS + i) * 1024), 16, 0, 0);
    }
    ++ck;
    if (!PURE) {
      const bool roll_c = ++c_cc == cpt;
      const bool roll_w = roll_c && c_kw + 1 == p.KW;
      c_cc = roll_c ? 0 : c_cc;
      c_kw = roll_w ? 0 : (roll_c ? c_kw + 1 : c_kw);
      c_kh += roll_w ? 1 : 0;
      tap_update();
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fq = lane >> 4;

  // residual chunks of this thread's epilogue rows, requested before the K loop
  // (older than every LDS-DMA piece, so the counted vmcnt waits stay valid)
  constexpr int CPR = BN / 4;                 // 4-float chunks per output row
  constexpr int NCH = BM * CPR;
  constexpr int RPI = NT / CPR;               // rows per epilogue iteration
  constexpr int IT = (NCH + NT - 1) / NT;
  static_assert(NT % CPR == 0, "column chunk must be iteration-invariant");
  constexpr bool PRE = IT <= 8;
  const int ecc = tid % CPR, erow0 = tid / CPR;
  const int en = n0 + ecc * 4;
  const bool use_pre = PRE && p.res != nullptr && p.ksplit == 1 && sk.slot < 0;
  f32x4 rpre[PRE ? IT : 1];
  if (use_pre) {
#pragma unroll
    for (int u = 0; u < (PRE ? IT : 1); ++u) {
      const int row = erow0 + u * RPI, m = m0 + row;
      rpre[u] = (f32x4){0.f, 0.f, 0.f, 0.f};
      if (en < p.N && row < BM && m < p.M) rpre[u] = *(const f32x4*)(p.res + (size_t)m * p.N + en);
    }
  }

  constexpr int MT = NH * 4 * FM * FN;         // MFMAs per wave per K tile
  auto read_frags = [&](int slot, f32x4 (&af)[NH][FM], f32x4 (&bfr)[NH][FN]) {
    const char* sa = smem + slot * STAGE_BYTES;
    const char* sb = sa + TILE_A;
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      const int kq = (h + kg) * 4 + fq;       // this lane's 16-byte chunk of half h + kg
#pragma unroll
      for (int i = 0; i < FM; ++i) af[h][i] = *(const f32x4*)(sa + fswz2(wm * TM + i * 16 + fr, kq));
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[h][j] = *(const f32x4*)(sb + fswz2(wn * TN + j * 16 + fr, kq));
    }
  };
  // MFMA steps [S0, S1) of the NH * 4 (half, k) steps of one K tile
  auto mfma_steps = [&](const f32x4 (&af)[NH][FM], const f32x4 (&bfr)[NH][FN], auto s0c, auto s1c) {
    constexpr int S0 = decltype(s0c)::value, S1 = decltype(s1c)::value;
#pragma unroll
    for (int st = S0; st < S1; ++st)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[st / 4][i][st % 4], bfr[st / 4][j][st % 4], acc[i][j],
                                                           0, 0, 0);
  };

  if constexpr (!PIPE) {
#pragma unroll
    for (int s = 0; s < STAGES - 1; ++s) issue(s);

    for (int t = 0; t < nk; ++t) {
      fwait_vm<(STAGES - 2) * LPW>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      const int nslot = (t + STAGES - 1) % STAGES;
      f32x4 af[NH][FM], bfr[NH][FN];
      read_frags(t % STAGES, af, bfr);
      issue(nslot);
      mfma_steps(af, bfr, std::integral_constant<int, 0>{}, std::integral_constant<int, NH * 4>{});
      // LDS-DMA pieces of tile t+STAGES-1 spread between this tile's MFMAs
      constexpr int MPP = MT / LPW > 0 ? MT / LPW : 1;
      __builtin_amdgcn_sched_group_barrier(0x100, NH * (FM + FN), 0);   // ds_read
#pragma unroll
      for (int q = 0; q < LPW; ++q) {
        __builtin_amdgcn_sched_group_barrier(0x008, MPP, 0);            // MFMA
        __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);              // VMEM (LDS-DMA piece)
      }
      __builtin_amdgcn_sched_group_barrier(0x008, MT, 0);
    }
  } else {
    // Software-pipelined: the fragments of tile t+1 are read from LDS (and tile
    // t+STAGES is put in flight) between the two halves of tile t's MFMAs, so
    // the matrix pipe never waits out a barrier + ds_read round trip.  Slot
    // t % STAGES is refilled right after the mid-tile barrier of tile t: every
    // wave has its tile-t fragments in registers by then (lgkmcnt(0)).
#pragma unroll
    for (int s = 0; s < STAGES; ++s) issue(s);
    fwait_vm<(STAGES - 1) * LPW>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    f32x4 fa0[NH][FM], fb0[NH][FN], fa1[NH][FM], fb1[NH][FN];
    read_frags(0, fa0, fb0);
    constexpr int HALF = NH * 2;
    constexpr int MH = MT / 2;
    constexpr int MPP = MH / LPW > 0 ? MH / LPW : 1;
    auto step = [&](int t, const f32x4 (&ca)[NH][FM], const f32x4 (&cb)[NH][FN], f32x4 (&na)[NH][FM],
                    f32x4 (&nb)[NH][FN]) {
      mfma_steps(ca, cb, std::integral_constant<int, 0>{}, std::integral_constant<int, HALF>{});
      fwait_vm<(STAGES - 2) * LPW>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      read_frags((t + 1) % STAGES, na, nb);
      issue(t % STAGES);
      mfma_steps(ca, cb, std::integral_constant<int, HALF>{}, std::integral_constant<int, NH * 4>{});
      __builtin_amdgcn_sched_group_barrier(0x100, NH * (FM + FN), 0);   // ds_read (next tile)
#pragma unroll
      for (int q = 0; q < LPW; ++q) {
        __builtin_amdgcn_sched_group_barrier(0x008, MPP, 0);            // MFMA
        __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);              // VMEM (LDS-DMA piece)
      }
      __builtin_amdgcn_sched_group_barrier(0x008, MH, 0);
    };
    for (int t = 0; t < nk; t += 2) {
      step(t, fa0, fb0, fa1, fb1);
      if (t + 1 < nk) step(t + 1, fa1, fb1, fa0, fb0);
    }
  }
  fwait_vm<0>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  // ---- epilogue: acc[i][j][r] = C[row = wm*TM + i*16 + fq*4 + r][col = wn*TN + j*16 + fr]
  float* epi = (float*)smem;
  if (kg == 0) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int col = wn * TN + j * 16 + fr;
#pragma unroll
        for (int r = 0; r < 4; ++r) epi[(wm * TM + i * 16 + fq * 4 + r) * EPI_LD + col] = acc[i][j][r];
      }
  }
  __syncthreads();
  if constexpr (KG > 1) {
    if (kg == 1) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int col = wn * TN + j * 16 + fr;
#pragma unroll
          for (int r = 0; r < 4; ++r) epi[(wm * TM + i * 16 + fq * 4 + r) * EPI_LD + col] += acc[i][j][r];
        }
    }
    __syncthreads();
  }
  if (sk.slot >= 0) {
    // stream-K partial tile: publish it with 16-B sc1 stores, one lane counts the
    // arrival; the tile's last segment adds every partial in segment order
    // (deterministic) and runs the epilogue.  Nobody waits on anybody, so the
    // grid never needs to be co-resident (MI355X_MICROARCH.md inter-workgroup
    // visibility: sc1 stores drained, barrier, counter; sc1 loads on the reader).
    const __amdgpu_buffer_rsrc_t wsr = f32_ws_rsrc(p.ws);
    const int base = sk.slot * BM * BN;
#pragma unroll
    for (int u = 0; u < IT; ++u) {
      const int row = erow0 + u * RPI;
      if (row >= BM) continue;
      const u32x4 v = __builtin_bit_cast(u32x4, *(const f32x4*)(epi + row * EPI_LD + ecc * 4));
      __builtin_amdgcn_raw_buffer_store_b128(v, wsr, (base + row * BN + ecc * 4) * 4, 0, F32_CPOL_SC1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = (int*)(smem + S::LDS_BYTES);       // the 16 bytes past the ring / epilogue tile
    if (tid == 0) {
      const int old = __hip_atomic_fetch_add(p.counters + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = old == sk.nseg - 1;
      if (last) __hip_atomic_store(p.counters + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = last;
    }
    __syncthreads();
    if (!*flag) return;
    const int ktt = p.Kpad / GBK;
#pragma unroll
    for (int u = 0; u < IT; ++u) {
      const int row = erow0 + u * RPI;
      if (row >= BM) continue;
      f32x4 acc4 = (f32x4){0.f, 0.f, 0.f, 0.f};
      for (int sg = 0; sg < sk.nseg; ++sg) {
        if (sg == sk.seg) {
          acc4 += *(const f32x4*)(epi + row * EPI_LD + ecc * 4);
        } else {
          const int off = (f32_sk_slot(sk.g_first + sg, tile, ktt, p.sk_iters) * BM * BN + row * BN + ecc * 4) * 4;
          acc4 += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(wsr, off, 0, F32_CPOL_SC1));
        }
      }
      *(f32x4*)(epi + row * EPI_LD + ecc * 4) = acc4;           // each thread re-reads only its own chunks
    }
  }
  if (en >= p.N) return;
  if (p.ksplit > 1) {
    float* slab = p.ws + (size_t)split_idx * p.M * p.N;
#pragma unroll
    for (int u = 0; u < IT; ++u) {
      const int row = erow0 + u * RPI, m = m0 + row;
      if (row < BM && m < p.M) *(f32x4*)(slab + (size_t)m * p.N + en) = *(const f32x4*)(epi + row * EPI_LD + ecc * 4);
    }
    return;
  }
  const f32x4 b = p.bias ? *(const f32x4*)(p.bias + en) : (f32x4){0.f, 0.f, 0.f, 0.f};
  constexpr int EG = IT < 4 ? IT : 4;
#pragma unroll
  for (int g = 0; g < IT; g += EG) {
    f32x4 r[EG];
#pragma unroll
    for (int u = 0; u < EG; ++u) {
      const int row = erow0 + (g + u) * RPI, m = m0 + row;
      r[u] = (f32x4){0.f, 0.f, 0.f, 0.f};
      if (use_pre) {
        if (g + u < IT) r[u] = rpre[PRE ? g + u : 0];
      } else if (p.res && g + u < IT && row < BM && m < p.M) {
        r[u] = *(const f32x4*)(p.res + (size_t)m * p.N + en);
      }
    }
#pragma unroll
    for (int u = 0; u < EG; ++u) {
      const int row = erow0 + (g + u) * RPI, m = m0 + row;
      if (g + u >= IT || row >= BM || m >= p.M) continue;
      f32x4 v = *(const f32x4*)(epi + row * EPI_LD + ecc * 4) + b + r[u];
      const F32Dst d = f32_dst(p, en);
      v[0] = act_relu(v[0], d.relu); v[1] = act_relu(v[1], d.relu);
      v[2] = act_relu(v[2], d.relu); v[3] = act_relu(v[3], d.relu);
      *(f32x4*)(d.base + (size_t)m * d.ld + d.col) = v;
    }
  }
}

// One launch = (a) data-parallel tiles x split-K slices (p.ksplit >= 1), or (b)
// stream-K (p.ksplit < 0): the tiles x K-tiles iteration space is cut into equal
// contiguous ranges of p.sk_iters, one per block (256 x -ksplit blocks), so a
// ~200-tile layer keeps every CU busy instead of leaving a quarter of the chip
// idle: at 1/16 of the bf16 rate every fp32 conv is matrix-bound, and the
// partial-tile traffic is small beside its MFMA time.
template <int BM, int BN, int WM, int WN, int STAGES, bool PURE, int KG, bool PIPE>
__global__ __launch_bounds__(WM * WN * KG * 64, 1) void conv_f32g_kernel(ConvF32Params p,
                                                                         const float* __restrict__ zero) {
  using S = F32gShape<BM, BN, STAGES>;
  __shared__ __attribute__((aligned(16))) char smem[S::LDS_BYTES + 16];
  const int tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  const int kt = p.Kpad / GBK;
  if (p.ksplit >= 1) {
    const int tile = xcd_remap(blockIdx.x, tiles);
    const int kper = (kt + p.ksplit - 1) / p.ksplit;
    const int kt0 = blockIdx.y * kper, kt1 = min(kt, kt0 + kper);
    f32g_tile<BM, BN, WM, WN, STAGES, PURE, KG, PIPE>(p, zero, smem, tile, kt0, kt1, blockIdx.y, F32Seg{-1, 1, 0, 0});
    return;
  }
  const int g = blockIdx.x, iters = p.sk_iters;
  const int total = tiles * kt;
  int it = g * iters;
  const int it_end = min(total, it + iters);
  while (it < it_end) {
    const int tile = it / kt;
    const int kbeg = it - tile * kt;
    const int kend = min(kt, kbeg + (it_end - it));
    F32Seg sk{-1, 1, 0, 0};
    if (kbeg != 0 || kend != kt) {
      const int g_first = (tile * kt) / iters, g_last = ((tile + 1) * kt - 1) / iters;
      sk = F32Seg{f32_sk_slot(g, tile, kt, iters), g_last - g_first + 1, g - g_first, g_first};
    }
    f32g_tile<BM, BN, WM, WN, STAGES, PURE, KG, PIPE>(p, zero, smem, tile, kbeg, kend, 0, sk);
    it += kend - kbeg;
    __syncthreads();   // the next segment's DMA reuses the epilogue's LDS
  }
}

// 16-byte aligned zero page that out-of-range lanes fetch from
__device__ __attribute__((aligned(64))) float g_zero_page_f32[64];

template <int BM, int BN, int WM, int WN, int STAGES, int KG, bool PIPE>
hipError_t launch_f32g(const ConvF32Params& p, bool pure, hipStream_t s) {
  static float* zero = nullptr;
  if (!zero) {
    hipError_t e = hipGetSymbolAddress((void**)&zero, HIP_SYMBOL(g_zero_page_f32));
    if (e != hipSuccess) return e;
  }
  const int tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  dim3 grid(tiles, p.ksplit), block(WM * WN * KG * 64);
  if (p.ksplit < 0) {
    int g, iters;
    conv_f32g_sk_plan(tiles, p.Kpad / GBK, -p.ksplit, &g, &iters);
    if (!p.counters || !p.ws || iters != p.sk_iters) return hipErrorInvalidValue;
    grid = dim3(g, 1);
  }
  if (pure) hipLaunchKernelGGL((conv_f32g_kernel<BM, BN, WM, WN, STAGES, true, KG, PIPE>), grid, block, 0, s, p, zero);
  else hipLaunchKernelGGL((conv_f32g_kernel<BM, BN, WM, WN, STAGES, false, KG, PIPE>), grid, block, 0, s, p, zero);
  return hipGetLastError();
}

}  // namespace

// stream-K grid of the v2 fp32 kernels: `mult` x 256 blocks, each taking ceil(total / G)
// consecutive (tile, K-tile) iterations
void conv_f32g_sk_plan(int tiles, int kt, int mult, int* grid, int* iters) {
  const long long total = (long long)tiles * kt;
  long long G = 256LL * (mult > 0 ? mult : 1);
  if (G > total) G = total;
  const long long it = (total + G - 1) / G;
  *iters = (int)it;
  *grid = (int)((total + it - 1) / it);
}

// v2 fp32 tile configs: id -> BM, BN, WM, WN, STAGES, KG, PIPE (ops/conv.py F32_TILES mirrors the
// tile sizes); 30-41 are the software-pipelined twins of 10-21 (no 35 / 36: their two fragment sets
// spill at 256 x 128 / 128 x 256)
#define ADAPT_F32G_CFGS(X)            \
  X(10, 128, 128, 2, 2, 4, 1, false)  \
  X(11, 128, 128, 2, 2, 3, 2, false)  \
  X(12, 128, 64, 2, 2, 4, 1, false)   \
  X(13, 64, 128, 2, 2, 4, 1, false)   \
  X(14, 64, 64, 2, 2, 4, 1, false)    \
  X(15, 256, 128, 4, 2, 3, 1, false)  \
  X(16, 128, 256, 2, 4, 3, 1, false)  \
  X(17, 128, 128, 4, 2, 4, 1, false)  \
  X(18, 64, 64, 2, 2, 4, 2, false)    \
  X(19, 128, 64, 2, 2, 4, 2, false)   \
  X(20, 64, 128, 2, 2, 4, 2, false)   \
  X(21, 256, 64, 4, 2, 3, 1, false)   \
  X(30, 128, 128, 2, 2, 4, 1, true)   \
  X(31, 128, 128, 2, 2, 3, 2, true)   \
  X(32, 128, 64, 2, 2, 4, 1, true)    \
  X(33, 64, 128, 2, 2, 4, 1, true)    \
  X(34, 64, 64, 2, 2, 4, 1, true)     \
  X(37, 128, 128, 4, 2, 4, 1, true)   \
  X(38, 64, 64, 2, 2, 4, 2, true)     \
  X(39, 128, 64, 2, 2, 4, 2, true)    \
  X(40, 64, 128, 2, 2, 4, 2, true)    \
  X(41, 256, 64, 4, 2, 3, 1, true)

// cfg in the v2 family and the problem on its path (tap-major walk: Cin % 32 == 0; 16-byte output
// chunks: N % 4 == 0)
bool conv_f32g_ok(int cfg, int Cin, int N) {
  if (Cin % GBK || N % 4) return false;
  switch (cfg) {
#define X(id, BM_, BN_, WM_, WN_, S_, KG_, P_) case id: return true;
    ADAPT_F32G_CFGS(X)
#undef X
  }
  return false;
}

bool conv_f32g_cfg_tile(int cfg, int* bm, int* bn) {
  switch (cfg) {
#define X(id, BM_, BN_, WM_, WN_, S_, KG_, P_) case id: *bm = BM_; *bn = BN_; return true;
    ADAPT_F32G_CFGS(X)
#undef X
  }
  return false;
}

hipError_t conv_f32g_launch(const ConvF32Params& p, int cfg, bool pure, hipStream_t s) {
  switch (cfg) {
#define X(id, BM_, BN_, WM_, WN_, S_, KG_, P_) case id: return launch_f32g<BM_, BN_, WM_, WN_, S_, KG_, P_>(p, pure, s);
    ADAPT_F32G_CFGS(X)
#undef X
  }
  return hipErrorInvalidValue;
}

}  // namespace adapt
