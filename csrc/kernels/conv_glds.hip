// Implicit-GEMM convolution, v2: LDS-DMA (global_load_lds) multi-stage ring.
//
// Same contract as conv_igemm.hip (out = act(X*W^T + bias (+res)), BN folded
// on the host) but the A/B tiles move HBM -> LDS with
// `__builtin_amdgcn_global_load_lds` (16 B per lane, no VGPR round trip):
//
// * STAGES-deep ring of [BM|BN][64] bf16 tiles; STAGES-1 tiles stay in flight
//   across the K loop (counted `s_waitcnt vmcnt(N)`, raw `s_barrier`, never a
//   vmcnt(0) drain inside the loop: cdna_hip_programming.md §5 "Pipelining
//   across barriers").
// * The LDS image is lane-linear per wave instruction (1 KiB = 8 rows x 128 B);
//   the XOR chunk swizzle that makes the MFMA fragment reads conflict-free is
//   applied to the per-lane GLOBAL source address and again on the ds_read
//   (rule 21: linear dest + inverse-swizzled source + swizzled read).
// * Implicit im2col: each lane's source address is a (pixel, tap, channel)
//   gather; padding pixels, k >= K and m >= M read a 16-byte zero page, so the
//   DMA never needs a mask.
// * Fused epilogue identical to v1 (LDS fp32 tile -> 16-byte row segments).
#include "kernels.h"
#include "epilogue.h"

namespace adapt {

typedef __attribute__((address_space(3))) void lds_void;

namespace {
constexpr int BK2 = 64;

__device__ __forceinline__ int swz2(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }

template <int N> __device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// wait until at most min(ahead, K) tiles (LPW glds each) are still in flight
template <int LPW, int K> __device__ __forceinline__ void wait_tiles(int ahead) {
  if constexpr (K == 0) {
    wait_vm<0>();
  } else {
    if (ahead >= K) wait_vm<K * LPW>();
    else wait_tiles<LPW, K - 1>(ahead);
  }
}
}  // namespace

// Stream-K bookkeeping of one (tile, K-range) segment.  slot < 0: the segment
// covers the whole K range (normal epilogue).
struct SkSeg {
  int slot;      // this segment's fp32 partial slot in p.ws
  int nseg;      // segments (= consecutive blocks) covering the tile
  int seg;       // this segment's index among them (summation order)
  int g_first;   // first block covering the tile
};

__device__ __forceinline__ int sk_slot(int g, int tile, int kt, int iters) {
  // a block's first segment uses slot 2g, its last (when it started in an earlier tile) 2g+1
  return 2 * g + ((long long)g * iters >= (long long)tile * kt ? 0 : 1);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t ws_rsrc(const float* base) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, 0x7fffffff, 0x00020000);
}
constexpr int CPOL_SC1 = 16;   // gfx950 cache policy: sc1 (bypass L1, write-through L2)

template <int BM, int BN, int WM, int WN, int STAGES>
struct GldsShape {
  static constexpr int NW = WM * WN, NT = NW * 64;
  static constexpr int STAGE_BYTES = (BM + BN) * 128;
  static constexpr int EPI_BYTES = BM * (BN + 4) * 4;
  static constexpr int LDS_BYTES = (STAGES * STAGE_BYTES > EPI_BYTES) ? STAGES * STAGE_BYTES : EPI_BYTES;
};

// ABL: ablation switches for tools/conv_ablate.hip (0 in every production
// instance): 1 = no MFMA, 2 = no LDS-DMA, 4 = every K tile re-fetches the
// block's first one (L2-hot operands), 8 = no fragment ds_reads, 16 = no K
// loop at all (launch + prologue + epilogue only).
//
// NL > 0: NL dedicated loader waves beside the WM x WN compute waves.  The
// ablation (tools/conv_ablate.hip, profiles/r2/conv_ablate.txt) showed the
// LDS-DMA feed and the MFMA work of one K tile SERIALISE when the compute
// waves issue the pieces themselves (a piece's issue stalls its wave while the
// CU's address path is busy, and the MFMAs behind it in program order wait):
// base ~= DMA-only + compute-only.  Loader waves only issue pieces and wait for
// them (counted vmcnt, then the shared barrier); compute waves only ds_read and
// MFMA, so the two overlap.
//
// KG = 2: two K-groups of WM x WN compute waves per block.  Each 64-wide K tile
// is two 32-wide MFMA K steps; group g runs step g only, so a wave covers a
// (BM/WM) x (BN/WN) sub-tile twice as large as the KG = 1 block of the same
// wave count and reads a quarter to a third fewer LDS fragment bytes per MFMA
// (the ablation's no-DMA/skeleton rows: the fragment ds_reads are ~6 us of a
// stage-4 3x3).  The two partial accumulators meet in the fp32 epilogue tile.
template <int BM, int BN, int WM, int WN, int STAGES, bool ILV, bool PURE, bool OUT_F32, int ABL = 0, int NL = 0,
          int KG = 1>
__device__ __forceinline__ void glds_tile(const ConvParams& p, const bf16* __restrict__ zero, char* smem,
                                          int tile, int kt0, int kt1, int split_idx, const SkSeg& sk) {
  using S = GldsShape<BM, BN, WM, WN, STAGES>;
  constexpr int NW = S::NW;                  // compute waves per K-group
  constexpr int NWC = NW * KG;               // compute waves
  constexpr int NT = (NWC + NL) * 64;        // all threads of the block
  constexpr int NWI = NL > 0 ? NL : NWC;     // waves that issue the LDS-DMA pieces
  constexpr int NKS = 2 / KG;                // 32-wide MFMA K steps per wave per K tile
  static_assert(KG == 1 || (KG == 2 && NL == 0), "K-groups");
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16;
  constexpr int A_INS = BM / (8 * NWI), B_INS = BN / (8 * NWI);   // glds instructions per issuing wave per tile
  constexpr int LPW = A_INS + B_INS;
  constexpr int TILE_A = BM * 128, STAGE_BYTES = S::STAGE_BYTES;
  constexpr int EPI_LD = BN + 4;
  static_assert((NWC == 4 || NWC == 8 || NWC == 16) && A_INS * 8 * NWI == BM && B_INS * 8 * NWI == BN,
                "waves / tile split");
  static_assert(STAGES >= 2 && S::LDS_BYTES + 16 <= 160 * 1024, "stages");
  static_assert((STAGES - 2) * LPW <= 63, "vmcnt range");

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool loader = NL > 0 && wave >= NW;  // wave-uniform
  const int iwave = NL > 0 ? (loader ? wave - NW : 0) : wave;   // index among the issuing waves
  const int kg = KG > 1 ? wave / NW : 0;     // K-group: first 32-wide MFMA K step it runs
  const int wsub = (loader ? 0 : wave) % NW;
  const int wm = wsub / WN, wn = wsub % WN;

  const int tilesN = (p.N + BN - 1) / BN;
  const int tm = tile / tilesN, tn = tile % tilesN;
  const int m0 = tm * BM, n0 = tn * BN;
  const int nk = (ABL & 16) ? 0 : (kt1 > kt0 ? kt1 - kt0 : 0);

  // ---- per-lane source bookkeeping (rows fixed over the K loop)
  //
  // Tap-major K walk: when Cin % 64 == 0 (every ResNet conv except the stem) a
  // 64-wide K tile never straddles a filter tap, so the loop visits taps
  // (kh, kw) in order and the 64-channel slices of each tap.  Each lane keeps
  // one 64-bit source pointer per A row for the *centre* pixel; a tap moves it
  // by a wave-uniform (kh*W + kw)*Cin element offset and the per-row bounds
  // test runs once per tap, so the steady-state cost per glds is a pointer add
  // and a select (the per-tile integer division of v1 is gone).
  const int lrow = lane >> 3;      // row within the 8-row piece
  const int pchunk = lane & 7;     // physical LDS chunk this lane writes
  const bf16* a_ptr[A_INS];        // element (pixel row0 tap origin, channel chunk) or null
  int a_ih0[A_INS], a_iw0[A_INS];
  const int ohw = p.OH * p.OW;
#pragma unroll
  for (int i = 0; i < A_INS; ++i) {
    const int r = (iwave * A_INS + i) * 8 + lrow;       // tile row
    const int m = m0 + r;
    const int c = pchunk ^ ((r >> 1) & 7);              // logical chunk this lane fetches
    a_ih0[i] = a_iw0[i] = 0;
    a_ptr[i] = nullptr;
    if (m < p.M) {
      if (PURE) {
        a_ptr[i] = p.x + (size_t)m * p.Cin + c * 8;
      } else {
        const int img = m / ohw;
        const int rr = m - img * ohw;
        const int oh = rr / p.OW;
        const int ow = rr - oh * p.OW;
        a_ih0[i] = oh * p.stride - p.pad_t;
        a_iw0[i] = ow * p.stride - p.pad_l;
        // origin of the receptive field (may point outside the image; only
        // dereferenced after the per-tap bounds test)
        a_ptr[i] = p.x + ((size_t)img * p.H * p.W + (ptrdiff_t)a_ih0[i] * p.W + a_iw0[i]) * p.Cin + c * 8;
      }
    }
  }
  const bf16* b_src[B_INS];
#pragma unroll
  for (int i = 0; i < B_INS; ++i) {
    const int r = (iwave * B_INS + i) * 8 + lrow;
    b_src[i] = p.w + (size_t)(n0 + r) * p.Kpad + (pchunk ^ ((r >> 1) & 7)) * 8;
  }
  // issue cursor (wave-uniform): tap (kh, kw) and channel slice cc of the next tile to fetch
  const int cpt = p.Cin >> 6;          // 64-channel slices per tap (>= 1 on this path)
  int ck = kt0;                        // next K tile to issue
  int c_kh = 0, c_kw = 0, c_cc = 0;
  if (!PURE) {
    const int tap = ck / cpt;
    c_cc = ck - tap * cpt;
    c_kh = tap / p.KW;
    c_kw = tap - c_kh * p.KW;
  }
  unsigned a_ok = 0;                   // per-row validity bits for the current tap
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

  // Branch-free issue of the next K tile into ring slot `slot` (one basic
  // block, so the interleaved schedule below can place its pieces between
  // MFMAs).  Tiles past this block's K range fetch the zero page: the ring
  // is always STAGES-1 tiles ahead and the wait count is a constant.
  auto issue = [&](int slot) {
    char* sa = smem + slot * STAGE_BYTES;
    char* sb = sa + TILE_A;
    const int kt = (ABL & 4) ? kt0 : ck;
    const bool live = ck < kt1;
#pragma unroll
    for (int i = 0; i < ((ABL & 2) ? 0 : A_INS); ++i) {
      const bf16* src;
      if (PURE) src = (live && a_ptr[i] != nullptr) ? a_ptr[i] + (size_t)kt * BK2 : zero;
      else src = (live && ((a_ok >> i) & 1u)) ? a_ptr[i] + tap_off + c_cc * BK2 : zero;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(sa + (iwave * A_INS + i) * 1024), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < ((ABL & 2) ? 0 : B_INS); ++i) {
      const bf16* src = live ? b_src[i] + (size_t)kt * BK2 : zero;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(sb + (iwave * B_INS + i) * 1024), 16, 0, 0);
    }
    ++ck;
    if (!PURE && !(ABL & 4)) {
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
  // data-parallel tile with a residual: its loads go out before the K loop
  // (older than every LDS-DMA piece, so the counted vmcnt waits stay valid)
  EpiRes<BM, BN, NT> rpre;
  const bool use_pre = sk.slot < 0 && p.ksplit == 1 && p.res != nullptr;
  if (use_pre) rpre.prefetch(p, m0, n0, tid, p.M);
  if (NL == 0 || loader) {
#pragma unroll
    for (int s = 0; s < STAGES - 1; ++s) issue(s);
  }

  constexpr int MT = NKS * FM * FN;        // MFMAs per wave per K tile
  for (int t = 0; t < nk; ++t) {
    // tile t must have landed (the issuing waves' counted wait + the barrier
    // orders it for every reader); the STAGES-2 tiles issued after it stay in flight
    if (NL == 0 || loader) wait_vm<(STAGES - 2) * LPW>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int nslot = (t + STAGES - 1) % STAGES;
    if constexpr (NL > 0) {
      if (loader) {
        issue(nslot);
        continue;
      }
    } else if constexpr (!ILV) {
      issue(nslot);
    }
    const char* sa = smem + (t % STAGES) * STAGE_BYTES;
    const char* sb = sa + TILE_A;
    bf16x8 af[NKS][FM], bfr[NKS][FN];
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const int kq = (ks + kg) * 4 + fq;     // 16-byte chunk of this lane's K slice
      if constexpr (ABL & 8) {
#pragma unroll
        for (int i = 0; i < FM; ++i) af[ks][i] = (bf16x8){};
#pragma unroll
        for (int j = 0; j < FN; ++j) bfr[ks][j] = (bf16x8){};
      } else {
#pragma unroll
        for (int i = 0; i < FM; ++i) af[ks][i] = *(const bf16x8*)(sa + swz2(wm * TM + i * 16 + fr, kq));
#pragma unroll
        for (int j = 0; j < FN; ++j) bfr[ks][j] = *(const bf16x8*)(sb + swz2(wn * TN + j * 16 + fr, kq));
      }
    }
    if constexpr (ABL & 1) {
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
#pragma unroll
        for (int i = 0; i < FM; ++i) asm volatile("" ::"v"(af[ks][i]));
#pragma unroll
        for (int j = 0; j < FN; ++j) asm volatile("" ::"v"(bfr[ks][j]));
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks][i], bfr[ks][j], acc[i][j], 0, 0, 0);
    }
    if constexpr (ILV && NL == 0) {
      // LDS-DMA pieces for tile t+STAGES-1 spread between this tile's MFMAs
      // (one wave per SIMD: a piece costs ~100 issue cycles that otherwise
      // serialise in front of the MFMA block)
      issue(nslot);
      constexpr int MPP = MT / LPW > 0 ? MT / LPW : 1;
      __builtin_amdgcn_sched_group_barrier(0x100, 2 * NKS * (FM + FN), 0);   // ds_read
#pragma unroll
      for (int q = 0; q < LPW; ++q) {
        __builtin_amdgcn_sched_group_barrier(0x008, MPP, 0);          // MFMA
        __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);            // VMEM (LDS-DMA piece)
      }
      __builtin_amdgcn_sched_group_barrier(0x008, MT, 0);             // the rest
    }
  }
  wait_vm<0>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  // ---- epilogue (as conv_igemm.hip)
  float* epi = (float*)smem;
  if (!loader && kg == 0) {
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
    // K-group 1 adds its partial sums onto group 0's (same fragment layout)
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
  constexpr int CPR = BN / 8;
  constexpr int NCH = BM * CPR;
  if (p.ksplit > 1) {
    float* slab = p.ws + (size_t)split_idx * p.M * p.N;
    for (int c = tid; c < NCH; c += NT) {
      const int row = c / CPR, cc = c % CPR;
      const int m = m0 + row, n = n0 + cc * 8;
      if (m >= p.M || n >= p.N) continue;
      const float* e = epi + row * EPI_LD + cc * 8;
      *(f32x4*)(slab + (size_t)m * p.N + n) = *(const f32x4*)e;
      *(f32x4*)(slab + (size_t)m * p.N + n + 4) = *(const f32x4*)(e + 4);
    }
    return;
  }
  if (sk.slot < 0) {
    fused_epilogue<BM, BN, NT, EPI_LD, OUT_F32>(p, epi, m0, n0, tid, p.M, &rpre, use_pre);
    return;
  }
  const __amdgpu_buffer_rsrc_t wsr = ws_rsrc(p.ws);
  {
    // Stream-K partial tile: publish it with 16-B sc1 stores, then one lane
    // counts the arrival; the last of the tile's segments combines all partials
    // in segment order (deterministic) and runs the epilogue.  Nobody waits
    // on anybody, so co-residency of the grid is never required.
    // (MI355X_MICROARCH.md "inter-workgroup visibility", hand-off row 1.)
    const int base = sk.slot * BM * BN;
    for (int c = tid; c < NCH; c += NT) {
      const int row = c / CPR, cc = c % CPR;
      const float* e = epi + row * EPI_LD + cc * 8;
      const int off = (base + row * BN + cc * 8) * 4;
      __builtin_amdgcn_raw_buffer_store_b128(*(const u32x4*)e, wsr, off, 0, CPOL_SC1);
      __builtin_amdgcn_raw_buffer_store_b128(*(const u32x4*)(e + 4), wsr, off + 16, 0, CPOL_SC1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = (int*)(smem + S::LDS_BYTES);
    if (tid == 0) {
      const int old = __hip_atomic_fetch_add(p.counters + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = old == sk.nseg - 1;
      if (last) __hip_atomic_store(p.counters + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = last;
    }
    __syncthreads();
    if (!*flag) return;
  }
  const int ktt = p.Kpad / BK2;
  for (int c = tid; c < NCH; c += NT) {
    const int row = c / CPR, cc = c % CPR;
    const int m = m0 + row, n = n0 + cc * 8;
    if (m >= p.M || n >= p.N) continue;
    const float* e = epi + row * EPI_LD + cc * 8;
    float v[8];
    {
#pragma unroll
      for (int t = 0; t < 8; ++t) v[t] = 0.f;
      for (int sg = 0; sg < sk.nseg; ++sg) {
        f32x4 v0, v1;
        if (sg == sk.seg) {
          v0 = *(const f32x4*)e;
          v1 = *(const f32x4*)(e + 4);
        } else {
          const int off = (sk_slot(sk.g_first + sg, tile, ktt, p.sk_iters) * BM * BN + row * BN + cc * 8) * 4;
          u32x4 r0 = __builtin_amdgcn_raw_buffer_load_b128(wsr, off, 0, CPOL_SC1);
          u32x4 r1 = __builtin_amdgcn_raw_buffer_load_b128(wsr, off + 16, 0, CPOL_SC1);
          v0 = __builtin_bit_cast(f32x4, r0);
          v1 = __builtin_bit_cast(f32x4, r1);
        }
        v[0] += v0[0]; v[1] += v0[1]; v[2] += v0[2]; v[3] += v0[3];
        v[4] += v1[0]; v[5] += v1[1]; v[6] += v1[2]; v[7] += v1[3];
      }
    }
    if (p.bias) {
      f32x4 b0 = *(const f32x4*)(p.bias + n), b1 = *(const f32x4*)(p.bias + n + 4);
      v[0] += b0[0]; v[1] += b0[1]; v[2] += b0[2]; v[3] += b0[3];
      v[4] += b1[0]; v[5] += b1[1]; v[6] += b1[2]; v[7] += b1[3];
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
      *(f32x4*)o = (f32x4){v[0], v[1], v[2], v[3]};
      *(f32x4*)(o + 4) = (f32x4){v[4], v[5], v[6], v[7]};
    } else {
      V8 o;
#pragma unroll
      for (int t = 0; t < 8; ++t) o.e[t] = f2bf(v[t]);
      *(u32x4*)((bf16*)d.base + (size_t)m * d.ld + d.col) = o.u;
    }
  }
}

// One launch = (a) data-parallel tiles x split-K slices (p.ksplit >= 1), or
// (b) stream-K (p.ksplit < 0): the tiles x K-tiles iteration space is cut into
// equal contiguous ranges of p.sk_iters, one per block, so ~200-tile problems
// keep every CU busy instead of leaving a quarter of the chip idle.
template <int BM, int BN, int WM, int WN, int STAGES, bool ILV, bool PURE, bool OUT_F32, int ABL = 0, int NL = 0,
          int KG = 1>
__global__ __launch_bounds__((WM * WN * KG + NL) * 64, 1) void conv_glds_kernel(ConvParams p, const bf16* __restrict__ zero) {
  using S = GldsShape<BM, BN, WM, WN, STAGES>;
  __shared__ __attribute__((aligned(16))) char smem[S::LDS_BYTES + 16];
  const int tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  const int kt = p.Kpad / BK2;
  if (p.ksplit >= 1) {
    const int tile = xcd_remap(blockIdx.x, tiles);
    const int kt_per = (kt + p.ksplit - 1) / p.ksplit;
    const int kt0 = blockIdx.y * kt_per;
    const int kt1 = min(kt, kt0 + kt_per);
    glds_tile<BM, BN, WM, WN, STAGES, ILV, PURE, OUT_F32, ABL, NL, KG>(p, zero, smem, tile, kt0, kt1, blockIdx.y,
                                                                   SkSeg{-1, 1, 0, 0});
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
    SkSeg sk{-1, 1, 0, 0};
    if (kbeg != 0 || kend != kt) {
      const int g_first = (tile * kt) / iters, g_last = ((tile + 1) * kt - 1) / iters;
      sk = SkSeg{sk_slot(g, tile, kt, iters), g_last - g_first + 1, g - g_first, g_first};
    }
    glds_tile<BM, BN, WM, WN, STAGES, ILV, PURE, OUT_F32, ABL, NL, KG>(p, zero, smem, tile, kbeg, kend, 0, sk);
    it += kend - kbeg;
    __syncthreads();   // the next segment's DMA reuses the epilogue's LDS
  }
}

// 16-byte aligned zero page that out-of-range lanes fetch from
__device__ __attribute__((aligned(64))) bf16 g_zero_page[64];

// v2 tile configs: id -> BM, BN, WM, WN (WM*WN = 4 or 8 waves), STAGES, interleaved issue
// (ids continue after the v1 configs)
#define ADAPT_GLDS_CFGS(X)          \
  X(6, 128, 128, 2, 2, 3, false)    \
  X(7, 128, 128, 2, 2, 2, false)    \
  X(8, 128, 64, 2, 2, 4, false)     \
  X(9, 64, 128, 2, 2, 4, false)     \
  X(10, 64, 64, 2, 2, 4, false)     \
  X(11, 256, 64, 4, 1, 3, false)    \
  X(12, 64, 256, 1, 4, 3, false)    \
  X(13, 128, 128, 2, 2, 3, true)    \
  X(14, 128, 128, 4, 2, 3, false)   \
  X(15, 64, 128, 2, 4, 4, false)    \
  X(16, 64, 64, 2, 2, 4, true)      \
  X(17, 128, 64, 4, 2, 4, false)    \
  X(18, 64, 128, 2, 2, 4, true)     \
  X(19, 256, 64, 4, 2, 3, false)    \
  X(20, 128, 128, 4, 2, 3, true)    \
  X(21, 64, 64, 2, 4, 4, false)     \
  X(22, 128, 128, 4, 2, 4, true)    \
  X(23, 64, 128, 2, 4, 4, true)     \
  X(24, 64, 64, 2, 4, 4, true)      \
  X(25, 128, 64, 4, 2, 4, true)     \
  X(26, 256, 64, 4, 2, 3, true)     \
  X(27, 64, 256, 2, 4, 3, true)     \
  X(28, 128, 256, 4, 2, 3, true)    \
  X(29, 256, 128, 4, 2, 3, true)    \
  X(30, 128, 128, 4, 2, 2, true)    \
  X(31, 64, 128, 2, 4, 3, true)     \
  X(32, 128, 64, 4, 2, 3, true)     \
  X(33, 128, 128, 2, 2, 2, true)    \
  X(34, 64, 64, 2, 2, 3, true)     \
  X(35, 64, 128, 2, 4, 6, true)    \
  X(36, 128, 64, 4, 2, 6, true)    \
  X(37, 64, 64, 2, 2, 8, true)     \
  X(38, 64, 128, 2, 4, 5, true)    \
  X(39, 64, 64, 2, 4, 8, true)     \
  X(53, 128, 128, 4, 4, 4, true)   \
  X(54, 128, 128, 4, 4, 3, true)   \
  X(55, 256, 128, 8, 2, 3, true)   \
  X(56, 128, 256, 2, 8, 3, true)   \
  X(57, 256, 128, 4, 4, 3, true)   \
  X(58, 128, 128, 4, 4, 2, true)

// 62-70: two K-groups (KG = 2) of WM x WN waves, 8 waves per block; per-wave
// sub-tiles of 32x64 .. 64x128 (see glds_tile)
#define ADAPT_GLDS_KG_CFGS(X)       \
  X(62, 64, 128, 2, 2, 4, true)     \
  X(63, 128, 128, 2, 2, 3, true)    \
  X(64, 64, 256, 1, 4, 3, true)     \
  X(65, 128, 128, 2, 2, 4, true)    \
  X(66, 64, 128, 2, 2, 3, true)     \
  X(67, 128, 64, 2, 2, 4, true)     \
  X(68, 64, 64, 2, 2, 4, true)      \
  X(69, 128, 256, 2, 2, 3, true)    \
  X(70, 256, 128, 2, 2, 3, true)

// 53-58: 16 waves (4 per SIMD) per block: twice the LDS-DMA pieces in flight per
// CU at the same tile size.  Measured (profiles/conv_bench_v7_16w.txt): within
// 1-2 % of the 8-wave tiles on every ResNet-50 shape (ahead only on the stage-3
// 1x1 512->128), so per-CU issue depth is not what bounds these layers; kept as
// autotuner candidates.
// 35-39: deeper rings (5-8 stages) for the small-grid layers, where one block
// per CU streams ~30 K-tiles whose ~0.2 us of MFMA work each cannot cover the
// L2/HBM latency with 2-3 tiles in flight
int conv_glds_num_cfgs() { return 34; }

// stream-K grid: `mult` x 256 blocks (one per CU), each taking ceil(total / G)
// consecutive (tile, K-tile) iterations
void conv_sk_plan(int tiles, int kt, int mult, int* grid, int* iters) {
  const long long total = (long long)tiles * kt;
  long long G = 256LL * (mult > 0 ? mult : 1);
  if (G > total) G = total;
  const long long it = (total + G - 1) / G;
  *iters = (int)it;
  *grid = (int)((total + it - 1) / it);
}

bool conv_glds_cfg_tile(int cfg, int* bm, int* bn) {
  switch (cfg) {
#define X(id, BM_, BN_, WM_, WN_, S_, I_) case id: *bm = BM_; *bn = BN_; return true;
    ADAPT_GLDS_CFGS(X)
    ADAPT_GLDS_KG_CFGS(X)
#undef X
  }
  return false;
}

template <int BM, int BN, int WM, int WN, int S, bool ILV, int KG = 1>
static hipError_t launch_glds(const ConvParams& p, hipStream_t s, bool pure, bool out_f32) {
  static bf16* zero = nullptr;
  if (!zero) {
    hipError_t e = hipGetSymbolAddress((void**)&zero, HIP_SYMBOL(g_zero_page));
    if (e != hipSuccess) return e;
  }
  const int tilesM = (p.M + BM - 1) / BM, tilesN = (p.N + BN - 1) / BN;
  dim3 grid(tilesM * tilesN, p.ksplit), block(WM * WN * KG * 64);
  if (p.ksplit < 0) {
    int g, iters;
    conv_sk_plan(tilesM * tilesN, p.Kpad / BK2, -p.ksplit, &g, &iters);
    if (!p.counters || !p.ws || iters != p.sk_iters) return hipErrorInvalidValue;
    grid = dim3(g, 1);
  }
  if (pure) {
    if (out_f32) hipLaunchKernelGGL((conv_glds_kernel<BM, BN, WM, WN, S, ILV, true, true, 0, 0, KG>), grid, block, 0, s, p, zero);
    else hipLaunchKernelGGL((conv_glds_kernel<BM, BN, WM, WN, S, ILV, true, false, 0, 0, KG>), grid, block, 0, s, p, zero);
  } else {
    if (out_f32) hipLaunchKernelGGL((conv_glds_kernel<BM, BN, WM, WN, S, ILV, false, true, 0, 0, KG>), grid, block, 0, s, p, zero);
    else hipLaunchKernelGGL((conv_glds_kernel<BM, BN, WM, WN, S, ILV, false, false, 0, 0, KG>), grid, block, 0, s, p, zero);
  }
  return hipGetLastError();
}

hipError_t conv_glds_launch(const ConvParams& p, int cfg, hipStream_t s, bool pure, bool out_f32) {
  switch (cfg) {
#define X(id, BM_, BN_, WM_, WN_, S_, I_) case id: return launch_glds<BM_, BN_, WM_, WN_, S_, I_>(p, s, pure, out_f32);
    ADAPT_GLDS_CFGS(X)
#undef X
#define X(id, BM_, BN_, WM_, WN_, S_, I_) case id: return launch_glds<BM_, BN_, WM_, WN_, S_, I_, 2>(p, s, pure, out_f32);
    ADAPT_GLDS_KG_CFGS(X)
#undef X
  }
  return hipErrorInvalidValue;
}

}  // namespace adapt
