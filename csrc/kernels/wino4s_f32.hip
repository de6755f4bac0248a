// fp32 3x3 / stride-1 / pad-1 convolution by Winograd F(4x4, 3x3), split into two launches so the matrix
// loop is pure MFMA:
//
//   1. wino4s_in_kernel   V = B^T d B of every 6x6 input patch (memory-bound, all VALU work of the input
//                         transform happens here, once per (tile, channel)), written in fragment order;
//   2. wino4s_gemm_kernel M_p = V_p U_p for the 36 positions p of a block of tiles x output channels, with
//                         the output transform y = A^T M A + bias (+ ReLU) applied to the accumulators in
//                         registers (every lane holds all 36 positions of its (tile, channel) pairs).
//   3. wino4s_reduce_kernel (split-K only): the splits' partial outputs summed in split order + bias / ReLU.
//
// Why this shape (MI355X-first): the fused F(4x4) kernels (conv_wino4_f32.hip) transform the input inside
// the K loop, and that fp32 VALU work takes issue cycles from the MFMA of the partner wave on the same SIMD
// (profiles/r5/wino4_attribution.md: 33.4 -> 38.6 cycles per MFMA).  Here the K loop issues nothing but
// LDS-DMA, ds_read_b128 and v_mfma_f32_16x16x4_f32.  F(4x4) does 2.25 multiplies per output against 4 for
// F(2x2) and 9 for direct convolution; everything stays fp32 (the reference's Keras float32
// `model.predict`, /root/reference/test/local_infer.py:22; ResNet-50 /root/reference/test/test.py:13).
//
// Fragment order (both operands, 1 KiB units, one per (16-group, 16-channel chunk kc, position p)):
//   V[tg][kc][p][lane][4]: lane l = 16 g + r holds V_p[tile 16 tg + r][channel 16 kc + 4 g + j] at j;
//   U[ng][kc][p][lane][4]: lane l = 16 g + n holds U_p[channel 16 kc + 4 g + j][cout 16 ng + n] at j.
// MFMA step j of a unit takes element j of every lane: A[row r][k = g] with channel 4 g + j, B[k = g][col n]
// with the same channel, so one ds_read_b128 per operand feeds 4 MFMAs and a unit is read lane-linear
// (conflict-free).  The same units are what the LDS-DMA moves, 16 B per lane.
//
// GEMM block = WT x WN waves, wave (wt, wn) owns 16 tiles x 16 channels x 36 positions = 144 accumulators
// (f32x4 acc[36]); the block's operands stream through an R-slot LDS ring of stages, a stage being PG
// positions of one chunk for all its tile and channel groups ((WT + WN) x PG units), each wave issuing an
// equal share of the stage's LDS-DMA pieces R - 1 stages ahead.  One s_barrier per stage: after it, every
// wave's pieces of this stage have landed (each waited for its own with a partial vmcnt first) and every
// wave is done reading the previous stage, whose slot is then refilled.
#include <cstdlib>

#include "kernels.h"

namespace adapt {

namespace {

typedef float f32x4v __attribute__((ext_vector_type(4)));

constexpr unsigned W4S_OOB = 0x80000000u;        // a voff past the descriptor's range: the DMA writes zeros

__device__ __forceinline__ u32x4 w4s_desc(const float* base) {
  const unsigned long long a = (unsigned long long)(uintptr_t)base;
  return (u32x4){(unsigned)a, (unsigned)(a >> 32) & 0xffffu, 0x7fffffffu, 0x00020000u};
}

// one 1 KiB LDS-DMA piece: 16 B per lane from descriptor base + voff + soff to LDS byte address `lds` + 16 lane
// (inline asm: M0 is set in the same statement; the compiler's wait-count model never sees the DMA, the
// kernel waits for it with explicit vmcnt)
__device__ __forceinline__ void w4s_dma(unsigned voff, u32x4 rsrc, unsigned soff, unsigned lds) {
  asm volatile("s_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds" ::"v"(voff), "s"(rsrc),
               "s"(soff), "s"(lds)
               : "memory");
}

template <int N>
__device__ __forceinline__ void w4s_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// B^T of F(4x4, 3x3) on 6 values: rows [4 0 -5 0 1 0], [0 -4 -4 1 1 0], [0 4 -4 -1 1 0], [0 -2 -1 2 1 0],
// [0 2 -1 -2 1 0], [0 4 0 -5 0 1] (elementwise on T = float or a float vector)
template <typename T>
__device__ __forceinline__ void w4s_bt(T& d0, T& d1, T& d2, T& d3, T& d4, T& d5) {
  const T s12 = d1 + d2, s34 = d3 + d4, m12 = d1 - d2, m43 = d4 - d3, m13 = d1 - d3, m42 = d4 - d2;
  const T t0 = 4.f * d0 - 5.f * d2 + d4;
  const T t5 = 4.f * d1 - 5.f * d3 + d5;
  d1 = s34 - 4.f * s12;
  d2 = 4.f * m12 + m43;
  d3 = m42 - 2.f * m13;
  d4 = 2.f * m13 + m42;
  d0 = t0;
  d5 = t5;
}

// A^T of F(4x4, 3x3) on 6 values -> 4: rows [1 1 1 1 1 0], [0 1 -1 2 -2 0], [0 1 1 4 4 0], [0 1 -1 8 -8 1]
__device__ __forceinline__ void w4s_at(float m0, float m1, float m2, float m3, float m4, float m5, float& o0,
                                       float& o1, float& o2, float& o3) {
  const float s12 = m1 + m2, d12 = m1 - m2, s34 = m3 + m4, d34 = m3 - m4;
  o0 = m0 + s12 + s34;
  o1 = fmaf(2.f, d34, d12);
  o2 = fmaf(4.f, s34, s12);
  o3 = fmaf(8.f, d34, d12) + m5;
}

// ---------------------------------------------------------------- 1. input transform
// One block of 256 threads per (tile group, chunk) unit and CPT channels per thread (CPT = 1, 2, 4; 4 / CPT
// units per block): thread (l, jj) owns fragment lane l = 16 g + r (tile 16 tg + r) and elements
// CPT jj .. CPT jj + CPT - 1 (channels 16 kc + 4 g + CPT jj + e).  Each of the 36 position stores of a unit is
// one contiguous KiB; each pixel read is a CPT x 4-byte load whose lane neighbours fill a 64-B segment.
// CPT trades load width (4: 16-B loads, 1/4 of the threads) against parallelism (1: 4x the waves, for the
// small late-stage maps whose unit count alone would not fill the chip).
template <int CPT>
__global__ __launch_bounds__(256) void wino4s_in_kernel(Wino4sParams p) {
  typedef float vec __attribute__((ext_vector_type(CPT)));
  constexpr int TPU = 64 * 4 / CPT;                // threads per unit
  const int unit = blockIdx.x * (256 / TPU) + threadIdx.x / TPU;
  if (unit >= p.TG * p.KC) return;
  const int tid = threadIdx.x % TPU;
  const int tg = unit / p.KC, kc = unit - tg * p.KC;
  const int l = tid / (4 / CPT), jj = tid % (4 / CPT);
  const int r = l & 15, g = l >> 4;
  const int t = tg * 16 + r;
  vec d[6][6];
  const vec z = (vec)(0.f);
  if (t < p.T) {
    const int per = p.TH * p.TW;
    const int b = t / per, rem = t - b * per;
    const int th = rem / p.TW, tw = rem - th * p.TW;
    const int h0 = 4 * th - 1, w0 = 4 * tw - 1;
    const float* xb = p.x + (size_t)b * p.H * p.W * p.C + kc * 16 + 4 * g + CPT * jj;
#pragma unroll
    for (int dy = 0; dy < 6; ++dy) {
      const int h = h0 + dy;
#pragma unroll
      for (int dx = 0; dx < 6; ++dx) {
        const int w = w0 + dx;
        d[dy][dx] = (h >= 0 && h < p.H && w >= 0 && w < p.W) ? *(const vec*)(xb + ((size_t)h * p.W + w) * p.C) : z;
      }
    }
  } else {
#pragma unroll
    for (int dy = 0; dy < 6; ++dy)
#pragma unroll
      for (int dx = 0; dx < 6; ++dx) d[dy][dx] = z;
  }
#pragma unroll
  for (int dx = 0; dx < 6; ++dx) w4s_bt(d[0][dx], d[1][dx], d[2][dx], d[3][dx], d[4][dx], d[5][dx]);
#pragma unroll
  for (int a = 0; a < 6; ++a) w4s_bt(d[a][0], d[a][1], d[a][2], d[a][3], d[a][4], d[a][5]);
  vec* vo = (vec*)(p.v + (size_t)unit * 36 * 256) + tid;
#pragma unroll
  for (int a = 0; a < 6; ++a)
#pragma unroll
    for (int b = 0; b < 6; ++b) vo[(a * 6 + b) * TPU] = d[a][b];
}

// ---------------------------------------------------------------- 2. GEMM + output transform
// PIPE: the fragments of stage st + 1 are read (after its barrier) before the MFMAs of stage st are issued,
// so the LDS read latency runs under the MFMA burst instead of in front of it (two fragment register sets)
// STAMP (measurement only, tools/wino4s_timeline.py): lane 0 of every wave writes 8 words to p.dbg --
// shader clock at start / first stage landed / K loop done / epilogue done, the summed clocks spent in the
// per-stage land wait (vmcnt + barrier), the summed clocks from each barrier to the stage's last MFMA issue,
// the stage count and HW_ID
template <int WT, int WN, int PG, int R, bool PIPE, bool STAMP = false>
__global__ __launch_bounds__(WT * WN * 64, 2) void wino4s_gemm_kernel(Wino4sParams p) {
  constexpr int NW = WT * WN;
  constexpr int NST = 36 / PG;                   // stages per 16-channel chunk
  constexpr int PIECES = (WT + WN) * PG;         // 1 KiB units per stage
  constexpr int PPW = PIECES / NW;               // LDS-DMA pieces per wave per stage
  constexpr int SLOT = PIECES * 1024;
  static_assert(36 % PG == 0 && (WT * PG) % NW == 0 && (WN * PG) % NW == 0, "stage geometry");
  static_assert(R >= 2 && R * SLOT <= 160 * 1024, "LDS ring");
  static_assert((R - 2) * PPW < 64, "vmcnt range");
  __shared__ __attribute__((aligned(16))) char smem[R * SLOT];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wt = wave / WN, wn = wave - wt * WN;
  // block -> (split, tile block, channel block); blocks whose index differs by a multiple of 8 run on one XCD,
  // so consecutive logical ids (which share operands) are gathered onto one XCD when the grid allows
  const int TBn = (p.TG + WT - 1) / WT, NBn = p.N / (16 * WN), S = p.ksplit;
  const int nblk = TBn * NBn * S;
  int L = blockIdx.x;
  if ((nblk & 7) == 0) L = (L & 7) * (nblk >> 3) + (L >> 3);
  int s, tb, nb;
  if (p.order == 0) {
    nb = L % NBn;
    L /= NBn;
    tb = L % TBn;
    s = L / TBn;
  } else {
    tb = L % TBn;
    L /= TBn;
    nb = L % NBn;
    s = L / NBn;
  }
  const int KCs = p.KC / S, kc0 = s * KCs;
  const int NS = KCs * NST;
  const u32x4 rv = w4s_desc(p.v), ru = w4s_desc(p.u);
  const unsigned lds0 = (unsigned)(uintptr_t)smem;

  // this wave's pieces of a stage: i = NW j + wave.  With WT PG and WN PG multiples of NW, piece j is an A
  // unit (tile group, position) for j < WT PG / NW and a B unit (channel group, position) after that, for
  // every wave alike, so the descriptor is chosen at compile time; a piece's group / position part of its
  // source offset is fixed for the whole loop (sbase), the stage adds (kc 36 + p0) KiB.
  constexpr int PJA = WT * PG / NW;
  unsigned sbase[PPW];
  bool aval[PJA > 0 ? PJA : 1];
#pragma unroll
  for (int j = 0; j < PPW; ++j) {
    const int i = NW * j + wave;
    if (j < PJA) {
      const int wi = i / PG, pp = i - wi * PG;
      const int tgi = tb * WT + wi;
      aval[j] = tgi < p.TG;
      sbase[j] = (unsigned)((tgi * p.KC * 36 + pp) * 1024);
    } else {
      const int i2 = i - WT * PG;
      const int wi = i2 / PG, pp = i2 - wi * PG;
      sbase[j] = (unsigned)(((nb * WN + wi) * p.KC * 36 + pp) * 1024);
    }
  }
  const unsigned vlane = (unsigned)lane * 16u;
  auto issue = [&](int st) {
    const int kc = kc0 + st / NST, p0 = (st % NST) * PG;
    const unsigned soff = (unsigned)((kc * 36 + p0) * 1024);
    const unsigned slot = lds0 + (unsigned)((st % R) * SLOT) + (unsigned)wave * 1024u;
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
      if (j < PJA) w4s_dma(aval[j] ? vlane : W4S_OOB, rv, sbase[j] + soff, slot + NW * j * 1024);
      else w4s_dma(vlane, ru, sbase[j] + soff, slot + NW * j * 1024);
    }
  };

  f32x4v acc[36];
#pragma unroll
  for (int q = 0; q < 36; ++q) acc[q] = (f32x4v){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int st = 0; st < R - 1; ++st)
    if (st < NS) issue(st);

  const char* const ra = smem + (wt * PG) * 1024 + lane * 16;
  const char* const rb = smem + (WT * PG + wn * PG) * 1024 + lane * 16;
  unsigned long long t_start = 0, t_first = 0, t_wait = 0, t_mfma = 0, t_mark = 0;
  if constexpr (STAMP) t_start = __builtin_amdgcn_s_memtime();
  auto wait_land = [&](int st) {        // this wave's pieces of stage st have landed, then every wave's
    unsigned long long t0 = 0;
    if constexpr (STAMP) t0 = __builtin_amdgcn_s_memtime();
    if (NS - 1 - st >= R - 2) w4s_vmcnt<(R - 2) * PPW>();
    else w4s_vmcnt<0>();
    __builtin_amdgcn_s_barrier();       // every wave's pieces of st landed; st - 1 fully read
    asm volatile("" ::: "memory");
    if constexpr (STAMP) {
      t_mark = __builtin_amdgcn_s_memtime();
      t_wait += t_mark - t0;
      if (st == 0) t_first = t_mark;
    }
    if (st + R - 1 < NS) issue(st + R - 1);
  };
  auto read = [&](int st, f32x4v (&a)[PG], f32x4v (&b)[PG]) {
    const int so = (st % R) * SLOT;
#pragma unroll
    for (int pp = 0; pp < PG; ++pp) {
      a[pp] = *(const f32x4v*)(ra + so + pp * 1024);
      b[pp] = *(const f32x4v*)(rb + so + pp * 1024);
    }
  };
  // MFMAs step-major: consecutive MFMAs accumulate into different positions (a dependent 16x16x4 f32 MFMA
  // waits 40 cycles, an independent one issues at 32)
  auto mfmas = [&](int sg, const f32x4v (&a)[PG], const f32x4v (&b)[PG]) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int pp = 0; pp < PG; ++pp)
        acc[sg * PG + pp] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[pp][j], b[pp][j], acc[sg * PG + pp], 0, 0, 0);
  };
  if constexpr (!PIPE) {
    for (int kcl = 0; kcl < KCs; ++kcl) {
#pragma unroll
      for (int sg = 0; sg < NST; ++sg) {
        const int st = kcl * NST + sg;
        wait_land(st);
        f32x4v a[PG], b[PG];
        read(st, a, b);
        mfmas(sg, a, b);
        if constexpr (STAMP) t_mfma += __builtin_amdgcn_s_memtime() - t_mark;
      }
    }
  } else {
    f32x4v ca[PG], cb[PG];
    wait_land(0);
    read(0, ca, cb);
    for (int kcl = 0; kcl < KCs; ++kcl) {
#pragma unroll
      for (int sg = 0; sg < NST; ++sg) {
        const int st = kcl * NST + sg;
        f32x4v na[PG], nb_[PG];
        if (st + 1 < NS) {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // own reads of st done: its slot is refilled
          wait_land(st + 1);                                      // after this barrier
          read(st + 1, na, nb_);
        }
        mfmas(sg, ca, cb);
#pragma unroll
        for (int pp = 0; pp < PG; ++pp) {
          ca[pp] = na[pp];
          cb[pp] = nb_[pp];
        }
      }
    }
  }

  unsigned long long t_loop = 0;
  if constexpr (STAMP) t_loop = __builtin_amdgcn_s_memtime();
  // ---- output transform on the accumulators: lane l holds M_p[tile 16 tg + 4 (l >> 4) + i][cout] at acc[p][i]
  const int tg = tb * WT + wt;
  const int n = (nb * WN + wn) * 16 + (lane & 15);
  float y[4][16];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float tr[6][4];                                 // A^T applied along b: tr[a][j]
#pragma unroll
    for (int a = 0; a < 6; ++a)
      w4s_at(acc[a * 6 + 0][i], acc[a * 6 + 1][i], acc[a * 6 + 2][i], acc[a * 6 + 3][i], acc[a * 6 + 4][i],
             acc[a * 6 + 5][i], tr[a][0], tr[a][1], tr[a][2], tr[a][3]);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      w4s_at(tr[0][j], tr[1][j], tr[2][j], tr[3][j], tr[4][j], tr[5][j], y[i][j], y[i][4 + j], y[i][8 + j],
             y[i][12 + j]);
  }
  // Output rows leave through LDS: the block's (tile, pixel) rows of WN x 16 channels are staged, then stored
  // as 16-B chunks, 8 lanes per 128-B row segment (direct from the fragments every store instruction would
  // write 4 x 64 B with 4-B lanes: 12 us of the stage-2 epilogue, tools/wino4s_timeline.py)
  constexpr int CB = WN * 16, RP = CB + 4;
  constexpr bool STAGE = WT * 16 * 16 * RP * 4 <= R * SLOT;      // the padded rows fit in the ring
  const int per = p.TH * p.TW;
  auto store_rows = [&](auto&& rowp) {
    if constexpr (STAGE) {
      __syncthreads();                               // every wave is done with the ring
      float* stg = (float*)smem;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int u = 0; u < 16; ++u)
          stg[((wt * 16 + 4 * (lane >> 4) + i) * 16 + u) * RP + wn * 16 + (lane & 15)] = y[i][u];
      __syncthreads();
      constexpr int C4 = CB / 4, TOTAL = WT * 16 * 16 * C4;
      for (int e = threadIdx.x; e < TOTAL; e += NW * 64) {
        const int c4 = e % C4, row = e / C4;
        const int t = tb * WT * 16 + row / 16;
        float* dst = rowp(t, row & 15);
        if (dst) *(f32x4v*)(dst + nb * CB + c4 * 4) = *(const f32x4v*)(stg + row * RP + c4 * 4);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          float* dst = rowp(tg * 16 + 4 * (lane >> 4) + i, u);
          if (dst) dst[n] = y[i][u];
        }
    }
  };
  auto write_stamps = [&]() {
    if constexpr (STAMP) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned long long t_end = __builtin_amdgcn_s_memtime();
      if (lane == 0 && p.dbg) {
        unsigned long long* d = p.dbg + (size_t)(blockIdx.x * NW + wave) * 8;
        d[0] = t_start;
        d[1] = t_first;
        d[2] = t_loop;
        d[3] = t_end;
        d[4] = t_wait;
        d[5] = t_mfma;
        d[6] = (unsigned long long)NS;
        d[7] = ((unsigned long long)__builtin_amdgcn_s_getreg(0x7814) << 32) | (unsigned)__builtin_amdgcn_s_getreg(0xF804);
      }
    }
  };
  if (S > 1 && p.counters == nullptr) {
    // split-K through wino4s_reduce_kernel: partial outputs [split][tile][16 pixels][N]
    store_rows([&](int t, int u) -> float* {
      return t < p.T ? p.ws + (((size_t)s * p.TG * 16 + t) * 16 + u) * p.N : nullptr;
    });
    write_stamps();
    return;
  }
  if (S > 1) {
    // fused split-K: every split publishes its partial outputs as 16-B sc1 stores in lane order (each lane
    // re-reads exactly what the same lane of the other splits wrote); the last split of the (tile, channel)
    // block to arrive adds the splits in split order -- deterministic whichever arrives last
    const int blk = tb * NBn + nb;
    const __amdgpu_buffer_rsrc_t wsr =
        __builtin_amdgcn_make_buffer_rsrc((void*)p.ws, (short)0, 0x7fffffff, 0x00020000);
    const unsigned lane_base = (unsigned)(((size_t)blk * NW + wave) * 4096 + lane * 4) * 4u;
    const unsigned split_stride = (unsigned)((size_t)TBn * NBn * NW * 4096 * 4);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const f32x4v v = {y[q >> 2][(q & 3) * 4], y[q >> 2][(q & 3) * 4 + 1], y[q >> 2][(q & 3) * 4 + 2],
                        y[q >> 2][(q & 3) * 4 + 3]};
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), wsr,
                                             lane_base + s * split_stride + q * 1024u, 0, 16 /* sc1 */);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = (int*)smem;
    if (threadIdx.x == 0) {
      int* ctr = p.counters + blk;
      const int old = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = old == S - 1;
      if (last) __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = last;
    }
    __syncthreads();
    if (!*flag) return;
    // the other splits' slabs, 2 float4 per split per round with every load of a round in flight at once
    // (their latency is a cross-XCD round trip), then the sums in split order
#pragma unroll
    for (int q0 = 0; q0 < 16; q0 += 2) {
      f32x4v sl[7][2];
#pragma unroll
      for (int zz = 0; zz < 7; ++zz) {
        const int z = zz < s ? zz : zz + 1;            // the splits other than this one, in order
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          sl[zz][k] = (f32x4v){0.f, 0.f, 0.f, 0.f};
          if (z < S)
            sl[zz][k] = __builtin_bit_cast(f32x4v, __builtin_amdgcn_raw_buffer_load_b128(
                                                     wsr, lane_base + z * split_stride + (q0 + k) * 1024u, 0, 16));
        }
      }
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int q = q0 + k;
        const f32x4v mine = {y[q >> 2][(q & 3) * 4], y[q >> 2][(q & 3) * 4 + 1], y[q >> 2][(q & 3) * 4 + 2],
                             y[q >> 2][(q & 3) * 4 + 3]};
        // split order with this split's own partial at position s; every array index is a constant (a
        // runtime index would put sl in scratch)
        f32x4v v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int z = 0; z < 8; ++z) {
          if (z >= S) break;
          const f32x4v other = z < 7 ? sl[z < 7 ? z : 6][k] : (f32x4v){0.f, 0.f, 0.f, 0.f};
          const f32x4v prev = z > 0 ? sl[z > 0 ? z - 1 : 0][k] : (f32x4v){0.f, 0.f, 0.f, 0.f};
          v += z < s ? other : (z == s ? mine : prev);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) y[q >> 2][(q & 3) * 4 + e] = v[e];
      }
    }
  }
  const float bv = p.bias[n];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int u = 0; u < 16; ++u) y[i][u] = act_relu(y[i][u] + bv, p.relu);
  store_rows([&](int t, int u) -> float* {
    if (t >= p.T) return nullptr;
    const int b = t / per, rem = t - b * per;
    const int th = rem / p.TW, tw = rem - th * p.TW;
    const int h = 4 * th + (u >> 2), w = 4 * tw + (u & 3);
    return h < p.H && w < p.W ? p.out + (((size_t)b * p.H + h) * p.W + w) * p.N : nullptr;
  });
  write_stamps();
}

// ---------------------------------------------------------------- 3. split-K reduce
// one thread per (tile, pixel, 4 channels): sum the splits in order, bias, activation, scatter to NHWC
__global__ __launch_bounds__(256) void wino4s_reduce_kernel(Wino4sParams p) {
  const int N4 = p.N / 4;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  const long total = (long)p.T * 16 * N4;
  if (idx >= total) return;
  const int n4 = (int)(idx % N4);
  const long tp = idx / N4;
  const int u = (int)(tp & 15);
  const int t = (int)(tp >> 4);
  const int per = p.TH * p.TW;
  const int b = t / per, rem = t - b * per;
  const int th = rem / p.TW, tw = rem - th * p.TW;
  const int h = 4 * th + (u >> 2), w = 4 * tw + (u & 3);
  if (h >= p.H || w >= p.W) return;
  const size_t slab = (size_t)p.TG * 16 * 16 * p.N;
  const f32x4v* src = (const f32x4v*)(p.ws + ((size_t)t * 16 + u) * p.N) + n4;
  f32x4v acc = src[0];
  for (int s = 1; s < p.ksplit; ++s) acc += src[s * (slab / 4)];
  const f32x4v bv = *((const f32x4v*)p.bias + n4);
  f32x4v o;
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = act_relu(acc[j] + bv[j], p.relu);
  *((f32x4v*)(p.out + (((size_t)b * p.H + h) * p.W + w) * p.N) + n4) = o;
}

// the same with the split count a template parameter (every split's load in flight at once) and 32-bit index
// math (the generic kernel's 64-bit divisions are software sequences)
template <int KS>
__global__ __launch_bounds__(256) void wino4s_reduce_ks_kernel(Wino4sParams p) {
  const int N4 = p.N >> 2;
  const unsigned idx = blockIdx.x * 256u + threadIdx.x;
  const unsigned total = (unsigned)p.T * 16u * (unsigned)N4;
  if (idx >= total) return;
  const unsigned tp = idx / (unsigned)N4;
  const int n4 = (int)(idx - tp * (unsigned)N4);
  const int u = (int)(tp & 15u), t = (int)(tp >> 4);
  const int per = p.TH * p.TW;
  const int b = t / per, rem = t - b * per;
  const int th = rem / p.TW, tw = rem - th * p.TW;
  const int h = 4 * th + (u >> 2), w = 4 * tw + (u & 3);
  if (h >= p.H || w >= p.W) return;
  const unsigned slab4 = (unsigned)p.TG * 16u * 16u * (unsigned)N4;        // f32x4 per split slab
  const f32x4v* src = (const f32x4v*)p.ws + tp * (unsigned)N4 + n4;
  f32x4v part[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) part[s] = src[s * slab4];
  f32x4v acc = part[0];
#pragma unroll
  for (int s = 1; s < KS; ++s) acc += part[s];
  const f32x4v bv = *((const f32x4v*)p.bias + n4);
  f32x4v o;
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = act_relu(acc[j] + bv[j], p.relu);
  *((f32x4v*)(p.out + (((size_t)b * p.H + h) * p.W + w) * p.N) + n4) = o;
}

struct W4sCfg {
  int wt, wn, pg, r, order;
};

// cfg id -> geometry (WT x WN waves, PG positions per stage, R-slot ring, block order 0: channel blocks
// fastest / 1: tile blocks fastest)
bool w4s_cfg(int cfg, W4sCfg* c) {
  switch (cfg) {
    case 220: *c = {2, 2, 6, 4, 0}; return true;
    case 221: *c = {2, 2, 6, 3, 0}; return true;
    case 222: *c = {1, 2, 6, 4, 0}; return true;
    case 223: *c = {2, 4, 4, 4, 0}; return true;
    case 224: *c = {2, 2, 6, 4, 1}; return true;
    case 225: *c = {2, 1, 6, 4, 0}; return true;
    case 226: *c = {1, 1, 9, 4, 0}; return true;
    case 227: *c = {2, 2, 4, 4, 0}; return true;
    case 228: *c = {4, 2, 4, 4, 0}; return true;
    case 229: *c = {4, 2, 4, 4, 1}; return true;
    case 230: *c = {2, 2, 12, 3, 0}; return true;
    case 231: *c = {2, 2, 12, 3, 1}; return true;
    case 232: *c = {2, 2, 4, 4, 0}; return true;     // 232-235: pipelined fragment reads (PIPE)
    case 233: *c = {2, 2, 6, 3, 0}; return true;
    case 234: *c = {2, 2, 6, 4, 0}; return true;
    case 235: *c = {2, 4, 4, 4, 0}; return true;
    case 236: *c = {2, 2, 4, 5, 0}; return true;     // 236-237: deeper rings at 2 blocks per CU
    case 237: *c = {2, 2, 2, 8, 0}; return true;
    case 299: *c = {2, 2, 6, 3, 0}; return true;     // 221 + per-wave stamps (measurement, wino4s_set_debug)
  }
  return false;
}

template <int WT, int WN, int PG, int R, bool PIPE = false, bool STAMP = false>
hipError_t launch_gemm(const Wino4sParams& p, hipStream_t s) {
  const int TBn = (p.TG + WT - 1) / WT, NBn = p.N / (16 * WN);
  hipLaunchKernelGGL((wino4s_gemm_kernel<WT, WN, PG, R, PIPE, STAMP>), dim3(TBn * NBn * p.ksplit),
                     dim3(WT * WN * 64), 0, s, p);
  return hipGetLastError();
}

}  // namespace

// ksplit >= 1: whole K (1) or split-K through the reduce launch; <= -2: split-K with the fixup fused (needs
// one int32 arrival counter per (tile, channel) block, wino4s_blocks, zero before and left zero after)
bool wino4s_ok(int cfg, int C, int N, int ksplit) {
  W4sCfg c;
  const int ks = ksplit < 0 ? -ksplit : ksplit;
  if (!w4s_cfg(cfg, &c) || C % 16 || N % (16 * c.wn) || ks < 1 || ks > 8 || ksplit == -1) return false;
  return (C / 16) % ks == 0;
}

int wino4s_blocks(int cfg, int B, int H, int W, int N) {
  W4sCfg c;
  if (!w4s_cfg(cfg, &c)) return 0;
  const int T = B * ((H + 3) / 4) * ((W + 3) / 4);
  const int TG = (T + 15) / 16;
  return ((TG + c.wt - 1) / c.wt) * (N / (16 * c.wn));
}

size_t wino4s_ws_floats(int B, int H, int W, int C, int N, int ksplit) {
  const int T = B * ((H + 3) / 4) * ((W + 3) / 4);
  const size_t TG = (size_t)(T + 15) / 16;
  size_t v = TG * 16 * (size_t)C * 36;
  const int ks = ksplit < 0 ? -ksplit : ksplit;
  // split slabs: [split][tile][16][N] (reduce launch) or [split][block][wave][4096] (fused); the fused form
  // covers whole blocks (tile groups rounded up to the block's WT, at most 4 more)
  if (ks > 1) v += (size_t)ks * (TG + 4) * 16 * 16 * N;
  return v;
}

static unsigned long long* g_w4s_dbg = nullptr;
void wino4s_set_debug(unsigned long long* buf) { g_w4s_dbg = buf; }

hipError_t wino4s_forward(const Wino4sParams& p_in, int cfg, hipStream_t s) {
  Wino4sParams p = p_in;
  p.dbg = g_w4s_dbg;
  W4sCfg c;
  if (!wino4s_ok(cfg, p.C, p.N, p.ksplit) || !w4s_cfg(cfg, &c)) return hipErrorInvalidValue;
  const bool fused = p.ksplit < 0;
  if (fused && !p.counters) return hipErrorInvalidValue;
  if (!fused) p.counters = nullptr;
  p.ksplit = fused ? -p.ksplit : p.ksplit;
  p.TH = (p.H + 3) / 4;
  p.TW = (p.W + 3) / 4;
  p.T = p.B * p.TH * p.TW;
  p.TG = (p.T + 15) / 16;
  p.KC = p.C / 16;
  p.order = c.order;
  const size_t vfl = (size_t)p.TG * 16 * p.C * 36;
  if (vfl * 4 >= 0x7fffffffu || (size_t)(p.N / 16) * p.KC * 36 * 1024 >= 0x7fffffffu) return hipErrorInvalidValue;
  if (!p.ws) return hipErrorInvalidValue;
  p.v = p.ws;
  float* slabs = p.ws + vfl;
  // channels per thread of the input transform: the widest loads that still give ~8 waves per CU
  const long units = (long)p.TG * p.KC;
  int cpt = units * 64 >= 2048L * 64 ? 4 : (units * 128 >= 2048L * 64 ? 2 : 1);
  if (const char* e = getenv("ADAPT_W4S_CPT")) cpt = atoi(e);
  if (cpt == 4) hipLaunchKernelGGL(wino4s_in_kernel<4>, dim3((unsigned)((units + 3) / 4)), dim3(256), 0, s, p);
  else if (cpt == 2) hipLaunchKernelGGL(wino4s_in_kernel<2>, dim3((unsigned)((units + 1) / 2)), dim3(256), 0, s, p);
  else hipLaunchKernelGGL(wino4s_in_kernel<1>, dim3((unsigned)units), dim3(256), 0, s, p);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  Wino4sParams q = p;
  q.ws = slabs;
  switch (cfg) {
    case 220: case 224: e = launch_gemm<2, 2, 6, 4>(q, s); break;
    case 221: e = launch_gemm<2, 2, 6, 3>(q, s); break;
    case 227: e = launch_gemm<2, 2, 4, 4>(q, s); break;
    case 228: case 229: e = launch_gemm<4, 2, 4, 4>(q, s); break;
    case 230: case 231: e = launch_gemm<2, 2, 12, 3>(q, s); break;
    case 232: e = launch_gemm<2, 2, 4, 4, true>(q, s); break;
    case 233: e = launch_gemm<2, 2, 6, 3, true>(q, s); break;
    case 234: e = launch_gemm<2, 2, 6, 4, true>(q, s); break;
    case 235: e = launch_gemm<2, 4, 4, 4, true>(q, s); break;
    case 236: e = launch_gemm<2, 2, 4, 5>(q, s); break;
    case 237: e = launch_gemm<2, 2, 2, 8>(q, s); break;
    case 299: e = launch_gemm<2, 2, 6, 3, false, true>(q, s); break;
    case 222: e = launch_gemm<1, 2, 6, 4>(q, s); break;
    case 223: e = launch_gemm<2, 4, 4, 4>(q, s); break;
    case 225: e = launch_gemm<2, 1, 6, 4>(q, s); break;
    case 226: e = launch_gemm<1, 1, 9, 4>(q, s); break;
    default: return hipErrorInvalidValue;
  }
  if (e != hipSuccess || p.ksplit == 1 || fused) return e;
  const long total = (long)p.T * 16 * (p.N / 4);
  const dim3 grid((unsigned)((total + 255) / 256));
  const char* rk = getenv("ADAPT_W4S_REDUCE");
  const bool generic = (rk && rk[0] == '0') || (size_t)p.TG * 256 * (p.N / 4) * p.ksplit >= 0xffffffffu;
  if (!generic && p.ksplit == 2) hipLaunchKernelGGL(wino4s_reduce_ks_kernel<2>, grid, dim3(256), 0, s, q);
  else if (!generic && p.ksplit == 4) hipLaunchKernelGGL(wino4s_reduce_ks_kernel<4>, grid, dim3(256), 0, s, q);
  else if (!generic && p.ksplit == 8) hipLaunchKernelGGL(wino4s_reduce_ks_kernel<8>, grid, dim3(256), 0, s, q);
  else hipLaunchKernelGGL(wino4s_reduce_kernel, grid, dim3(256), 0, s, q);
  return hipGetLastError();
}

}  // namespace adapt
