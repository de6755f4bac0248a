// fp32 1x1 convolution as a big-tile GEMM on the fp32 matrix cores (v_mfma_f32_16x16x4_f32), cfg ids 300+:
//
//   out[m][n] = act( sum_k X[m][k] * W[n][k] + bias[n] (+ res[m][n]) )      (dual output: merged siblings)
//
// Why another fp32 GEMM: every ResNet-50 bs=32 1x1 is 3.29 GFLOP (21.9 us at the 150 TF/s fp32 MFMA ceiling)
// and the existing kernels run them at 33-42 us: the LDS-DMA ring kernel (conv_f32g.hip) tops out at ~86 TF/s
// whatever its tile (profiles/r5/gemm1x1_bigtiles.log), and the streaming pointwise kernel re-reads the
// activations once per channel group.  The chunk body of this kernel is the one tools/mfma_loop_bench.hip
// measured at 33.4 cycles per MFMA (96 % of the pipe) -- 4 MFMA K-steps per 16-float fragment read, reads of the
// next half while the current half multiplies, one barrier per 32-float K chunk -- fed by an LDS-DMA ring:
//
// * tile BM x BN = (16 MF) x (64 NF): the block's 4 waves (one per SIMD) sit side by side along N, each owning
//   all BM rows x 64 NF columns (MF x NF accumulators, up to 224 AGPRs); MF is chosen per layer so the tile
//   count lands just under a multiple of the 256 CUs (112 / 224-row tiles at ResNet-50 bs=32) instead of
//   splitting K;
// * a K chunk = 32 floats = one 128-byte LDS row per operand row, XOR-swizzled by (row >> 1) & 7 so the 16-row
//   fragment reads (one ds_read_b128 per 4 MFMA K-steps, k = 16 h + 4 q + s) are conflict-free; (BM + BN) / 8
//   LDS-DMA pieces per chunk dealt over the 4 waves, an equal count per wave (padded with duplicate pieces) so
//   the ring's counted vmcnt waits are compile-time constants; rows past M read zeros through an out-of-range
//   buffer offset;
// * epilogue per wave, no block barrier: 64-row groups of its accumulators staged in LDS (ds_write_b32, 2-way
//   at most), read back as 16-byte row segments: bias, residual, ReLU / ReLU6, 16-byte stores (a 64-channel row
//   segment per 16 lanes);
// * ksplit -1: stream-K over 256 blocks (XCD-grouped: consecutive K ranges of a tile run on one XCD, so the
//   partial tiles meet in that XCD's L2); a partial tile goes to a workspace slot (write-through), the last
//   arriving block of the tile adds every slot in block order (deterministic) and runs the epilogue.
// Strided 1x1 (the stride-2 shortcut / first conv of a stage) maps output pixel m to its input pixel per row.
#include "kernels.h"

namespace adapt {

namespace {

constexpr int GS_K = 32;                  // floats per K chunk (one 128-byte LDS row)
constexpr int GS_LDS = 160 * 1024;
constexpr unsigned GS_OOB = 0x80000000u;  // voffset past the descriptor: the DMA writes zeros
constexpr int GS_CPOL_SC1 = 16;
constexpr int GS_EPI_LD = 68;             // epilogue staging row: 64 floats + 4 pad
constexpr int GS_MAXSEG = 16;             // stream-K: most blocks contributing to one tile

template <int MF, int NF>
struct GsShape {
  static constexpr int BM = 16 * MF, BN = 64 * NF;
  static constexpr int ROWS = BM + BN;
  static constexpr int PA = (BM / 8 + 3) / 4, PB = (BN / 8 + 3) / 4;   // A / B pieces per wave and chunk
  static constexpr int PW = PA + PB;
  static constexpr int STAGE = ROWS * 128;
  static constexpr int STAGES = 4 * STAGE <= GS_LDS ? 4 : (3 * STAGE <= GS_LDS ? 3 : 2);
  static constexpr int WAIT = (STAGES - 2) * PW;
  static_assert(BM % 8 == 0 && 2 * STAGE <= GS_LDS, "tile too large for LDS");
  static_assert(WAIT <= 63, "vmcnt range");
  static_assert(4 * 64 * GS_EPI_LD * 4 <= GS_LDS, "epilogue staging");
};

__device__ __forceinline__ int gs_swz(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }

__device__ __forceinline__ unsigned gs_sgpr(unsigned v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ u32x4 gs_desc(const float* base) {
  const unsigned long long a = (unsigned long long)(uintptr_t)base;
  return (u32x4){gs_sgpr((unsigned)a), gs_sgpr((unsigned)(a >> 32)) & 0xffffu, 0x7fffffffu, 0x00020000u};
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t gs_rsrc(const float* base) {
  const unsigned long long a = (unsigned long long)(uintptr_t)base;
  const unsigned long long u = ((unsigned long long)gs_sgpr((unsigned)(a >> 32)) << 32) | gs_sgpr((unsigned)a);
  return __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)u, (short)0, 0x7fffffff, 0x00020000);
}

// one 1 KiB LDS-DMA piece: 16 B per lane at LDS byte address `lds` + 16 lane; M0 set in the same statement
__device__ __forceinline__ void gs_dma(int voff, u32x4 rsrc, int soff, unsigned lds) {
  asm volatile("s_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds" ::"v"(voff), "s"(rsrc),
               "s"(gs_sgpr(soff)), "s"(gs_sgpr(lds))
               : "memory");
}

// measurement only (tools/gemm_f32s_timeline.py): 8 words per wave -- shader clock at start / prologue issued /
// K loop done / epilogue done, wall clock at start and end
__device__ __forceinline__ void gs_stamp(unsigned long long* d, int i) {
  if (d != nullptr && (threadIdx.x & 63) == 0) d[i] = __builtin_amdgcn_s_memtime();
}

// NHWC element offset of input row (output pixel) m of a (possibly strided) 1x1 conv, channel 0
__device__ __forceinline__ long long gs_row_in(const ConvF32Params& p, int m) {
  if (p.stride == 1) return (long long)m * p.Cin;
  const int ohw = p.OH * p.OW;
  const int img = m / ohw, rr = m - img * ohw, oy = rr / p.OW, ox = rr - oy * p.OW;
  return ((long long)(img * p.H + oy * p.stride) * p.W + ox * p.stride) * p.Cin;
}

template <int MF, int NF, int EXP = 0>
struct GsTile {
  using S = GsShape<MF, NF>;
  const ConvF32Params& p;
  char* smem;
  int wave, lane;
  u32x4 xdesc, wdesc;
  int tm = S::BM;                                      // rows a tile owns (tile stride, <= BM): rows past it read zeros
  unsigned long long* dbg = nullptr;

  __device__ GsTile(const ConvF32Params& p_, char* smem_, int wave_, int lane_)
      : p(p_), smem(smem_), wave(wave_), lane(lane_) {
    xdesc = gs_desc(p.x);
    wdesc = gs_desc(p.w);
  }

  // one tile segment: chunks [c0, c1) of tile (m0, n0) accumulated into acc
  __device__ __forceinline__ void run(int m0, int n0, int c0, int c1, f32x4 (&acc)[MF][NF]) {
    const unsigned lds0 = (unsigned)(uintptr_t)smem;
    // this lane's source offsets of its PA activation pieces and PB weight pieces (rows fixed over K): the A and
    // B pieces are dealt out separately, so each issue loop has one fixed descriptor; piece indices clamped (the
    // padding pieces of the last waves reload the last piece: same bytes, same LDS place)
    int voffA[S::PA], voffB[S::PB];
#pragma unroll
    for (int j = 0; j < S::PA; ++j) {
      const int r = min(wave * S::PA + j, S::BM / 8 - 1) * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((r >> 1) & 7);                  // logical 4-float unit this lane fetches
      const int m = m0 + r;
      voffA[j] = (r < tm && m < p.M) ? (int)((gs_row_in(p, m) + c * 4) * 4) : (int)GS_OOB;
    }
#pragma unroll
    for (int j = 0; j < S::PB; ++j) {
      const int rb = min(wave * S::PB + j, S::BN / 8 - 1) * 8 + (lane >> 3);
      const int c = (lane & 7) ^ (((S::BM + rb) >> 1) & 7);
      voffB[j] = ((n0 + rb) * p.Kpad + c * 4) * 4;
    }
    // piece j of this wave's PW (A pieces first, then B); j is a compile-time constant at every call
    auto issue1 = [&](int j, int kc, int stage) {
      const unsigned base = lds0 + stage * S::STAGE;
      if (j < S::PA) gs_dma(voffA[j], xdesc, kc * (GS_K * 4), base + min(wave * S::PA + j, S::BM / 8 - 1) * 1024);
      else
        gs_dma(voffB[j - S::PA], wdesc, kc * (GS_K * 4),
               base + S::BM * 128 + min(wave * S::PB + j - S::PA, S::BN / 8 - 1) * 1024);
    };
    auto issue = [&](int kc, int stage) {
#pragma unroll
      for (int j = 0; j < S::PW; ++j) issue1(j, kc, stage);
    };
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
      for (int j = 0; j < NF; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    const int nk = c1 - c0;
    // prologue: STAGES - 1 chunks in flight (past the segment: reload its last chunk, never read)
#pragma unroll
    for (int s = 0; s < S::STAGES - 1; ++s) issue(c0 + min(s, nk - 1), s);
    const int fi = lane & 15, fq = lane >> 4;
    const int brow0 = S::BM + wave * 16 * NF;       // this wave's NF column fragments
    for (int it = 0; it < nk; ++it) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(S::WAIT) : "memory");
      __builtin_amdgcn_s_barrier();                 // chunk it landed for every wave; stage (it - 1) is free
      asm volatile("" ::: "memory");
      if (it == 0) gs_stamp(dbg, 1);
      const int kn = c0 + min(it + S::STAGES - 1, nk - 1), sn = (it + S::STAGES - 1) % S::STAGES;
      const char* st = smem + (it % S::STAGES) * S::STAGE;
      f32x4 a[2][MF], b[2][NF];
      auto rd = [&](int h, f32x4 (&av)[MF], f32x4 (&bv)[NF]) {
#pragma unroll
        for (int i = 0; i < MF; ++i) av[i] = *(const f32x4*)(st + gs_swz(16 * i + fi, 4 * h + fq));
#pragma unroll
        for (int j = 0; j < NF; ++j) bv[j] = *(const f32x4*)(st + gs_swz(brow0 + 16 * j + fi, 4 * h + fq));
      };
      rd(0, a[0], b[0]);
      rd(1, a[1], b[1]);                            // the second half's fragments under the first half's MFMAs
      // 8 K-steps of MF x NF MFMAs; the next chunk's PW LDS-DMA pieces spread over them (issued between MFMA
      // groups instead of as one burst at the top, where the matrix pipe idled ~100 cycles a piece)
#pragma unroll
      for (int step = 0; step < 8; ++step) {
        const int h = step >> 2, s4 = step & 3;
        if constexpr (!(EXP & 1)) {
#pragma unroll
          for (int j = (step * S::PW) / 8; j < ((step + 1) * S::PW) / 8; ++j) issue1(j, kn, sn);
        }
        if constexpr (EXP & 2) {
          acc[0][0][0] += a[h][MF - 1][s4] + b[h][NF - 1][s4];
        } else {
#pragma unroll
          for (int i = 0; i < MF; ++i)
#pragma unroll
            for (int j = 0; j < NF; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[h][i][s4], b[h][j][s4], acc[i][j], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the tail's reload pieces have landed
    __syncthreads();                                   // every wave is done with the ring
  }
};

// output column n of the GEMM -> destination (dual output: merged sibling convs, n_split % 4 == 0)
__device__ __forceinline__ void gs_finish(const ConvF32Params& p, int m, int n, f32x4 v) {
  v += *(const f32x4*)(p.bias + n);
  const F32Dst d = f32_dst(p, n);
  if (p.res) v += *(const f32x4*)(p.res + (size_t)m * p.N + n);
#pragma unroll
  for (int e = 0; e < 4; ++e) v[e] = act_relu(v[e], d.relu);
  *(f32x4*)(d.base + (size_t)m * d.ld + d.col) = v;
}

// wave-local epilogue: the wave's BM x 16 NF accumulators -> LDS, 64 rows per pass -> 16-byte row segments
// (4 NF lanes per row); emit(m, n, v) for rows < M and columns < N
template <int MF, int NF, typename F>
__device__ __forceinline__ void gs_epilogue(char* smem, int wave, int lane, int m0, int n0w, int M, int N,
                                            const f32x4 (&acc)[MF][NF], F&& emit) {
  constexpr int C4 = 4 * NF;                         // float4 per staged row
  constexpr int RPP = 64 / C4;                       // rows per read-back step
  float* stg = (float*)(smem + wave * 64 * GS_EPI_LD * 4);
  const int fi = lane & 15, fq = lane >> 4;
#pragma unroll
  for (int g = 0; g < (MF + 3) / 4; ++g) {
#pragma unroll
    for (int i = 4 * g; i < 4 * g + 4 && i < MF; ++i)
#pragma unroll
      for (int j = 0; j < NF; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) stg[(16 * (i - 4 * g) + 4 * fq + r) * GS_EPI_LD + 16 * j + fi] = acc[i][j][r];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const int rows = 16 * min(4, MF - 4 * g);
#pragma unroll
    for (int k = 0; k < 64 / RPP; ++k) {
      const int row = RPP * k + lane / C4, c4 = lane % C4;
      const int m = m0 + 64 * g + row, n = n0w + 4 * c4;
      if (row < rows) {
        const f32x4 v = *(const f32x4*)(stg + row * GS_EPI_LD + 4 * c4);
        if (m < M && n < N) emit(m, n, v);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
}

// the final epilogue of a whole-K tile: gs_epilogue's staging, with the lane's bias float4 (one column group
// per lane for the whole tile) loaded once and each 64-row pass's residual float4s issued as one batch before
// the staging writes, so their HBM latency hides under the LDS round trip instead of serialising per store
template <int MF, int NF>
__device__ __forceinline__ void gs_epilogue_direct(const ConvF32Params& p, char* smem, int wave, int lane, int m0,
                                                   int n0w, int mlim, const f32x4 (&acc)[MF][NF]) {
  constexpr int C4 = 4 * NF;
  constexpr int RPP = 64 / C4;
  constexpr int KS = 64 / RPP;
  float* stg = (float*)(smem + wave * 64 * GS_EPI_LD * 4);
  const int fi = lane & 15, fq = lane >> 4;
  const int c4 = lane % C4, n = n0w + 4 * c4;
  const bool nok = n < p.N;
  const f32x4 bv = nok ? *(const f32x4*)(p.bias + n) : (f32x4){0.f, 0.f, 0.f, 0.f};
  const F32Dst d = f32_dst(p, nok ? n : 0);
#pragma unroll
  for (int g = 0; g < (MF + 3) / 4; ++g) {
    const int rows = 16 * min(4, MF - 4 * g);
    f32x4 rv[KS];
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      const int row = RPP * k + lane / C4, m = m0 + 64 * g + row;
      rv[k] = (f32x4){0.f, 0.f, 0.f, 0.f};
      if (p.res && nok && row < rows && m < mlim) rv[k] = *(const f32x4*)(p.res + (size_t)m * p.N + n);
    }
#pragma unroll
    for (int i = 4 * g; i < 4 * g + 4 && i < MF; ++i)
#pragma unroll
      for (int j = 0; j < NF; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) stg[(16 * (i - 4 * g) + 4 * fq + r) * GS_EPI_LD + 16 * j + fi] = acc[i][j][r];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      const int row = RPP * k + lane / C4, m = m0 + 64 * g + row;
      if (row < rows && m < mlim && nok) {
        f32x4 v = *(const f32x4*)(stg + row * GS_EPI_LD + 4 * c4) + bv + rv[k];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = act_relu(v[e], d.relu);
        *(f32x4*)(d.base + (size_t)m * d.ld + d.col) = v;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
}

// EXP (measurement variants, outputs wrong by design): bit 0 no LDS-DMA in the K loop, bit 1 no MFMAs.
// TM: rows a tile owns (0 = BM).  TM < BM places tiles TM rows apart, so the tile count can hit a multiple of
// the 256 CUs (98-row tiles: 6272 rows x 256 / 64 columns = 256 tiles); the BM - TM rows past it read zeros.
template <int MF, int NF, int EXP = 0, int TM = 0>
__global__ __launch_bounds__(256, 1) void gemm_f32s_kernel(ConvF32Params p, unsigned long long* dbg_all) {
  static_assert(NF <= 4, "one 64-column staging pass per wave");
  using S = GsShape<MF, NF>;
  constexpr int TMV = TM ? TM : S::BM;
  static_assert(TMV <= S::BM, "owned rows within the tile");
  __shared__ __attribute__((aligned(16))) char smem[GS_LDS];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tilesN = (p.N + S::BN - 1) / S::BN;
  const int tilesM = (p.M + TMV - 1) / TMV;
  const int KT = p.Kpad / GS_K;
  GsTile<MF, NF, EXP> T(p, smem, wave, lane);
  T.tm = TMV;
  unsigned long long* const dbg = dbg_all ? dbg_all + 8 * (wave + 4 * blockIdx.x) : nullptr;
  T.dbg = dbg;
  gs_stamp(dbg, 0);
  if (dbg && lane == 0) dbg[6] = __builtin_amdgcn_s_memrealtime();
  f32x4 acc[MF][NF];
  if (p.ksplit == 1) {                               // one block per tile, whole K
    const int t = blockIdx.x;
    if (t >= tilesM * tilesN) return;
    const int m0 = (t / tilesN) * TMV, n0 = (t % tilesN) * S::BN;
    T.run(m0, n0, 0, KT, acc);
    gs_stamp(dbg, 2);
    gs_epilogue_direct<MF, NF>(p, smem, wave, lane, m0, n0 + 16 * NF * wave, min(p.M, m0 + TMV), acc);
    if (dbg) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      gs_stamp(dbg, 3);
      if (lane == 0) dbg[7] = __builtin_amdgcn_s_memrealtime();
    }
    return;
  }
  // stream-K: G blocks split the T x KT (tile, chunk) units into equal contiguous ranges; block b runs range
  // v = (b % 8) * (G / 8) + b / 8, so the ranges of one XCD are contiguous
  const int G = gridDim.x;
  const int b = blockIdx.x;
  const int v = (b & 7) * (G >> 3) + (b >> 3);
  const long long U = (long long)tilesM * tilesN * KT;
  const long long u0 = (long long)v * U / G, u1 = (long long)(v + 1) * U / G;
  const size_t tile_elems = (size_t)S::BM * S::BN;
  const __amdgpu_buffer_rsrc_t wsr = gs_rsrc(p.ws);
  int* const flag = (int*)(smem + GS_LDS - 16);
  auto vof = [&](long long u) { return (int)(((u + 1) * G - 1) / U); };      // block whose range holds unit u
  for (long long u = u0; u < u1;) {
    const int t = (int)(u / KT);
    const int c0 = (int)(u - (long long)t * KT);
    const int c1 = (int)min((long long)KT, c0 + (u1 - u));
    const int m0 = (t / tilesN) * TMV, n0 = (t % tilesN) * S::BN;
    const int mlim = min(p.M, m0 + TMV);
    T.run(m0, n0, c0, c1, acc);
    const int n0w = n0 + 16 * NF * wave;
    if (c0 == 0 && c1 == KT) {
      gs_epilogue_direct<MF, NF>(p, smem, wave, lane, m0, n0w, mlim, acc);
      __syncthreads();                               // the staging is free before the next segment's DMA
    } else {
      // partial: this block's slot (2v for its first segment, 2v + 1 for a later one), written through L2
      const int slot = 2 * v + (u == u0 ? 0 : 1);
      gs_epilogue<MF, NF>(smem, wave, lane, m0, n0w, mlim, p.N, acc, [&](int m, int n, f32x4 val) {
        const int off = (int)(((size_t)slot * tile_elems + (size_t)(m - m0) * S::BN + (n - n0)) * 4);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, val), wsr, off, 0, GS_CPOL_SC1);
      });
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      const long long ut0 = (long long)t * KT;
      const int vf = vof(ut0), vl = vof(ut0 + KT - 1);
      if (threadIdx.x == 0) {
        const int old = __hip_atomic_fetch_add(p.counters + t, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = old == vl - vf;
        if (last) __hip_atomic_store(p.counters + t, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *flag = last;
      }
      __syncthreads();
      if (*flag) {
        // the tile's partial slots in block order: block w's segment here is its first (slot 2w) unless it
        // began in an earlier tile (2w + 1); at most GS_MAXSEG contributors (host check)
        int sls[GS_MAXSEG];
#pragma unroll
        for (int k = 0; k < GS_MAXSEG; ++k) {
          const int w = min(vf + k, vl);
          sls[k] = 2 * w + ((long long)w * U / G >= ut0 ? 0 : 1);
        }
        const int nseg = vl - vf + 1;
        for (int idx = threadIdx.x; idx < S::BM * (S::BN / 4); idx += 256) {
          const int row = idx / (S::BN / 4), c4 = idx - row * (S::BN / 4);
          const int m = m0 + row, n = n0 + 4 * c4;
          if (m >= mlim || n >= p.N) continue;
          f32x4 acc4 = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int k = 0; k < GS_MAXSEG; ++k) {
            if (k >= nseg) break;
            const int off = (int)(((size_t)sls[k] * tile_elems + (size_t)row * S::BN + 4 * c4) * 4);
            acc4 += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(wsr, off, 0, GS_CPOL_SC1));
          }
          gs_finish(p, m, n, acc4);
        }
      }
      __syncthreads();                               // the flag and the staging are free again
    }
    u += c1 - c0;
  }
}

static unsigned long long* g_gs_dbg = nullptr;
static int g_gs_exp = 0;

template <int MF, int NF, int TM>
hipError_t gs_launch(const ConvF32Params& p, hipStream_t s) {
  using S = GsShape<MF, NF>;
  constexpr int TMV = TM ? TM : S::BM;
  const int tiles = ((p.M + TMV - 1) / TMV) * ((p.N + S::BN - 1) / S::BN);
  int grid = tiles;
  if (p.ksplit < 0) {
    if (TM) return hipErrorInvalidValue;             // stream-K only with whole BM-row tiles
    grid = 256;
    if ((long long)tiles * (p.Kpad / GS_K) < grid || !p.ws || !p.counters) return hipErrorInvalidValue;
    if ((size_t)2 * grid * S::BM * S::BN * 4 > 0x7fffffffu) return hipErrorInvalidValue;
    // a tile's K range spans at most GS_MAXSEG blocks: ceil(KT / floor(units per block)) + 1
    const long long U = (long long)tiles * (p.Kpad / GS_K);
    const long long per = U / grid;
    if (per < 1 || (p.Kpad / GS_K + per - 1) / per + 1 > GS_MAXSEG) return hipErrorInvalidValue;
  }
  switch (g_gs_exp) {
    case 0: hipLaunchKernelGGL((gemm_f32s_kernel<MF, NF, 0, TM>), dim3(grid), dim3(256), 0, s, p, g_gs_dbg); break;
    case 1: hipLaunchKernelGGL((gemm_f32s_kernel<MF, NF, 1, TM>), dim3(grid), dim3(256), 0, s, p, g_gs_dbg); break;
    case 2: hipLaunchKernelGGL((gemm_f32s_kernel<MF, NF, 2, TM>), dim3(grid), dim3(256), 0, s, p, g_gs_dbg); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace

// cfg -> (MF, NF, TM): tile (16 MF) x (64 NF), TM owned rows (0 = 16 MF); ops/conv.py F32S_CFGS mirrors this
// (307 / 308 / 309: 98- / 98- / 49-row tiles on the ResNet-50 bs=32 K-heavy 1x1s, 256 tiles each: 6272 x 256,
// 1568 x 2048 and 1568 x 512)
// (301 / 303-306, the other whole-row tiles, were never picked in-graph and are no longer built; 300 / 302 keep
// the whole-row and stream-K paths tested)
#define ADAPT_F32S_CFGS(X) \
  X(300, 7, 4, 0)          \
  X(302, 7, 2, 0)          \
  X(307, 7, 1, 98)         \
  X(308, 7, 2, 98)         \
  X(309, 4, 1, 49)

void gemm_f32s_set_debug(unsigned long long* buf, int exp) {
  g_gs_dbg = buf;
  g_gs_exp = exp;
}

bool gemm_f32s_cfg(int cfg, int* bm, int* bn) {
  switch (cfg) {
#define X(id, MF_, NF_, TM_)     \
  case id:                       \
    *bm = TM_ ? TM_ : 16 * MF_;  \
    *bn = 64 * NF_;              \
    return true;
    ADAPT_F32S_CFGS(X)
#undef X
  }
  return false;
}

// stream-K workspace (floats) and counters of a cfg-300+ launch with ksplit -1
size_t gemm_f32s_ws_elems(int cfg) {
  switch (cfg) {
#define X(id, MF_, NF_, TM_) \
  case id:                   \
    return (size_t)2 * 256 * (16 * MF_) * (64 * NF_);
    ADAPT_F32S_CFGS(X)
#undef X
  }
  return 0;
}

hipError_t gemm_f32s_launch(const ConvF32Params& p, int cfg, hipStream_t s) {
  if (p.KH != 1 || p.KW != 1 || p.pad_t != 0 || p.pad_l != 0 || (p.stride != 1 && p.stride != 2) ||
      p.Cin % GS_K || p.Kpad != p.Cin || p.N % 16 || (p.ksplit != 1 && p.ksplit != -1))
    return hipErrorInvalidValue;
  if ((long long)p.B * p.H * p.W * p.Cin * 4 >= 0x7fffffffLL) return hipErrorInvalidValue;   // 31-bit offsets
  int bm = 0, bn = 0;
  if (!gemm_f32s_cfg(cfg, &bm, &bn)) return hipErrorInvalidValue;
  if ((long long)((p.N + bn - 1) / bn * bn) * p.Kpad * 4 >= 0x7fffffffLL) return hipErrorInvalidValue;
  switch (cfg) {
#define X(id, MF_, NF_, TM_) \
  case id: return gs_launch<MF_, NF_, TM_>(p, s);
    ADAPT_F32S_CFGS(X)
#undef X
  }
  return hipErrorInvalidValue;
}

}  // namespace adapt
