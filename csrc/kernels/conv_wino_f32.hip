// fp32 3x3 / stride-1 / pad-1 convolution by Winograd F(2x2, 3x3) on the fp32
// matrix cores (v_mfma_f32_16x16x4_f32), transforms fused: one launch reads
// the NHWC input and writes the NHWC output (BN folded, bias, ReLU).
//
// Why: at fp32 every ResNet 3x3 conv is matrix-bound (the fp32 MFMA runs at
// 1/16 of the bf16 rate) and the direct implicit-GEMM kernels (conv_f32g.hip)
// spend 76-86 us per layer at ~97 TF/s (tools/conv_bench_f32.py).  F(2x2, 3x3)
// computes each 2x2 output tile from a 4x4 input patch with 16 multiplies per
// (cin, cout) instead of 36: 2.25x less matrix work.  All arithmetic stays
// fp32 (the input / output transforms use only +/-1 coefficients, the weight
// transform's 1/2 factors are exact and done on the host in fp64), which is
// the algorithm cuDNN applies to float32 3x3 convs under TensorFlow -- the
// reference's Keras model (`/root/reference/test/test.py:13`, float32).
//
//   V_p[t][c] = (B^T d_t,c B)_p     (d = the 4x4 input patch of tile t, p = 0..15)
//   M_p[t][n] = sum_c V_p[t][c] U_p[c][n]          U = G g G^T  (host)
//   y_t[n]    = A^T M[t][n] A + bias[n]   (2x2 outputs)
//
// Block = NWM waves; wave w owns 16 tiles (the MFMA rows) x 16*FN output
// channels x all 16 positions (acc 64*FN VGPRs).  K walks the input channels
// in chunks of 16: MFMA step s of a chunk takes channel 4q+s from lane group q
// (the K permutation of conv_f32g.hip), so
//   * a lane's share of the input patch is 16 float4 loads (its tile, its 4
//     channels), transformed in registers -- no LDS, the A operand never exists
//     as a matrix;
//   * the transformed weights are host-packed in MFMA fragment order
//     ([chunk][n-frag][p][lane][4]) and streamed into an LDS ring by LDS-DMA,
//     one contiguous 16*FN KiB run per chunk per block, read back with
//     conflict-free lane-linear ds_read_b128 (one per (p, n-frag) per chunk).
// The accumulator layout puts all 16 positions of (tile, channel) in one lane,
// so the output transform is lane-local: no shuffle, no LDS round trip.
// Split-K (gridDim.z) writes the transformed partial outputs to fp32 slabs
// (linear, so A^T (sum M) A = sum A^T M A); splitk_reduce_f32 adds bias / ReLU,
// or (fused split-K, p.counters) the last split of each output tile does.
#include "kernels.h"

namespace adapt {

namespace {

typedef __attribute__((address_space(3))) void lds_void_w;

__device__ __attribute__((aligned(64))) float g_wino_zero[256];   // 1 KiB: a whole dummy DMA piece

constexpr int WINO_CPOL_SC1 = 16;   // gfx950 cache policy: sc1 (write-through L2, bypass L1)

// floor(a / b) for 0 <= a < 2^20 and 1 <= b < 2^12, with rb = 1.0f / b correctly rounded:
// (a + 1/2) / b lies at least 1/(2b) away from an integer and the float product errs by at
// most a * 2^-23 / b, so the truncation is exact.  Replaces the ~25-VALU integer division
// sequence the index math of a block's prologue and epilogue otherwise runs once per piece
// and per tile (a C = 64 layer has only 4 K chunks to amortise it over).
__device__ __forceinline__ int wino_div(int a, float rb) { return (int)(((float)a + 0.5f) * rb); }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t wino_ws_rsrc(const float* base) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, 0x7fffffff, 0x00020000);
}

// LDS-DMA of one 1 KiB piece (16 B per lane, lane-linear at lds_dst) issued from inline asm, so the
// compiler does not see it.  Its wait-count model counts an LDS DMA as an LDS access as well as a vector
// memory access; with one in flight no LDS wait can be partial and every wait in the chunk loop is
// lgkmcnt(0) -- a group waits on the reads it issued for later groups too.  Hidden, the DMA needs the
// explicit vmcnt waits the v3 body already has (before the patch reads, before each chunk barrier).
// M0 (the LDS base of the DMA) is set here; nothing else in these kernels reads M0.
__device__ __forceinline__ void wino_dma16(const void* src, void* lds_dst) {
  const unsigned m = (unsigned)(uintptr_t)lds_dst;
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(m) : "memory");
}

// fused split-K, last split of a block: out = act(sum_z slab_z + bias (+ res)) in split order, with
// this split's own partials from registers; all (S - 1) x 4 x FN x 4 slab loads issue before the sum
template <int FN, int S>
__device__ __forceinline__ void wino_fixup(const WinoF32Params& p, const float (&yk)[4][FN][4], const int (&ok)[4],
                                           int tw0, int r, int q, int nf0, __amdgpu_buffer_rsrc_t wsr, int MN, int zs,
                                           int ns) {
  const int tpi = p.TH * p.TW;
  float ld[S][4][FN][4];
  const float rtpi = 1.0f / (float)tpi, rtw = 1.0f / (float)p.TW;
  int oys[4], oxs[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int tt = tw0 + 4 * q + i;
    const int rr = tt - wino_div(tt, rtpi) * tpi;
    const int ry = wino_div(rr, rtw);
    oys[i] = 2 * ry;
    oxs[i] = 2 * (rr - ry * p.TW);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int oy = oys[i], ox = oxs[i];
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int dy = k >> 1, dx = k & 1;
        const bool in = ok[i] >= 0 && oy + dy < p.H && ox + dx < p.W;
        const int o = ok[i] + (dy * p.W + dx) * p.N + (nf0 + j) * 16 + r;
#pragma unroll
        for (int z = 0; z < S; ++z)
          ld[z][i][j][k] = (in && z < ns && z != zs)
                               ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                               wsr, (z * MN + o) * 4, 0, WINO_CPOL_SC1))
                               : 0.f;
      }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (ok[i] < 0) continue;
    const int oy = oys[i], ox = oxs[i];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = (nf0 + j) * 16 + r;
      const float bn = p.bias[n];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int dy = k >> 1, dx = k & 1;
        if (oy + dy >= p.H || ox + dx >= p.W) continue;
        const int o = ok[i] + (dy * p.W + dx) * p.N + n;
        float v = 0.f;
#pragma unroll
        for (int z = 0; z < S; ++z)
          if (z < ns) v += z == zs ? yk[i][j][k] : ld[z][i][j][k];
        v += bn;
        if (p.res) v += p.res[o];
        p.out[o] = act_relu(v, p.relu);
      }
    }
  }
}

// output transform A^T M A (lane-local) + bias / residual / ReLU, or a split-K slab (blockIdx.z);
// acc[p][j][i] = M_p[tile tw0 + 4q + i][channel 16 (nf0 + j) + r]
//
// Fused split-K (p.counters set, cfgs with ksplit < 0 on the host): every split stores its
// transformed partial outputs to its slab with sc1 stores, one lane counts the arrival of the
// (tile group, channel group), and the last split to arrive re-reads the others' slabs (sc1) in
// split order -- deterministic, whoever is last -- and runs the epilogue: no splitk_reduce_f32
// launch.  Nobody waits on anybody, so the grid never needs to be co-resident.
template <int FN, int ABL>
__device__ __forceinline__ void wino_epilogue(const WinoF32Params& p, const f32x4 (&acc)[16][FN], int tw0, int r,
                                              int q, int nf0, int* flag, int zs, int ns, int ctr_idx,
                                              char* stage = nullptr, unsigned long long* dbg = nullptr) {
  // zs / ns: this partial's slab index / the partials of its output block (ns == 1: whole K);
  // fused fixup when the host passed arrival counters, else slab ws[zs] for splitk_reduce_f32
  const bool split = ns > 1;
  if (stage != nullptr && (!split || p.counters != nullptr)) {
    // Whole-K output through the wave's own LDS image (free after its last patch read): the
    // accumulator layout puts 16 channels of a pixel in 16 lanes, which the plain path stores as
    // 4-byte scattered writes (32 store instructions per lane at FN = 2); transposed through LDS, a
    // lane stores 16 contiguous bytes (4 FN dwordx4 per lane), with bias / residual / ReLU applied on
    // the float4.  Runs: (tile of the wave 0..15, pixel 0..3) x 16 FN channels.
    constexpr int RUN = 16 * FN;                        // floats per (tile, pixel) run
    float* st = (float*)stage;
    // FN = 2: the float4 column of a run is XORed with 4 on odd lane groups (runs 16..31, 48..63), so a
    // staging write's four lane groups, which land on rows 16 apart (same banks), split over both halves
    // of the 32 banks: 2-way instead of 4-way conflicts; the read-back applies the same XOR per run
    // the bias quad of this lane ((16 q + r) % (4 FN) = r % (4 FN)), loaded first so its L2 round trip
    // runs under the staging; the opaque index keeps the load below the K loop
    int bidx = nf0 * 16 + (r % (4 * FN)) * 4;
    asm volatile("" : "+v"(bidx));
    const f32x4 bsv = *(const f32x4*)(p.bias + bidx);
    const int swq = FN == 2 ? 4 * (q & 1) : 0;
    auto swr = [&](int run) { return FN == 2 ? 4 * ((run >> 4) & 1) : 0; };
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int tl = 4 * q + i;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        float m[4][4];
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int b = 0; b < 4; ++b) m[a][b] = acc[a * 4 + b][j][i];
        float w0[4], w1[4];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          w0[b] = m[0][b] + m[1][b] + m[2][b];
          w1[b] = m[1][b] - m[2][b] - m[3][b];
        }
        const int cw = ((((j * 16 + r) >> 2) ^ swq) << 2) | (r & 3);
        st[(tl * 4 + 0) * RUN + cw] = w0[0] + w0[1] + w0[2];
        st[(tl * 4 + 1) * RUN + cw] = w0[1] - w0[2] - w0[3];
        st[(tl * 4 + 2) * RUN + cw] = w1[0] + w1[1] + w1[2];
        st[(tl * 4 + 3) * RUN + cw] = w1[1] - w1[2] - w1[3];
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // wave-private region: LDS is in order per wave
    if (dbg) dbg[8] = __builtin_amdgcn_s_memtime();      // staged (tools/wino_timeline.py)
    // opaque copies: keep the store-phase index math from being hoisted above the K loop, where its
    // registers would be live beside the accumulators (the FN = 2 kernels sit at 250+ VGPRs)
    int lane = q * 16 + r;
    asm volatile("" : "+v"(lane));
    const int tpi = p.TH * p.TW;
    const float rtpi = 1.0f / (float)tpi, rtw = 1.0f / (float)p.TW;
    int oo[4 * FN];                                     // NHWC offset of each float4 this lane owns (-1: outside)
#pragma unroll
    for (int it = 0; it < 4 * FN; ++it) {
      const int g = it * 64 + lane;                     // float4 index in the wave's 64 runs
      const int run = g / (4 * FN), part = g - run * (4 * FN);
      const int tl = run >> 2, px = run & 3;
      const int tt = tw0 + tl;
      const int im = wino_div(tt, rtpi), rr = tt - im * tpi;
      const int ry = wino_div(rr, rtw);
      const int oy = 2 * ry + (px >> 1), ox = 2 * (rr - ry * p.TW) + (px & 1);
      oo[it] = (tt < p.T && oy < p.H && ox < p.W) ? ((im * p.H + oy) * p.W + ox) * p.N + nf0 * 16 + part * 4 : -1;
    }
    auto own = [&](int it) -> f32x4 {
      const int g = it * 64 + lane;
      const int run = g / (4 * FN);
      return *(const f32x4*)(st + run * RUN + ((g % (4 * FN)) ^ swr(run)) * 4);
    };
    // a lane's channel quad is the same for every float4 it owns (64 runs per pass, 4 FN quads per run),
    // so the bias is one load (above); the LDS reads and residual loads of all passes issue before the
    // first store -- inside the per-pass `oo >= 0` branches each would wait out its own latency in turn
    auto finish = [&](int it, f32x4 v, f32x4 rv) {
      const int o = oo[it];
      v += bsv;
      if (p.res) v += rv;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = act_relu(v[e], p.relu);
      if constexpr (ABL & 4) asm volatile("" ::"v"(v));
      else *(f32x4*)(p.out + o) = v;
    };
    f32x4 rvs[4 * FN];
#pragma unroll
    for (int it = 0; it < 4 * FN; ++it)
      rvs[it] = p.res ? *(const f32x4*)(p.res + max(oo[it], 0)) : (f32x4){0.f, 0.f, 0.f, 0.f};
    if (!split) {
      f32x4 ov[4 * FN];
#pragma unroll
      for (int it = 0; it < 4 * FN; ++it) ov[it] = own(it);
      if (dbg) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        dbg[9] = __builtin_amdgcn_s_memtime();           // offsets computed, staged values read back
      }
#pragma unroll
      for (int it = 0; it < 4 * FN; ++it)
        if (oo[it] >= 0) finish(it, ov[it], rvs[it]);
      if (dbg) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        dbg[10] = __builtin_amdgcn_s_memtime();          // stores done
      }
      return;
    }
    // fused split-K: every split publishes its partial outputs as 16-byte sc1 stores to its slab; the
    // last split of the output block (arrival counter) adds the slabs in split order -- the same sums,
    // in the same order, as the per-element path and splitk_reduce_f32 -- then bias / residual / ReLU
    const int MN = p.B * p.H * p.W * p.N;
    const __amdgpu_buffer_rsrc_t wsr = wino_ws_rsrc(p.ws);
#pragma unroll
    for (int it = 0; it < 4 * FN; ++it)
      if (oo[it] >= 0)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, own(it)), wsr, (zs * MN + oo[it]) * 4, 0,
                                               WINO_CPOL_SC1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      int* ctr = p.counters + ctr_idx;
      const int old = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = old == ns - 1;
      if (last) __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = last;
    }
    __syncthreads();
    if (!*flag) return;
    // two passes' slab loads in flight at a time (all eight would hold 128 VGPRs of slabs)
#pragma unroll
    for (int it0 = 0; it0 < 4 * FN; it0 += 2) {
      f32x4 sl[2][4];
#pragma unroll
      for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int z = 0; z < 4; ++z)
          sl[k][z] = (z < ns && z != zs)
                         ? __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                         wsr, (z * MN + max(oo[it0 + k], 0)) * 4, 0, WINO_CPOL_SC1))
                         : (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int it = it0 + k;
        const f32x4 mine = own(it);
        f32x4 v = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int z = 0; z < 4; ++z)
          if (z < ns) v += z == zs ? mine : sl[k][z];
        if (oo[it] >= 0) finish(it, v, rvs[it]);
      }
    }
    return;
  }
  const bool fused = split && p.counters != nullptr;
  float* dst = split ? p.ws + (size_t)zs * p.B * p.H * p.W * p.N : p.out;
  const int tpi = p.TH * p.TW;
  const int MN = p.B * p.H * p.W * p.N;
  const __amdgpu_buffer_rsrc_t wsr = wino_ws_rsrc(p.ws);
  float yk[4][FN][4];                                 // fused: this split's partial outputs
  int ok[4];                                          // their NHWC offsets at channel 0 (-1: outside)
  const float rtpi = 1.0f / (float)tpi, rtw = 1.0f / (float)p.TW;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int tt = tw0 + 4 * q + i;
    ok[i] = -1;
    if (tt >= p.T) continue;
    const int im = wino_div(tt, rtpi), rr = tt - im * tpi;
    const int ry = wino_div(rr, rtw);
    const int oy = 2 * ry, ox = 2 * (rr - ry * p.TW);
    ok[i] = ((im * p.H + oy) * p.W + ox) * p.N;
    const bool iny = oy + 1 < p.H, inx = ox + 1 < p.W;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = (nf0 + j) * 16 + r;
      float m[4][4];
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) m[a][b] = acc[a * 4 + b][j][i];
      float w0[4], w1[4];
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        w0[b] = m[0][b] + m[1][b] + m[2][b];
        w1[b] = m[1][b] - m[2][b] - m[3][b];
      }
      float y[2][2];
      y[0][0] = w0[0] + w0[1] + w0[2];
      y[0][1] = w0[1] - w0[2] - w0[3];
      y[1][0] = w1[0] + w1[1] + w1[2];
      y[1][1] = w1[1] - w1[2] - w1[3];
      const float bn = split ? 0.f : p.bias[n];
#pragma unroll
      for (int dy = 0; dy < 2; ++dy)
#pragma unroll
        for (int dx = 0; dx < 2; ++dx) {
          if ((dy && !iny) || (dx && !inx)) continue;
          const int o = ok[i] + (dy * p.W + dx) * p.N + n;
          float v = y[dy][dx] + bn;
          if (fused) {
            yk[i][j][dy * 2 + dx] = v;
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), wsr,
                                                  (int)((zs * (size_t)MN + o) * 4), 0, WINO_CPOL_SC1);
            continue;
          }
          if (!split) {
            if (p.res) v += p.res[o];
            v = act_relu(v, p.relu);
          }
          if constexpr (ABL & 4) asm volatile("" ::"v"(v));
          else dst[(size_t)o] = v;
        }
    }
  }
  if (!fused) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    int* ctr = p.counters + ctr_idx;
    const int old = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == ns - 1;
    if (last) __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = last;
  }
  __syncthreads();
  if (!*flag) return;                                // (a stream-K block's next segment starts with a barrier
                                                      // before its DMA can reuse the flag's LDS word)
  if (ns == 2) wino_fixup<FN, 2>(p, yk, ok, tw0, r, q, nf0, wsr, MN, zs, ns);   // other slabs' loads in flight
  else wino_fixup<FN, 4>(p, yk, ok, tw0, r, q, nf0, wsr, MN, zs, ns);           // together (3 or 4)
}

// two waves per SIMD (<= 256 VGPRs) up to FN = 2 without prefetch; FN = 3 (192 accumulators) or the
// register prefetch of the next chunk's patch (64 more VGPRs) keep one
template <int NWM, int FN, bool PF>
constexpr int wino_min_blocks() {
  return (FN <= 2 && !PF) ? (8 / NWM > 0 ? 8 / NWM : 1) : (4 / NWM > 0 ? 4 / NWM : 1);
}

// ABL: ablation switches for the cfg 90+ twins of cfg 80 (tools/conv_bench_f32.py; 0 in production):
// 1 = every patch load from one address (no scattered loads), 2 = no MFMA, 4 = no output stores,
// 8 = no weight DMA
// PF: the next chunk's patch loads are issued into a second register set right after the chunk's
// barrier, so they are in flight under the chunk's MFMAs instead of exposed at the next chunk's start.
template <int NWM, int FN, int STAGES, bool PF, int ABL = 0>
__global__ __launch_bounds__(NWM * 64, (wino_min_blocks<NWM, FN, PF>())) void conv_wino_f32_kernel(WinoF32Params p) {
  constexpr int NT = NWM * 64;
  constexpr int BT = 16 * NWM;                       // tiles per block
  constexpr int PIECES = 16 * FN;                    // 1 KiB weight pieces per chunk
  constexpr int PPW = (PIECES + NWM - 1) / NWM;      // pieces per wave
  constexpr int SLOT = PIECES * 1024;
  __shared__ __attribute__((aligned(16))) char ring[STAGES * SLOT];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 15, q = lane >> 4;
  const int nf0 = blockIdx.y * FN;                   // first 16-channel output fragment
  const int NF = p.N / 16;
  const int KC = p.C / 16;                           // 16-channel chunks
  const int kper = (KC + p.ksplit - 1) / p.ksplit;
  const int kc0 = blockIdx.z * kper, kc1 = min(KC, kc0 + kper);

  // ---- this lane's tile (A row r of the wave) and its 4x4 input patch
  const int t = blockIdx.x * BT + wave * 16 + r;
  const int tpi = p.TH * p.TW;
  const bool tok = t < p.T;
  const int img = tok ? t / tpi : 0;
  const int tr = tok ? t - img * tpi : 0;
  const int ty = tr / p.TW, tx = tr - ty * p.TW;
  const int iy0 = 2 * ty - 1, ix0 = 2 * tx - 1;
  unsigned ok = 0;                                   // bit 4*dy + dx: patch pixel inside the image
#pragma unroll
  for (int dy = 0; dy < 4; ++dy)
#pragma unroll
    for (int dx = 0; dx < 4; ++dx)
      if (tok && (unsigned)(iy0 + dy) < (unsigned)p.H && (unsigned)(ix0 + dx) < (unsigned)p.W) ok |= 1u << (4 * dy + dx);
  const float* xb = p.x + (((ptrdiff_t)img * p.H + iy0) * p.W + ix0) * p.C + 4 * q;
  const ptrdiff_t rstride = (ptrdiff_t)p.W * p.C;

  // ---- weight pieces of chunk kc -> ring slot
  const float* ub = p.u + (size_t)nf0 * 16 * 256;    // 256 floats per piece
  const size_t uchunk = (size_t)NF * 16 * 256;
  auto issue_w = [&](int kc, int slot) {
    const float* src = ub + (size_t)kc * uchunk;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int pc = wave * PPW + i;
      if (PIECES % NWM == 0 || pc < PIECES)
        __builtin_amdgcn_global_load_lds((const void*)(src + pc * 256 + lane * 4),
                                         (lds_void_w*)(ring + slot * SLOT + pc * 1024), 16, 0, 0);
    }
  };

  f32x4 acc[16][FN];
#pragma unroll
  for (int i = 0; i < 16; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // this lane's patch, channels 16kc + 4q .. +3 (zero outside the image)
  auto load_patch = [&](f32x4 (&dd)[4][4], int kc) {
#pragma unroll
    for (int dy = 0; dy < 4; ++dy)
#pragma unroll
      for (int dx = 0; dx < 4; ++dx) {
        const float* src = (!(ABL & 1) && (!PF || kc < kc1) && ((ok >> (4 * dy + dx)) & 1u))
                               ? xb + dy * rstride + dx * p.C + kc * 16 : g_wino_zero;
        dd[dy][dx] = *(const f32x4*)src;
      }
  };
  f32x4 dn[PF ? 4 : 1][PF ? 4 : 1];
  if (!(ABL & 8) && kc0 < kc1) issue_w(kc0, 0);
  if constexpr (PF) load_patch(dn, kc0);
  for (int kc = kc0; kc < kc1; ++kc) {
    const int slot = (kc - kc0) % STAGES;
    f32x4 d[4][4];
    if constexpr (PF) {
#pragma unroll
      for (int dy = 0; dy < 4; ++dy)
#pragma unroll
        for (int dx = 0; dx < 4; ++dx) d[dy][dx] = dn[dy][dx];
    } else {
      load_patch(d, kc);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();                    // every wave's pieces of chunk kc are in; slot kc+1 is free
    asm volatile("" ::: "memory");
    if (!(ABL & 8) && kc + 1 < kc1) issue_w(kc + 1, (slot + 1) % STAGES);
    if constexpr (PF) load_patch(dn, kc + 1);

    // B^T d: rows
#pragma unroll
    for (int dx = 0; dx < 4; ++dx) {
      const f32x4 a0 = d[0][dx], a1 = d[1][dx], a2 = d[2][dx], a3 = d[3][dx];
      d[0][dx] = a0 - a2;
      d[1][dx] = a1 + a2;
      d[2][dx] = a2 - a1;
      d[3][dx] = a1 - a3;
    }
    const char* sl = ring + slot * SLOT;
#pragma unroll
    for (int pa = 0; pa < 4; ++pa) {
      // (B^T d B)[pa][0..3] for this lane's 4 channels
      f32x4 v[4];
      v[0] = d[pa][0] - d[pa][2];
      v[1] = d[pa][1] + d[pa][2];
      v[2] = d[pa][2] - d[pa][1];
      v[3] = d[pa][1] - d[pa][3];
#pragma unroll
      for (int pb = 0; pb < 4; ++pb) {
        f32x4 u[FN];
#pragma unroll
        for (int j = 0; j < FN; ++j) u[j] = *(const f32x4*)(sl + ((j * 16 + pa * 4 + pb) * 64 + lane) * 16);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            if constexpr (ABL & 2) acc[pa * 4 + pb][j][s] += v[pb][s] * u[j][s];
            else acc[pa * 4 + pb][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(v[pb][s], u[j][s], acc[pa * 4 + pb][j], 0, 0, 0);
          }
      }
    }
  }

  wino_epilogue<FN, ABL>(p, acc, blockIdx.x * BT + wave * 16, r, q, nf0, (int*)ring, blockIdx.z, p.ksplit,
                        blockIdx.x + gridDim.x * blockIdx.y);
}

// ---------------------------------------------------------------------------
// v2: the wave's input patches staged in LDS by LDS-DMA (cfg 100+).
//
// The v1 ablation (tools/conv_bench_f32.py, cfgs 90-99) put the cost in the
// per-lane patch loads: 16 scattered float4 loads per lane per chunk, waited on
// right away (stage-3 3x3: 65 us, 41 us without them).  Here a wave's 16 tiles
// (16 consecutive tiles in (image, tile row, tile column) order, as in v1) form
// at most four row segments; a segment of `len` tiles needs 4 input rows x
// (2 len + 2) pixels, so the wave's input is <= 160 pixels instead of 256, and
// it is fetched as whole 64-byte pixel chunks (16 channels) by LDS-DMA into the
// wave's own LDS image.  Each lane then reads its 16 patch pixels with
// ds_read_b128 at the start of the chunk and the wave immediately refills the
// same image with the next chunk (only this wave reads it, so no barrier is
// needed), which keeps the next chunk's input in flight under this chunk's
// MFMAs without a second register set.  The weight ring is as in v1.
//
// SW (cfgs 103-105): the wave image is bank-swizzled.  Unswizzled, quad q of
// pixel P sits in 16-B slot 4P + q, i.e. at position 4(P & 3) + q of its 256-B
// bank row; consecutive tiles are 2 pixels apart, so a ds_read_b128 lane group
// ({0-3,12-15,20-27}, ...) lands on 4 positions: 4-way conflicts, 256 LDS cycles
// per wave per chunk for the 16 patch reads (329 at stage 4).  With SW the
// position is XORed with h(row) = (2 row + 8 (row >> 2)) & 15, row = slot >> 4
// (a bijection inside each bank row; the LDS-DMA lanes fetch the inverse-mapped
// pixel / quad, since a DMA piece lands lane-linear): 73 / 110 / 142 / 64 cycles
// for stages 2-5 (tools/wino_swizzle_search.py, exhaustive over that family).
__device__ __forceinline__ int wino_sw(int slot) {
  const int row = slot >> 4;
  return slot ^ ((2 * row + 8 * (row >> 2)) & 15);
}

// EP (cfgs 106-108): each wave reads the next chunk's patch from its image right after its own
// MFMAs of this chunk (its LDS-DMA has had the whole chunk to land), before the chunk barrier,
// instead of every wave reading its patch right after the barrier while no MFMA runs.
template <int NW, int FN>
struct WinoV2Shape {
  static constexpr int PMAX = 10;                    // 1 KiB input pieces per wave (<= 160 pixels)
  static constexpr int PIECES = 16 * FN;
  static constexpr int PPW = (PIECES + NW - 1) / NW;
  static constexpr int SLOT = PIECES * 1024;
  static constexpr int LDS = 2 * SLOT + NW * PMAX * 1024;
  static constexpr int CTR = LDS;                    // + 64 B: the counter-synchronised body's 4 counters (cfg 171)
};

// one (tile group tg, channel group cg, K chunks [kc0, kc1)) unit of work; zs / ns / ctr_idx: its partial's
// slab, the partials of its output block and their arrival counter (ns == 1: whole K, plain epilogue)
template <int NW, int FN, bool SW, bool EP, int PL = 0>
__device__ __forceinline__ void wino_v2_unit(const WinoF32Params& p, char* smem, int tg, int cg, int kc0, int kc1,
                                             int zs, int ns, int ctr_idx) {
  using S = WinoV2Shape<NW, FN>;
  constexpr int PMAX = S::PMAX, PIECES = S::PIECES, PPW = S::PPW, SLOT = S::SLOT;
  char* ring = smem;
  // opaque thread index: in the stream-K loop (several units per block) everything derived from the
  // lane would otherwise be hoisted out of the loop and held beside the accumulators (128 VGPRs spilled)
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
  const int lane = tid & 63;
  // the dummy DMA source's address, materialised once: referenced inside the chunk loop, the symbol is
  // re-loaded from the GOT by an s_load there every chunk, and a scalar load in flight (it returns out of
  // order) turns every LDS wait of the loop into lgkmcnt(0) -- no group could wait on just its older reads
  const float* wzero = g_wino_zero;
  asm volatile("" : "+s"(wzero));
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 15, q = lane >> 4;
  char* pimg = smem + 2 * SLOT + wave * PMAX * 1024;
  const int nf0 = cg * FN;
  const int NF = p.N / 16;
  const int TR = p.B * p.TH;                         // tile rows over the batch

  // ---- the wave's row segments (wave-uniform)
  const float rtw = 1.0f / (float)p.TW, rth = 1.0f / (float)p.TH;
  const int tw0 = (tg * NW + wave) * 16;
  const int tlast = min(tw0 + 15, p.T - 1);
  const int R0 = wino_div(tw0, rtw);
  const int nseg = tw0 < p.T ? wino_div(tlast, rtw) - R0 + 1 : 0;
  int seg_lo[4], seg_w[4], seg_b[5];
  float seg_rw[4];
  seg_b[0] = 0;
#pragma unroll
  for (int sg = 0; sg < 4; ++sg) {
    const int lo = sg == 0 ? tw0 - R0 * p.TW : 0;
    const int hi = sg == nseg - 1 ? tlast - (R0 + sg) * p.TW : p.TW - 1;
    seg_lo[sg] = lo;
    seg_w[sg] = sg < nseg ? 2 * (hi - lo + 1) + 2 : 0;
    seg_rw[sg] = sg < nseg ? 1.0f / (float)seg_w[sg] : 0.f;
    seg_b[sg + 1] = seg_b[sg] + 4 * seg_w[sg];
  }

  // ---- LDS-DMA sources: piece i, lane l -> image pixel (element offset), chunk-invariant
  int src_off[PMAX];
  unsigned src_ok = 0;
#pragma unroll
  for (int i = 0; i < PMAX; ++i) {
    const int sl = SW ? wino_sw(i * 64 + lane) : i * 64 + lane;   // the slot this lane's DMA fills holds
    const int pix = sl >> 2, qq = sl & 3;                          // (pixel, quad); wino_sw is an involution
    int sg = 0;
#pragma unroll
    for (int k = 1; k < 4; ++k) sg += pix >= seg_b[k] ? 1 : 0;
    const int wdt = sg == 0 ? seg_w[0] : sg == 1 ? seg_w[1] : sg == 2 ? seg_w[2] : seg_w[3];
    const float rw = sg == 0 ? seg_rw[0] : sg == 1 ? seg_rw[1] : sg == 2 ? seg_rw[2] : seg_rw[3];
    const int lo = sg == 0 ? seg_lo[0] : 0;
    const int bb = sg == 0 ? seg_b[0] : sg == 1 ? seg_b[1] : sg == 2 ? seg_b[2] : seg_b[3];
    const int lp = pix - bb;
    const int prow = (wdt && lp >= 0) ? wino_div(lp, rw) : 0, pcol = lp - prow * wdt;
    const int R = R0 + sg;
    const int img = wino_div(R, rth), ty = R - img * p.TH;
    const int iy = 2 * ty - 1 + prow, ix = 2 * lo - 1 + pcol;
    const bool in = pix < seg_b[4] && R < TR && (unsigned)iy < (unsigned)p.H &&
                    (unsigned)ix < (unsigned)p.W;
    src_off[i] = in ? ((img * p.H + iy) * p.W + ix) * p.C + 4 * qq : 0;
    src_ok |= in ? 1u << i : 0u;
  }
  auto issue_x = [&](int kc) {
#pragma unroll
    for (int i = 0; i < PMAX; ++i) {
      const float* src = ((src_ok >> i) & 1u) ? p.x + src_off[i] + kc * 16 : wzero;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void_w*)(pimg + i * 1024), 16, 0, 0);
    }
  };

  // ---- this lane's patch in the wave image: pixel index of (dy, dx) = prow0 + dy * pw + dx
  const int t = tw0 + r;
  const int tsg = t < p.T ? wino_div(t, rtw) - R0 : 0;
  const int pw = tsg == 0 ? seg_w[0] : tsg == 1 ? seg_w[1] : tsg == 2 ? seg_w[2] : seg_w[3];
  const int pb0 = tsg == 0 ? seg_b[0] : tsg == 1 ? seg_b[1] : tsg == 2 ? seg_b[2] : seg_b[3];
  const int plo = tsg == 0 ? seg_lo[0] : 0;
  const int prow0 = t < p.T ? pb0 + 2 * (t - (R0 + tsg) * p.TW - plo) : 0;
  const int ps0 = prow0 * 4 + q;                     // slot of patch pixel (0, 0)
  const char* prd = pimg + ps0 * 16;
  const int pws = pw * 64;                           // bytes per patch-row step

  const float* ub = p.u + (size_t)nf0 * 16 * 256;
  const size_t uchunk = (size_t)NF * 16 * 256;
  auto issue_w = [&](int kc, int slot) {
    const float* src = ub + (size_t)kc * uchunk;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int pc = wave * PPW + i;
      if (PIECES % NW == 0 || pc < PIECES)
        __builtin_amdgcn_global_load_lds((const void*)(src + pc * 256 + lane * 4),
                                         (lds_void_w*)(ring + slot * SLOT + pc * 1024), 16, 0, 0);
    }
  };

  f32x4 acc[16][FN];
#pragma unroll
  for (int i = 0; i < 16; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  f32x4 d[4][4];
  auto read_patch = [&]() {
#pragma unroll
    for (int dy = 0; dy < 4; ++dy)
#pragma unroll
      for (int dx = 0; dx < 4; ++dx) {
        if constexpr (SW) d[dy][dx] = *(const f32x4*)(pimg + wino_sw(ps0 + dy * pw * 4 + dx * 4) * 16);
        else d[dy][dx] = *(const f32x4*)(prd + dy * pws + dx * 64);
      }
  };
  if constexpr (PL != 0) {
    constexpr int PLM = PL & 7;                      // chunk body; PL & 8 / 16: stagger / priority (below)
    // phase stamps (tools/wino_timeline.py), 16 words per block: shader clock at unit start / first chunk
    // landed / loop end / epilogue end, the 100 MHz wall clock at start and end, HW_ID and XCC_ID, and
    // inside a whole-K epilogue: staged / read back / stores done; thread 0 only, vector stores
    unsigned long long* const dbg =
        p.dbg ? p.dbg + 16 * (blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z)) : nullptr;
    const bool stamp = dbg && threadIdx.x == 0;
    if (stamp) {
      dbg[0] = __builtin_amdgcn_s_memtime();
      dbg[4] = __builtin_amdgcn_s_memrealtime();
      dbg[6] = (unsigned)__builtin_amdgcn_s_getreg(0xF804);       // HW_ID
      dbg[7] = (unsigned)__builtin_amdgcn_s_getreg(0x7814);       // XCC_ID
    }
    // v3 (cfgs 116-117, FN = 1; PL = 2, cfgs 118-119: FN = 2 with only the DMA spread): one basic block per
    // chunk, software-pipelined.
    //  * the 16 (pa, pb) MFMA groups each read the NEXT group's weight fragments (FN ds_read_b128) ahead
    //    of their own MFMAs, so an LDS read latency is never exposed right before the MFMA that needs it
    //    (v2: `R R R R lgkmcnt(0) M...` eight times per chunk);
    //  * the next chunk's LDS-DMA pieces (PPW weight pieces, then PMAX input pieces) are spread one per
    //    group instead of 14 back to back after the barrier, where both waves of a SIMD issued them at
    //    once and left the matrix core idle;
    //  * FN = 1: two groups' accumulation chains alternate (a dependent 16x16x4 f32 MFMA waits 40 of its
    //    32 issue cycles);
    //  * the next chunk's patch is read at the end of the chunk (as EP), unconditionally: the last chunk
    //    reads / DMAs a harmless dummy, so nothing in the loop branches.
    f32x4 d[4][4];
    auto read_patch_pl = [&]() {
#pragma unroll
      for (int dy = 0; dy < 4; ++dy)
#pragma unroll
        for (int dx = 0; dx < 4; ++dx) d[dy][dx] = *(const f32x4*)(pimg + wino_sw(ps0 + dy * pw * 4 + dx * 4) * 16);
    };
    f32x4 acc[16][FN];
#pragma unroll
    for (int i = 0; i < 16; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    // PL & 16: the second half of the waves (each SIMD's younger partner) at priority 1 for the whole
    // loop; PL & 8: it starts every chunk ~128 cycles late, so the two partners' LDS waits stop
    // coinciding (the two waves of a SIMD run the same program in lock step from each barrier,
    // MI355X_MICROARCH.md "two waves per SIMD", items 4 and 9)
    if constexpr ((PL & 16) != 0) {
      if (wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
    }
    constexpr bool OD = (PL & 32) != 0;             // DMA through wino_dma16 (cfgs 164-167)
    // PL & 128 (cfg 171): no block barrier per chunk.  The two-slot weight ring is guarded by LDS
    // counters instead -- wready[s]: waves whose weight pieces for slot s have landed, rdone[s]: waves done
    // reading slot s -- so a wave waits only for the data it needs and the waves of a block may drift up
    // to ~6 MFMA groups apart (the block barrier held every wave to the slowest: 0.9 us a chunk,
    // profiles/r4/r4v).  Inputs go out in groups 0-4, weights in 5-8 (after rdone of their slot), and
    // wready is raised at group 14 after this wave's vmcnt(0).  Every spin is bounded.
    constexpr bool CS = (PL & 128) != 0;
    int* const wready = (int*)(smem + S::CTR);
    int* const rdone = wready + 2;
    // the counter accesses are inline asm: as plain LDS accesses the compiler cannot tell them from the
    // LDS-DMA destinations and puts a vmcnt(0) before each, i.e. waits for the DMA just issued
    auto spin_ge = [&](int* c, int target) {
      const unsigned a = (unsigned)(uintptr_t)c;
      for (int it = 0; it < (1 << 22); ++it) {
        int v;
        asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
        if (__builtin_amdgcn_readfirstlane(v) >= target) break;
        __builtin_amdgcn_s_sleep(1);
      }
    };
    auto bump = [&](int* c) {
      const unsigned a = (unsigned)(uintptr_t)c;
      if (lane == 0) asm volatile("ds_add_u32 %0, %1" ::"v"(a), "v"(1) : "memory");
    };
    if constexpr (CS) {
      if (threadIdx.x < 4) wready[threadIdx.x] = 0;
      __syncthreads();
    }
    if (kc0 < kc1) {
      if constexpr (OD) {
        const float* src = ub + (size_t)kc0 * uchunk;
#pragma unroll
        for (int i = 0; i < PPW; ++i) {
          const int pc = wave * PPW + i;
          if (PIECES % NW == 0 || pc < PIECES) wino_dma16(src + pc * 256 + lane * 4, ring + pc * 1024);
        }
#pragma unroll
        for (int i = 0; i < PMAX; ++i)
          wino_dma16(((src_ok >> i) & 1u) ? p.x + src_off[i] + kc0 * 16 : wzero, pimg + i * 1024);
      } else {
        issue_w(kc0, 0);
        issue_x(kc0);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if constexpr (CS) bump(&wready[0]);          // chunk kc0's weight pieces of this wave are in
      read_patch_pl();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    if (stamp) dbg[1] = __builtin_amdgcn_s_memtime();
    for (int kc = kc0; kc < kc1; ++kc) {
      const int slot = (kc - kc0) & 1;
      // PL & 64 (measurement-only cfg 170): thread 0 stamps chunk kc0 + 2: before / after its barrier,
      // at group 8, after group 15's MFMAs issue, after the next patch has been read (words 11-15)
      constexpr bool TM = (PL & 64) != 0;
      const bool tmc = TM && stamp && kc == kc0 + 2;
      if (tmc) dbg[11] = __builtin_amdgcn_s_memtime();
      const int n = kc - kc0;                        // chunk index within the unit; its ring slot is n & 1
      if constexpr (CS) spin_ge(&wready[n & 1], 8 * (n / 2 + 1) * NW / 8);
      else __builtin_amdgcn_s_barrier();             // every wave's weight pieces of chunk kc are in
      asm volatile("" ::: "memory");
      if (tmc) dbg[12] = __builtin_amdgcn_s_memtime();
      if constexpr ((PL & 8) != 0) {
        if (wave >= NW / 2) __builtin_amdgcn_s_sleep(2);
      }
      const bool more = kc + 1 < kc1;
      const float* wsrc = more ? ub + (size_t)(kc + 1) * uchunk : wzero;
      const int wstep = more ? 256 : 0;              // the dummy piece: one 1 KiB buffer for every piece
      char* wdst = ring + (slot ^ 1) * SLOT;
      // B^T d: rows, in place
#pragma unroll
      for (int dx = 0; dx < 4; ++dx) {
        const f32x4 a0 = d[0][dx], a1 = d[1][dx], a2 = d[2][dx], a3 = d[3][dx];
        d[0][dx] = a0 - a2;
        d[1][dx] = a1 + a2;
        d[2][dx] = a2 - a1;
        d[3][dx] = a1 - a3;
      }
      const char* sl = ring + slot * SLOT;
      constexpr bool PFR = PLM == 1;                  // fragments of group g+1 read ahead of g's MFMAs
      // DMA pieces per group: PL >= 3 front-loads the next chunk's pieces (PL - 1 per group), so the
      // last one has most of the chunk to land instead of the last two groups (cfgs 150-153)
      // PLM 6 (cfgs 162/163): the DMA front-loaded 2 per group (done by group 6) and the next chunk's
      // patch rows 0-2 read during groups 12-15, into the registers of this chunk's rows 0-2 (dead after
      // group 11): the chunk end waits only on row 3's four reads instead of the DMA tail plus 16 reads
      constexpr bool EPR = PLM == 6;
      constexpr int DPG = (PLM == 3 || PLM == 4) ? PLM - 1 : EPR ? 2 : 1;
      constexpr int NPG = (PPW + PMAX + DPG - 1) / DPG;   // groups that issue DMA
      constexpr int NB = !PFR ? 1 : FN >= 2 ? 2 : 4; // FN = 1 pairs groups: g-1's fragments must survive g's read
      f32x4 u[NB][FN];
      // PLM 5 (FN = 2, cfgs 160/161): half prefetch -- the next group's j = 0 fragment is read during this
      // group, its j = 1 fragment at the group's start behind the four j = 0 MFMAs: 4 more VGPRs instead
      // of the 8 of a full prefetch (which spills at FN = 2), and no group waits on its first read
      constexpr bool HP = PLM == 5;
      static_assert(!HP || FN == 2, "half prefetch is for FN = 2");
      f32x4 un = {0.f, 0.f, 0.f, 0.f};
      if constexpr (HP) un = *(const f32x4*)(sl + ((0 * 16 + 0) * 64 + lane) * 16);
      if constexpr (PFR) {
#pragma unroll
        for (int j = 0; j < FN; ++j) u[0][j] = *(const f32x4*)(sl + ((j * 16 + 0) * 64 + lane) * 16);
      }
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int pa = g >> 2, pb = g & 3;
        if (TM && g == 8 && tmc) dbg[13] = __builtin_amdgcn_s_memtime();
        if (pb == 0) {                               // (B^T d B)[pa][*], in place over row pa
          const f32x4 e0 = d[pa][0], e1 = d[pa][1], e2 = d[pa][2], e3 = d[pa][3];
          d[pa][0] = e0 - e2;
          d[pa][1] = e1 + e2;
          d[pa][2] = e2 - e1;
          d[pa][3] = e1 - e3;
        }
        f32x4 u0h = {0.f, 0.f, 0.f, 0.f}, u1h = {0.f, 0.f, 0.f, 0.f};
        if constexpr (HP) {
          u0h = un;
          u1h = *(const f32x4*)(sl + ((1 * 16 + g) * 64 + lane) * 16);
          if (g < 15) un = *(const f32x4*)(sl + ((0 * 16 + g + 1) * 64 + lane) * 16);
        } else if constexpr (PFR) {
          if (g < 15) {
#pragma unroll
            for (int j = 0; j < FN; ++j)
              u[(g + 1) % NB][j] = *(const f32x4*)(sl + ((j * 16 + g + 1) * 64 + lane) * 16);
          }
        } else {
#pragma unroll
          for (int j = 0; j < FN; ++j) u[0][j] = *(const f32x4*)(sl + ((j * 16 + g) * 64 + lane) * 16);
          if constexpr (EPR) {
            // next patch rows 0-2, three reads a group in groups 12-15, issued right after the group's own
            // fragment reads so the group waits on its fragments only (LDS returns in order)
            if (g >= 12) {
              if (g == 12) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the input DMA (done by group 6)
#pragma unroll
              for (int rr = 3 * (g - 12); rr < 3 * (g - 12) + 3; ++rr) {
                const int dy = rr >> 2, dx = rr & 3;
                d[dy][dx] = *(const f32x4*)(pimg + wino_sw(ps0 + dy * pw * 4 + dx * 4) * 16);
              }
            }
          }
        }
        if constexpr (CS) {
          if (g < 5) {                               // next chunk's input pieces 2g, 2g+1 (own image: no hazard)
#pragma unroll
            for (int i = 2 * g; i < 2 * g + 2; ++i) {
              if (i >= PMAX) continue;
              const float* src = (more && ((src_ok >> i) & 1u)) ? p.x + src_off[i] + (kc + 1) * 16 : wzero;
              __builtin_amdgcn_global_load_lds((const void*)src, (lds_void_w*)(pimg + i * 1024), 16, 0, 0);
            }
          } else if (g < 5 + PPW && more) {          // next chunk's weight piece g - 5, once the slot is free
            if (g == 5) spin_ge(&rdone[(n + 1) & 1], 8 * ((n + 1) / 2) * NW / 8);
            const int pc = wave * PPW + (g - 5);
            if (PIECES % NW == 0 || pc < PIECES)
              __builtin_amdgcn_global_load_lds((const void*)(wsrc + pc * wstep + lane * 4),
                                               (lds_void_w*)(wdst + pc * 1024), 16, 0, 0);
          }
          if (g == 14) {                             // every DMA of this wave issued by group 8 has landed
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            bump(&wready[(n + 1) & 1]);
          }
        } else {
#pragma unroll
        for (int pi = g * DPG; pi < (g + 1) * DPG; ++pi) {
          if (pi < PPW) {                            // next chunk's weight piece pi of this wave
            const int pc = wave * PPW + pi;
            if (PIECES % NW == 0 || pc < PIECES) {
              if constexpr (OD) wino_dma16(wsrc + pc * wstep + lane * 4, wdst + pc * 1024);
              else __builtin_amdgcn_global_load_lds((const void*)(wsrc + pc * wstep + lane * 4),
                                                    (lds_void_w*)(wdst + pc * 1024), 16, 0, 0);
            }
          } else if (pi - PPW < PMAX) {              // next chunk's input piece
            const int i = pi - PPW;
            const float* src = (more && ((src_ok >> i) & 1u)) ? p.x + src_off[i] + (kc + 1) * 16 : wzero;
            if constexpr (OD) wino_dma16(src, pimg + i * 1024);
            else __builtin_amdgcn_global_load_lds((const void*)src, (lds_void_w*)(pimg + i * 1024), 16, 0, 0);
          }
        }
        }
        // fence: the next fragments' reads and the DMA piece issue above this group's MFMAs (left to
        // itself the scheduler sinks each prefetch next to its use, at ~250 VGPRs, and waits lgkmcnt(0))
        if constexpr (PFR || HP) __builtin_amdgcn_sched_barrier(0);
        const f32x4 vv = d[pa][pb];
        if constexpr (HP) {
#pragma unroll
          for (int ss = 0; ss < 4; ++ss)
            acc[g][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(vv[ss], u0h[ss], acc[g][0], 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);         // the prefetched half first: nothing waits on u1h yet
#pragma unroll
          for (int ss = 0; ss < 4; ++ss)
            acc[g][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(vv[ss], u1h[ss], acc[g][1], 0, 0, 0);
        } else if constexpr (!PFR) {
#pragma unroll
          for (int ss = 0; ss < 4; ++ss)
#pragma unroll
            for (int j = 0; j < FN; ++j)
              acc[g][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(vv[ss], u[0][j][ss], acc[g][j], 0, 0, 0);
          // this group: its fragment reads (+ EPR's patch reads), its DMA piece, then its MFMAs
          if (EPR && g >= 12) __builtin_amdgcn_sched_group_barrier(0x100, FN + 3, 0);
          else __builtin_amdgcn_sched_group_barrier(0x100, FN, 0);
          if constexpr (CS) {
            if (g < 5) __builtin_amdgcn_sched_group_barrier(0x010, 2, 0);
            else if (g < 5 + PPW) __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);
          } else {
            if (g < NPG - 1) __builtin_amdgcn_sched_group_barrier(0x010, DPG, 0);
            else if (g == NPG - 1) __builtin_amdgcn_sched_group_barrier(0x010, PPW + PMAX - (NPG - 1) * DPG, 0);
          }
          __builtin_amdgcn_sched_group_barrier(0x008, 4 * FN, 0);
        } else if constexpr (FN >= 2) {
#pragma unroll
          for (int ss = 0; ss < 4; ++ss)
#pragma unroll
            for (int j = 0; j < FN; ++j)
              acc[g][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(vv[ss], u[g % NB][j][ss], acc[g][j], 0, 0, 0);
        } else if ((g & 1) == 1) {                   // FN = 1: groups g-1 and g alternate their chains
          const f32x4 vp = d[pa][pb - 1];
#pragma unroll
          for (int ss = 0; ss < 4; ++ss) {
            acc[g - 1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(vp[ss], u[(g - 1) % NB][0][ss], acc[g - 1][0], 0, 0,
                                                                 0);
            acc[g][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(vv[ss], u[g % NB][0][ss], acc[g][0], 0, 0, 0);
          }
        }
      }
      if constexpr (CS) bump(&rdone[n & 1]);       // this wave is done reading slot n & 1
      if (tmc) dbg[14] = __builtin_amdgcn_s_memtime();
      // the next chunk's patch (its DMA went out during this chunk's groups)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if constexpr (PLM == 6) {
#pragma unroll
        for (int dx = 0; dx < 4; ++dx) d[3][dx] = *(const f32x4*)(pimg + wino_sw(ps0 + 3 * pw * 4 + dx * 4) * 16);
      } else {
        read_patch_pl();
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (tmc) dbg[15] = __builtin_amdgcn_s_memtime();
    }
    if (stamp) dbg[2] = __builtin_amdgcn_s_memtime();
    wino_epilogue<FN, 0>(p, acc, tw0, r, q, nf0, (int*)smem, zs, ns, ctr_idx, pimg, stamp ? dbg : nullptr);
    if (stamp) {
      dbg[3] = __builtin_amdgcn_s_memtime();
      dbg[5] = __builtin_amdgcn_s_memrealtime();
    }
    return;
  }
  if (kc0 < kc1) {
    issue_w(kc0, 0);
    issue_x(kc0);
    if constexpr (EP) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      read_patch();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  }
  for (int kc = kc0; kc < kc1; ++kc) {
    const int slot = (kc - kc0) & 1;
    if constexpr (!EP) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();                    // all weight pieces of chunk kc in; the other slot is free
    asm volatile("" ::: "memory");
    if (kc + 1 < kc1) issue_w(kc + 1, slot ^ 1);
    if constexpr (!EP) {
      read_patch();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    if (kc + 1 < kc1) issue_x(kc + 1);               // this wave's image is free again: refill it

#pragma unroll
    for (int dx = 0; dx < 4; ++dx) {
      const f32x4 a0 = d[0][dx], a1 = d[1][dx], a2 = d[2][dx], a3 = d[3][dx];
      d[0][dx] = a0 - a2;
      d[1][dx] = a1 + a2;
      d[2][dx] = a2 - a1;
      d[3][dx] = a1 - a3;
    }
    const char* sl = ring + slot * SLOT;
#pragma unroll
    for (int pa = 0; pa < 4; ++pa) {
      f32x4 v[4];
      v[0] = d[pa][0] - d[pa][2];
      v[1] = d[pa][1] + d[pa][2];
      v[2] = d[pa][2] - d[pa][1];
      v[3] = d[pa][1] - d[pa][3];
#pragma unroll
      for (int pb = 0; pb < 4; ++pb) {
        f32x4 u[FN];
#pragma unroll
        for (int j = 0; j < FN; ++j) u[j] = *(const f32x4*)(sl + ((j * 16 + pa * 4 + pb) * 64 + lane) * 16);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[pa * 4 + pb][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(v[pb][s], u[j][s], acc[pa * 4 + pb][j], 0, 0, 0);
      }
    }
    if constexpr (EP) {
      // the next chunk's patch, read while the other waves still run this chunk's MFMAs: the
      // barrier no longer releases every wave into the same LDS burst
      if (kc + 1 < kc1) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        read_patch();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
    }
  }
  // the fused split-K arrival flag lives in the ring (dead after the loop): a second __shared__ object
  // makes the compiler's LDS-DMA alias tracking put a vmcnt(0) between every chunk's weight DMA issue
  // and the patch reads, which serialises the whole prefetch
  if (!EP) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no DMA may still be landing in the image
  wino_epilogue<FN, 0>(p, acc, tw0, r, q, nf0, (int*)smem, zs, ns, ctr_idx, pimg);
}

// Stream-K (p.sk_iters > 0, cfgs 103-108 with ksplit <= -100 on the host): a 1-D grid of about
// (-ksplit - 100) x 256 blocks, each taking sk_iters consecutive (unit, K-chunk) iterations of the
// units x KC space (unit = channel group major, tile group minor).  A ResNet 3x3 has 196-400 units of
// 4-16 chunks, i.e. 0.77-1.53 rounds of the 256 CUs: the last partial round idled 23-50 % of the chip.
// Partial units meet through the fused fixup (deterministic, segment order).
// XM (cfgs 130-132): XCD-aware block order.  Blocks are dispatched round-robin over the 8 XCDs, each
// with its own 4 MiB L2, so with the plain grid every XCD fetches every tile group's input and every
// channel group's weights from the Infinity Cache.  Here the physical block id is remapped so XCD k
// runs one contiguous logical range, and that range is a 2-D patch: one half of the channel groups x
// a quarter of the tile groups -- per chunk step an input line is fetched by 2 L2s and a weight line
// by 4, instead of by all 8.
__device__ __forceinline__ void wino_xcd_unit(int& tg, int& cg, int& z) {
  const int gx = gridDim.x, gy = gridDim.y, plane = gx * gy;
  const int total = plane * gridDim.z;
  const int phys = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  const int lg = xcd_remap(phys, total);
  z = lg / plane;
  const int rem = lg - z * plane;
  const int h0 = (gy + 1) / 2, h1 = gy - h0;
  if (rem < gx * h0) {
    tg = rem / h0;
    cg = rem - tg * h0;
  } else {
    const int r2 = rem - gx * h0;
    tg = r2 / h1;
    cg = h0 + (r2 - tg * h1);
  }
}

template <int NW, int FN, bool SW = false, bool EP = false, bool SK = false, int PL = 0, bool XM = false>
__global__ __launch_bounds__(NW * 64, (NW == 4 && FN == 1) ? 2 : 1) void conv_wino_f32_v2_kernel(WinoF32Params p) {
  __shared__ __attribute__((aligned(16))) char smem[WinoV2Shape<NW, FN>::LDS + ((PL & 128) ? 64 : 0)];
  const int KC = p.C / 16;
  if constexpr (!SK) {
    int tg = blockIdx.x, cg = blockIdx.y, z = blockIdx.z;
    if constexpr (XM) wino_xcd_unit(tg, cg, z);
    const int kper = (KC + p.ksplit - 1) / p.ksplit;
    const int kc0 = z * kper;
    wino_v2_unit<NW, FN, SW, EP, PL>(p, smem, tg, cg, kc0, min(KC, kc0 + kper), z, p.ksplit, tg + gridDim.x * cg);
    return;
  }
  if constexpr (PL != 0) {
    // stream-K over the v3 chunk body: the host keeps sk_iters <= KC, so a block's range meets at most
    // two units; the two calls are straight-line code (a loop around the inlined unit kept values of
    // one unit live through the next one's MFMAs: 128 VGPRs spilled)
    const int gx = (p.T + 16 * NW - 1) / (16 * NW);
    const int iters = p.sk_iters;
    const int it0 = blockIdx.x * iters;
    const int it_end = min(gx * (p.N / (16 * FN)) * KC, it0 + iters);
    auto seg = [&](int it) {
      const int u = it / KC;
      const int kb = it - u * KC;
      const int ke = min(KC, kb + (it_end - it));
      int zs = 0, ns = 1;
      if (kb != 0 || ke != KC) {
        const int g_first = (u * KC) / iters, g_last = ((u + 1) * KC - 1) / iters;
        zs = blockIdx.x - g_first;
        ns = g_last - g_first + 1;
      }
      wino_v2_unit<NW, FN, SW, EP, PL>(p, smem, u % gx, u / gx, kb, ke, zs, ns, u);
      return it + (ke - kb);
    };
    const int it1 = seg(it0);
    if (it1 < it_end) {
      __syncthreads();                               // the first unit's ring / flag / images are dead
      seg(it1);
    }
    return;
  }
  const bool sk = SK;
  const int gx = (p.T + 16 * NW - 1) / (16 * NW);
  const int iters = p.sk_iters;
  int it = sk ? blockIdx.x * iters : 0;
  const int it_end = sk ? min(gx * (p.N / (16 * FN)) * KC, it + iters) : 1;
  while (it < it_end) {                              // one pass in grid mode: a single call site
    int tg, cg, kb, ke, zs, ns, ctr;
    if (!sk) {
      const int kper = (KC + p.ksplit - 1) / p.ksplit;
      tg = blockIdx.x;
      cg = blockIdx.y;
      kb = blockIdx.z * kper;
      ke = min(KC, kb + kper);
      zs = blockIdx.z;
      ns = p.ksplit;
      ctr = blockIdx.x + gridDim.x * blockIdx.y;
    } else {
      const int u = it / KC;
      kb = it - u * KC;
      ke = min(KC, kb + (it_end - it));
      tg = u % gx;
      cg = u / gx;
      ctr = u;
      zs = 0;
      ns = 1;
      if (kb != 0 || ke != KC) {
        const int g_first = (u * KC) / iters, g_last = ((u + 1) * KC - 1) / iters;
        zs = blockIdx.x - g_first;
        ns = g_last - g_first + 1;
      }
      __syncthreads();                               // the previous segment's ring / flag / images are dead
    }
    wino_v2_unit<NW, FN, SW, EP, PL>(p, smem, tg, cg, kb, ke, zs, ns, ctr);
    it = sk ? it + (ke - kb) : it_end;
  }
}

// v2 needs every wave's 16 tiles in <= 4 row segments (<= 160 input pixels)
bool wino_v2_shape_ok(int TW) { return TW >= 5 || TW == 4; }

// ---------------------------------------------------------------------------
// Persistent v2 (cfgs 140 / 141): a grid of two blocks per CU walks the (tile group, channel group) units
// u = blockIdx.x, + gridDim.x, ... as ONE flattened chunk stream.  The non-persistent grid pays, per round
// of blocks, the first chunk's load burst (every block's weights and wave images at once, nothing to
// overlap) and an exposed epilogue -- about 10 us a round, a third of the stage-2 layer
// (profiles/r4/wino_vs_cin.log: 19.5 us + 9.8 us per chunk at 56x56x64).  Here the DMA of the next unit's
// first chunk (its weights, its wave images from its own row-segment geometry) goes out under the
// current unit's last chunk, and the current unit's output transform and 16-byte stores (staged in the
// wave image, which the next unit's first patch has just left) run while the CU's other block keeps
// the matrix cores busy.  Whole units per block: no partial sums, no fixup.
struct WinoGeom {
  int src_off[10];
  unsigned src_ok;
  int ps0, pw, tw0;
};

template <int NW>
__device__ __forceinline__ void wino_geom(const WinoF32Params& p, int tg, int wave, int lane, WinoGeom& G) {
  const int r = lane & 15, q = lane >> 4;
  const int TR = p.B * p.TH;
  const float rtw = 1.0f / (float)p.TW, rth = 1.0f / (float)p.TH;
  const int tw0 = (tg * NW + wave) * 16;
  const int tlast = min(tw0 + 15, p.T - 1);
  const int R0 = wino_div(tw0, rtw);
  const int nseg = tw0 < p.T ? wino_div(tlast, rtw) - R0 + 1 : 0;
  int seg_lo[4], seg_w[4], seg_b[5];
  float seg_rw[4];
  seg_b[0] = 0;
#pragma unroll
  for (int sg = 0; sg < 4; ++sg) {
    const int lo = sg == 0 ? tw0 - R0 * p.TW : 0;
    const int hi = sg == nseg - 1 ? tlast - (R0 + sg) * p.TW : p.TW - 1;
    seg_lo[sg] = lo;
    seg_w[sg] = sg < nseg ? 2 * (hi - lo + 1) + 2 : 0;
    seg_rw[sg] = sg < nseg ? 1.0f / (float)seg_w[sg] : 0.f;
    seg_b[sg + 1] = seg_b[sg] + 4 * seg_w[sg];
  }
  G.src_ok = 0;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const int sl = wino_sw(i * 64 + lane);
    const int pix = sl >> 2, qq = sl & 3;
    int sg = 0;
#pragma unroll
    for (int k = 1; k < 4; ++k) sg += pix >= seg_b[k] ? 1 : 0;
    const int wdt = sg == 0 ? seg_w[0] : sg == 1 ? seg_w[1] : sg == 2 ? seg_w[2] : seg_w[3];
    const float rw = sg == 0 ? seg_rw[0] : sg == 1 ? seg_rw[1] : sg == 2 ? seg_rw[2] : seg_rw[3];
    const int lo = sg == 0 ? seg_lo[0] : 0;
    const int bb = sg == 0 ? seg_b[0] : sg == 1 ? seg_b[1] : sg == 2 ? seg_b[2] : seg_b[3];
    const int lp = pix - bb;
    const int prow = (wdt && lp >= 0) ? wino_div(lp, rw) : 0, pcol = lp - prow * wdt;
    const int R = R0 + sg;
    const int img = wino_div(R, rth), ty = R - img * p.TH;
    const int iy = 2 * ty - 1 + prow, ix = 2 * lo - 1 + pcol;
    const bool in = pix < seg_b[4] && R < TR && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
    G.src_off[i] = in ? ((img * p.H + iy) * p.W + ix) * p.C + 4 * qq : 0;
    G.src_ok |= in ? 1u << i : 0u;
  }
  const int t = tw0 + r;
  const int tsg = t < p.T ? wino_div(t, rtw) - R0 : 0;
  G.pw = tsg == 0 ? seg_w[0] : tsg == 1 ? seg_w[1] : tsg == 2 ? seg_w[2] : seg_w[3];
  const int pb0 = tsg == 0 ? seg_b[0] : tsg == 1 ? seg_b[1] : tsg == 2 ? seg_b[2] : seg_b[3];
  const int plo = tsg == 0 ? seg_lo[0] : 0;
  const int prow0 = t < p.T ? pb0 + 2 * (t - (R0 + tsg) * p.TW - plo) : 0;
  G.ps0 = prow0 * 4 + q;
  G.tw0 = tw0;
}

template <int NW, int FN>
__global__ __launch_bounds__(NW * 64, NW == 4 ? 2 : 1) void conv_wino_f32_pu_kernel(WinoF32Params p) {
  using S = WinoV2Shape<NW, FN>;
  constexpr int PMAX = S::PMAX, PIECES = S::PIECES, PPW = S::PPW, SLOT = S::SLOT;
  static_assert(PMAX == 10, "wave image pieces");
  __shared__ __attribute__((aligned(16))) char smem[S::LDS];
  char* ring = smem;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 15, q = lane >> 4;
  char* pimg = smem + 2 * SLOT + wave * PMAX * 1024;
  const int KC = p.C / 16;
  const int NF = p.N / 16;
  const int gx = (p.T + 16 * NW - 1) / (16 * NW), gy = p.N / (16 * FN);
  const int units = gx * gy;
  int u = blockIdx.x;
  if (u >= units) return;
  const size_t uchunk = (size_t)NF * 16 * 256;
  // unit -> (tile group, channel group), tile group fastest: blocks running at once share weights
  int tg = u % gx, cg = u / gx;
  WinoGeom cur;
  wino_geom<NW>(p, tg, wave, lane, cur);
  auto issue_w = [&](int cgi, int kc, int slot) {
    const float* src = p.u + (size_t)cgi * FN * 16 * 256 + (size_t)kc * uchunk;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int pc = wave * PPW + i;
      if (PIECES % NW == 0 || pc < PIECES)
        __builtin_amdgcn_global_load_lds((const void*)(src + pc * 256 + lane * 4),
                                         (lds_void_w*)(ring + slot * SLOT + pc * 1024), 16, 0, 0);
    }
  };
  auto issue_x = [&](const WinoGeom& G, int kc) {
#pragma unroll
    for (int i = 0; i < PMAX; ++i) {
      const float* src = ((G.src_ok >> i) & 1u) ? p.x + G.src_off[i] + kc * 16 : g_wino_zero;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void_w*)(pimg + i * 1024), 16, 0, 0);
    }
  };
  f32x4 d[4][4];
  auto read_patch = [&](const WinoGeom& G) {
#pragma unroll
    for (int dy = 0; dy < 4; ++dy)
#pragma unroll
      for (int dx = 0; dx < 4; ++dx) d[dy][dx] = *(const f32x4*)(pimg + wino_sw(G.ps0 + dy * G.pw * 4 + dx * 4) * 16);
  };
  issue_w(cg, 0, 0);
  issue_x(cur, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  read_patch(cur);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  int slot = 0;
  while (true) {
    // the next unit's geometry, computed here while no accumulator is live yet (inside the chunk loop
    // its temporaries would sit beside acc and d and spill)
    const int un = u + gridDim.x;
    const bool has_next = un < units;
    const int ntg = has_next ? un % gx : tg, ncg = has_next ? un / gx : cg;
    WinoGeom nxt;
    wino_geom<NW>(p, ntg, wave, lane, nxt);
    f32x4 acc[16][FN];
#pragma unroll
    for (int i = 0; i < 16; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    for (int kc = 0; kc < KC; ++kc) {
      __builtin_amdgcn_s_barrier();                  // every wave's pieces of this step landed
      asm volatile("" ::: "memory");
      const bool last = kc + 1 == KC;
      const bool step = !last || has_next;
      if (step) {
        issue_w(last ? ncg : cg, last ? 0 : kc + 1, slot ^ 1);
        issue_x(last ? nxt : cur, last ? 0 : kc + 1);  // this step's patch is already in registers
      }
#pragma unroll
      for (int dx = 0; dx < 4; ++dx) {
        const f32x4 a0 = d[0][dx], a1 = d[1][dx], a2 = d[2][dx], a3 = d[3][dx];
        d[0][dx] = a0 - a2;
        d[1][dx] = a1 + a2;
        d[2][dx] = a2 - a1;
        d[3][dx] = a1 - a3;
      }
      const char* sl = ring + slot * SLOT;
#pragma unroll
      for (int pa = 0; pa < 4; ++pa) {
        f32x4 v[4];
        v[0] = d[pa][0] - d[pa][2];
        v[1] = d[pa][1] + d[pa][2];
        v[2] = d[pa][2] - d[pa][1];
        v[3] = d[pa][1] - d[pa][3];
#pragma unroll
        for (int pb = 0; pb < 4; ++pb) {
          f32x4 uu[FN];
#pragma unroll
          for (int j = 0; j < FN; ++j) uu[j] = *(const f32x4*)(sl + ((j * 16 + pa * 4 + pb) * 64 + lane) * 16);
#pragma unroll
          for (int ss = 0; ss < 4; ++ss)
#pragma unroll
            for (int j = 0; j < FN; ++j)
              acc[pa * 4 + pb][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(v[pb][ss], uu[j][ss], acc[pa * 4 + pb][j],
                                                                           0, 0, 0);
        }
      }
      if (step) {                                    // the next step's patch (its DMA went out above)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        read_patch(last ? nxt : cur);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
      slot ^= 1;
    }
    // unit done: output transform + stores through the wave image (the next unit's first patch has
    // already left it for the registers; its next DMA goes out only after the coming barrier)
    wino_epilogue<FN, 0>(p, acc, cur.tw0, r, q, cg * FN, (int*)smem, 0, 1, 0, pimg);
    if (!has_next) break;
    u = un;
    tg = ntg;
    cg = ncg;
    cur = nxt;
  }
}

template <int NW, int FN>
hipError_t launch_wino_pu(const WinoF32Params& p, hipStream_t s) {
  if (p.N % (16 * FN) || !wino_v2_shape_ok(p.TW) || p.ksplit != 1 || p.sk_iters > 0 || p.counters)
    return hipErrorInvalidValue;
  const int units = ((p.T + 16 * NW - 1) / (16 * NW)) * (p.N / (16 * FN));
  const int slots = NW == 4 ? 512 : 256;             // 8 waves per CU: two 4-wave blocks or one 8-wave block
  const int grid = units < slots ? units : slots;
  hipLaunchKernelGGL((conv_wino_f32_pu_kernel<NW, FN>), dim3(grid), dim3(NW * 64), 0, s, p);
  return hipGetLastError();
}


template <int NW, int FN, bool SW, bool EP, bool SK, int PL, bool XM>
hipError_t launch_wino_v2(const WinoF32Params& p, hipStream_t s) {
  if (p.N % (16 * FN) || !wino_v2_shape_ok(p.TW) || SK != (p.sk_iters > 0)) return hipErrorInvalidValue;
  dim3 grid((p.T + 16 * NW - 1) / (16 * NW), p.N / (16 * FN), p.ksplit), block(NW * 64);
  if (SK) {
    int G, iters, smax;
    conv_wino_sk_plan(grid.x * grid.y, p.C / 16, p.sk_mult, &G, &iters, &smax);
    if (iters != p.sk_iters || smax > 4 || !p.counters || !p.ws) return hipErrorInvalidValue;
    if (PL != 0 && iters > p.C / 16) return hipErrorInvalidValue;   // v3 stream-K: <= 2 units per block
    grid = dim3(G, 1, 1);
  }
  hipLaunchKernelGGL((conv_wino_f32_v2_kernel<NW, FN, SW, EP, SK, PL, XM>), grid, block, 0, s, p);
  return hipGetLastError();
}

template <int NWM, int FN, int STAGES, bool PF, int ABL>
hipError_t launch_wino(const WinoF32Params& p, hipStream_t s) {
  if (p.N % (16 * FN)) return hipErrorInvalidValue;
  const dim3 grid((p.T + 16 * NWM - 1) / (16 * NWM), p.N / (16 * FN), p.ksplit), block(NWM * 64);
  hipLaunchKernelGGL((conv_wino_f32_kernel<NWM, FN, STAGES, PF, ABL>), grid, block, 0, s, p);
  return hipGetLastError();
}

}  // namespace

// Winograd cfg ids (ops/conv.py WINO_F32_CFGS mirrors them): id -> waves (16 tiles each), 16-channel
// output fragments per wave, LDS ring stages, patch prefetch, ablation
// (90-99: cfg 80 with ablation switches ABL = id - 90, measurement only)
#define ADAPT_WINO_CFGS(X)  \
  X(80, 4, 2, 2, false, 0) \
  X(81, 4, 1, 2, false, 0) \
  X(82, 2, 2, 2, false, 0) \
  X(83, 8, 2, 2, false, 0) \
  X(84, 4, 3, 2, false, 0) \
  X(85, 2, 1, 2, false, 0) \
  X(86, 4, 2, 2, true, 0)  \
  X(87, 4, 3, 2, true, 0)  \
  X(88, 8, 1, 2, true, 0)  \
  X(91, 4, 2, 2, false, 1) \
  X(92, 4, 2, 2, false, 2) \
  X(94, 4, 2, 2, false, 4) \
  X(95, 4, 2, 2, false, 5) \
  X(98, 4, 2, 2, false, 8) \
  X(99, 4, 2, 2, false, 9)
// v2 (input patches staged by LDS-DMA): id -> waves, 16-channel output fragments per wave, swizzled image,
// early patch read, stream-K (110-114: the host passes ksplit <= -100), pipelined chunk body (116-117: v3;
// FN = 2 spills once the next fragments are held across a group), XCD-aware block order (130-132)
#define ADAPT_WINO2_CFGS(X)                 \
  X(100, 8, 2, false, false, false, 0, false)  \
  X(101, 8, 1, false, false, false, 0, false)  \
  X(102, 4, 1, false, false, false, 0, false)  \
  X(103, 8, 2, true, false, false, 0, false)   \
  X(104, 8, 1, true, false, false, 0, false)   \
  X(105, 4, 1, true, false, false, 0, false)   \
  X(106, 8, 2, true, true, false, 0, false)    \
  X(107, 8, 1, true, true, false, 0, false)    \
  X(108, 4, 1, true, true, false, 0, false)    \
  X(110, 8, 2, true, true, true, 0, false)     \
  X(111, 8, 2, true, false, true, 0, false)    \
  X(112, 4, 1, true, true, true, 0, false)     \
  X(113, 4, 1, true, false, true, 0, false)    \
  X(114, 8, 1, true, true, true, 0, false)     \
  X(116, 8, 1, true, true, false, 1, false)     \
  X(117, 4, 1, true, true, false, 1, false)  \
  X(130, 4, 1, true, false, false, 0, true)  \
  X(131, 8, 2, true, false, false, 0, true)  \
  X(132, 4, 1, true, true, false, 1, true)  \
  X(118, 8, 2, true, true, false, 2, false)  \
  X(119, 8, 2, true, true, false, 2, true)  \
  X(150, 8, 2, true, true, false, 3, false)  \
  X(151, 8, 2, true, true, false, 3, true)   \
  X(152, 8, 2, true, true, false, 4, false)  \
  X(153, 8, 2, true, true, false, 4, true)   \
  X(154, 8, 2, true, true, false, 10, false) \
  X(155, 8, 2, true, true, false, 18, false) \
  X(156, 8, 2, true, true, false, 26, false) \
  X(157, 8, 2, true, true, true, 2, false)   \
  X(158, 8, 2, true, true, true, 18, false)  \
  X(160, 8, 2, true, true, false, 5, false)  \
  X(161, 8, 2, true, true, false, 21, false) \
  X(162, 8, 2, true, true, false, 6, false)  \
  X(163, 8, 2, true, true, false, 22, false) \
  X(164, 8, 2, true, true, false, 38, false) \
  X(165, 8, 2, true, true, false, 54, false) \
  X(166, 8, 1, true, true, false, 33, false) \
  X(167, 4, 1, true, true, false, 33, false) \
  X(170, 8, 2, true, true, false, 66, false) \
  X(171, 8, 2, true, true, false, 130, false) \
  X(172, 8, 2, true, true, false, 194, false)

// stream-K plan of a Winograd v2 launch: `units` output blocks of kc chunks over about mult x 256 blocks;
// smax = the most partials one unit is cut into (the fused fixup takes <= 4)
void conv_wino_sk_plan(int units, int kc, int mult, int* grid, int* iters, int* smax) {
  const long long total = (long long)units * kc;
  long long G = 256LL * (mult > 0 ? mult : 1);
  if (G > total) G = total;
  const long long it = (total + G - 1) / G;
  *iters = (int)it;
  *grid = (int)((total + it - 1) / it);
  int m = 1;
  for (int u = 0; u < units; ++u) {
    const long long g0 = ((long long)u * kc) / it, g1 = ((long long)(u + 1) * kc - 1) / it;
    if (g1 - g0 + 1 > m) m = (int)(g1 - g0 + 1);
  }
  *smax = m;
}

bool conv_wino_f32_cfg(int cfg, int* nw, int* fn) {
  switch (cfg) {
    case 140: *nw = 4; *fn = 1; return true;         // persistent (conv_wino_f32_pu_kernel)
    case 141: *nw = 8; *fn = 1; return true;
#define X(id, NW_, FN_, SW_, EP_, SK_, PL_, XM_) case id: *nw = NW_; *fn = FN_; return true;
    ADAPT_WINO2_CFGS(X)
#undef X
#define X(id, NWM_, FN_, S_, PF_, A_) case id: *nw = NWM_; *fn = FN_; return true;
    ADAPT_WINO_CFGS(X)
#undef X
  }
  return false;
}

bool conv_wino_f32_ok(int cfg, int C, int N) {
  switch (cfg) {
    case 140:
    case 141: return C % 16 == 0 && N % 16 == 0;
#define X(id, NW_, FN_, SW_, EP_, SK_, PL_, XM_) case id: return C % 16 == 0 && N % (16 * FN_) == 0;
    ADAPT_WINO2_CFGS(X)
#undef X
#define X(id, NWM_, FN_, S_, PF_, A_) case id: return C % 16 == 0 && N % (16 * FN_) == 0;
    ADAPT_WINO_CFGS(X)
#undef X
  }
  return false;
}

static unsigned long long* g_wino_dbg = nullptr;
void wino_set_debug(unsigned long long* buf) { g_wino_dbg = buf; }

hipError_t conv_wino_f32_launch(const WinoF32Params& p_in, int cfg, hipStream_t s) {
  WinoF32Params p = p_in;
  p.dbg = g_wino_dbg;
  if (p.C % 16 || p.ksplit < 1 || p.T != p.B * p.TH * p.TW) return hipErrorInvalidValue;
  if (p.ksplit > 1 && !p.ws) return hipErrorInvalidValue;
  if (p.sk_iters > 0) {                              // stream-K: v2 configs, <= 4 slabs, 32-bit slab offsets
    if (cfg < 110 || p.ksplit != 1 || (size_t)4 * p.B * p.H * p.W * p.N * 4 > 0x7fffffffu) return hipErrorInvalidValue;
  } else if (p.counters && (p.ksplit < 2 || p.ksplit > 4 || (size_t)p.ksplit * p.B * p.H * p.W * p.N * 4 > 0x7fffffffu)) {
    return hipErrorInvalidValue;                     // fused split-K: 32-bit slab offsets
  }
  switch (cfg) {
    case 140: return launch_wino_pu<4, 1>(p, s);
    case 141: return launch_wino_pu<8, 1>(p, s);
#define X(id, NW_, FN_, SW_, EP_, SK_, PL_, XM_) case id: return launch_wino_v2<NW_, FN_, SW_, EP_, SK_, PL_, XM_>(p, s);
    ADAPT_WINO2_CFGS(X)
#undef X
#define X(id, NWM_, FN_, S_, PF_, A_) case id: return launch_wino<NWM_, FN_, S_, PF_, A_>(p, s);
    ADAPT_WINO_CFGS(X)
#undef X
  }
  return hipErrorInvalidValue;
}

}  // namespace adapt
