// fp32 3x3 / stride-1 / pad-1 convolution by Winograd F(4x4, 3x3), producer / consumer form (cfg 210):
// 8 waves per block, two per SIMD -- waves 0-3 only multiply, waves 4-7 only stage and transform.
//
// Why (measured on the one-wave-per-SIMD form, conv_wino4_f32.hip, tools/wino4_timeline.py --exp): its K loop
// ran 1.9-2.1 us per 8-channel chunk against 1.05 us of MFMA, and stayed at 1.5-1.6 us with the loop's LDS-DMA
// and the input transform both removed -- one wave per SIMD has to issue 72 MFMAs, 17 LDS-DMA pieces, ~280
// transform VALU (a third of them packed, an anti-lever beside MFMAs) and the LDS reads, more issue time than
// the MFMAs take.  Here the SIMD's two waves split that stream (MI355X_MICROARCH.md: an MFMA-only wave and a
// VALU-only wave on one SIMD run side by side): the consumer issues MFMAs, its A-operand LDS reads and its
// weight loads; the producer issues the image LDS-DMA, the input transform and the transformed-input stores.
//
//   V_p[t][c] = (B^T d_t,c B)_p   (d = the 6x6 input patch of tile t, p = 6 pa + pb, 36 positions)
//   M_p[t][n] = sum_c V_p[t][c] U_p[c][n]           U = G g G^T  (host fp64, ops/conv.py wino4_pack_np)
//   y_t[n]    = A^T M[t][n] A + bias[n]   (4x4 outputs)
//
// Block = 32 4x4 tiles x 32 output channels; K walks 8-channel chunks, one block barrier per chunk.
//  * producers (waves 4-7): the block's input patches are staged per chunk by LDS-DMA (the pieces dealt out
//    over the 4 producers) into a double-buffered image laid out as in conv_wino4_f32.hip: per tile-row
//    segment 6 input rows of 4n + 2 pixels, 16-B units of 4 channels, column groups of 4 pixels + one pad
//    unit; segment bases aligned so a tile's unit index mod 8 follows the tile.  Producer lane = (tile, one
//    channel): 36 ds_read_b32 (8 tiles x 4 channels per 32-lane group: 32 distinct banks), the full 6x6
//    transform (12 B^T applications, 168 VALU, scalar fp32), 36 ds_write_b32 into the V buffer of the next
//    chunk; V[p][s][q][t ^ 16 (q & 1)] (channel c = 2 q + s) keeps both the writes (2-way, free for b32
//    stores) and the consumers' reads conflict-free.
//  * consumers (waves 0-3): wave w accumulates the 3x3 quadrant of positions (pa in 3 (w & 1) + 0..2,
//    pb in 3 (w >> 1) + 0..2) for all 32 tiles x 32 channels: 9 x 2 tile halves x 2 fragments = 144 AGPRs.
//    Its transformed weights come straight from L2 into registers (9 buffer_load_dwordx4 per chunk, one
//    chunk ahead; each weight is read by exactly one wave of the block), the A operand from the V buffer
//    (36 ds_read_b32 per chunk).  v_mfma_f32_16x16x4_f32: step s of a chunk takes channel 2 q + s in K slot q.
//  * epilogue: the output transform is linear, so each consumer turns its quadrant into a partial 4x4
//    output per (tile, channel) in registers; the partials meet in LDS per 16-tile half (4 x 32 KiB), every
//    wave of the block adds the four in a fixed order and stores 16-B pieces (bias, residual, ReLU fused).
// Split-K (gridDim.z): > 1 writes fp32 slabs for splitk_reduce_f32; the fused form (p.counters set) publishes
// the slabs write-through and the last split of each block adds them in split order.
#include "kernels.h"

namespace adapt {

namespace {

constexpr int PC_VBUF = 36 * 8 * 32 * 4;               // bytes of one chunk's transformed inputs (36 KiB)
constexpr int PC_LDS = 160 * 1024;
constexpr int PC_MAXP = (PC_LDS - 2 * PC_VBUF - 16) / 2048;   // image pieces (1 KiB) per buffer: 43
constexpr int PC_HPW = (PC_MAXP + 3) / 4;              // pieces per producer wave and buffer: <= 11
constexpr int PC_WCH = 36 * 64 * 4;                    // floats of one (channel group, chunk) weight run
constexpr int PC_CPOL_SC1 = 16;
constexpr unsigned PC_OOB = 0x80000000u;               // voffset past the descriptor: the DMA writes zeros
static_assert(PC_MAXP >= 30, "LDS budget");
static_assert(4 * 32768 + 16 <= PC_LDS, "epilogue staging");

// the block's tile-row segments (host mirror: pc_geom is __host__ __device__)
struct PcGeom {
  int tw0, tlast, R0, lo0, nseg, pitch0, pitchm, pitchl, base1, Sp, units;
};

__host__ __device__ inline void pc_geom(int bx, int T, int TW, PcGeom& g) {
  g.tw0 = bx * 32;
  g.tlast = g.tw0 + 31 < T - 1 ? g.tw0 + 31 : T - 1;
  g.R0 = g.tw0 / TW;
  g.lo0 = g.tw0 - g.R0 * TW;
  const int R1 = g.tlast / TW;
  g.nseg = R1 - g.R0 + 1;
  const int n0 = g.nseg == 1 ? g.tlast - g.tw0 + 1 : TW - g.lo0;
  const int nl = g.tlast - R1 * TW + 1;
  g.pitch0 = 9 * n0 + 4;                               // units per image row: n column groups of 9 + 2 pixels
  g.pitchm = 9 * TW + 4;
  g.pitchl = 9 * nl + 4;
  const int size0 = 6 * g.pitch0, sizem = 6 * g.pitchm;
  // segment sg > 0 starts on unit 9 r0 (mod 8), r0 = the tiles before it: the 8 tiles of a 32-lane read
  // group land on 8 distinct unit phases (x 4 channels = 32 banks) across segment boundaries too
  g.base1 = size0 + ((9 * n0 - size0) & 7);
  g.Sp = sizem + ((9 * TW - sizem) & 7);               // a middle segment plus its pad (same phase step)
  g.units = g.nseg == 1 ? size0 : g.base1 + (g.nseg - 2) * g.Sp + 6 * g.pitchl;
}

// floor(a / b) for 0 <= a < 2^20, 1 <= b < 2^12 with rb = 1.0f / b (exact: conv_wino_f32.hip wino_div)
__device__ __forceinline__ int pc_div(int a, float rb) { return (int)(((float)a + 0.5f) * rb); }

// buffer descriptors from wave-uniform bases, pinned to SGPRs (a descriptor the compiler cannot prove
// uniform turns every buffer access into a readfirstlane waterfall loop)
__device__ __forceinline__ const float* pc_uniform(const float* base) {
  const unsigned long long a = (unsigned long long)(uintptr_t)base;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  return (const float*)(uintptr_t)(((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ u32x4 pc_desc(const float* base) {
  const unsigned long long a = (unsigned long long)(uintptr_t)pc_uniform(base);
  return (u32x4){(unsigned)a, (unsigned)(a >> 32) & 0xffffu, 0x7fffffffu, 0x00020000u};
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t pc_rsrc(const float* base) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)pc_uniform(base), (short)0, 0x7fffffff, 0x00020000);
}

// one 1 KiB LDS-DMA piece (16 B per lane, lane-linear at LDS byte address `lds`); M0 is set in the same
// statement (conv_wino4_f32.hip w4_dma: the compiler's wait model never sees it, the kernel waits itself)
// (soff and lds are wave-uniform; readfirstlane pins them to SGPRs where the compiler computed them in VALU)
__device__ __forceinline__ void pc_dma(int voff, u32x4 rsrc, int soff, unsigned lds) {
  asm volatile("s_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds" ::"v"(voff), "s"(rsrc),
               "s"(__builtin_amdgcn_readfirstlane(soff)), "s"(__builtin_amdgcn_readfirstlane(lds))
               : "memory");
}

__device__ __forceinline__ void pc_stamp(unsigned long long* d, int i) {
  if (d != nullptr && (threadIdx.x & 63) == 0) d[i] = __builtin_amdgcn_s_memtime();
}

// B^T of F(4x4, 3x3) on 6 values (14 VALU): rows [4 0 -5 0 1 0], [0 -4 -4 1 1 0], [0 4 -4 -1 1 0],
// [0 -2 -1 2 1 0], [0 2 -1 -2 1 0], [0 4 0 -5 0 1]
__device__ __forceinline__ void pc_bt(float& d0, float& d1, float& d2, float& d3, float& d4, float& d5) {
  const float s12 = d1 + d2, s34 = d3 + d4, m12 = d1 - d2, m43 = d4 - d3, m13 = d1 - d3, m42 = d4 - d2;
  const float t0 = fmaf(4.f, d0, fmaf(-5.f, d2, d4));
  const float t5 = fmaf(4.f, d1, fmaf(-5.f, d3, d5));
  d1 = fmaf(-4.f, s12, s34);
  d2 = fmaf(4.f, m12, m43);
  d3 = fmaf(-2.f, m13, m42);
  d4 = fmaf(2.f, m13, m42);
  d0 = t0;
  d5 = t5;
}

// A^T columns 3h .. 3h + 2 of F(4x4, 3x3) applied to 3 values -> 4 outputs: h = 0: columns (1 0 0 0),
// (1 1 1 1), (1 -1 1 -1); h = 1: (1 2 4 8), (1 -2 4 -8), (0 0 0 1)
template <int HH>
__device__ __forceinline__ void pc_at3(float m0, float m1, float m2, float (&o)[4]) {
  if constexpr (HH == 0) {
    const float s = m1 + m2, d = m1 - m2;
    o[0] = m0 + s; o[1] = d; o[2] = s; o[3] = d;
  } else {
    const float s = m0 + m1, d = m0 - m1;
    o[0] = s; o[1] = 2.f * d; o[2] = 4.f * s; o[3] = fmaf(8.f, d, m2);
  }
}

__device__ __forceinline__ int pc_dxu(int dx) { return dx < 4 ? 2 * dx : 2 * dx + 1; }

struct PcCtx {
  const WinoF32Params* p;
  char* smem;
  int kper, k0, ns, zs, cg, pieces;
  PcGeom g;
  unsigned long long* dbg;
};

// NHWC element offset of output pixel px (0..15) of block tile tl (0..31) at channel 0 of the block's channel
// group, or -1 outside the map / past the last tile
__device__ __forceinline__ int pc_out_off(const PcCtx& c, int tl, int px) {
  const WinoF32Params& p = *c.p;
  const int t = c.g.tw0 + tl;
  const int tpi = p.TH * p.TW;
  const int im = pc_div(t, 1.0f / (float)tpi), rr = t - im * tpi;
  const int ty = pc_div(rr, 1.0f / (float)p.TW), tx = rr - ty * p.TW;
  const int oy = 4 * ty + (px >> 2), ox = 4 * tx + (px & 3);
  return (t <= c.g.tlast && oy < p.H && ox < p.W) ? ((im * p.H + oy) * p.W + ox) * p.N + c.cg * 32 : -1;
}

// read-back of one 16-tile half (tb): 1024 tasks (16 tiles x 16 pixels x 4 channel quads) over the block's 512
// lanes; a task adds the 4 consumers' partials (staging [w][px][tile][2 n + j]) in wave order
template <typename F>
__device__ __forceinline__ void pc_readback(const PcCtx& c, int tb, F&& emit) {
#pragma unroll
  for (int rep = 0; rep < 2; ++rep) {
    const int tk = threadIdx.x + 512 * rep;
    const int c4 = tk & 3, px = (tk >> 2) & 15, tile = tk >> 6;
    const int idx = ((px * 16 + tile) * 32 + 8 * c4) * 4;
    f32x4 a = (f32x4){0.f, 0.f, 0.f, 0.f}, b = a;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      a += *(const f32x4*)(c.smem + w * 32768 + idx);
      b += *(const f32x4*)(c.smem + w * 32768 + idx + 16);
    }
    // staging index 2 n + j: a = (n, 0) (n, 1) (n + 1, 0) (n + 1, 1), b likewise for n + 2, n + 3
    const f32x4 v0 = (f32x4){a[0], a[2], b[0], b[2]};   // channels 4 c4 .. + 3
    const f32x4 v1 = (f32x4){a[1], a[3], b[1], b[3]};   // channels 16 + 4 c4 .. + 3
    emit(pc_out_off(c, 16 * tb + tile, px), c4, v0, v1);
  }
}

// ------------------------------------------------------------------ producer (waves 4-7)
template <int EXP>
__device__ __forceinline__ void pc_producer(PcCtx& c, int pw) {
  const WinoF32Params& p = *c.p;
  const int lane = threadIdx.x & 63;
  const PcGeom& g = c.g;
  const unsigned smem_lds = (unsigned)(uintptr_t)c.smem;
  const int IMGB = c.pieces * 1024;
  const unsigned img_lds = smem_lds + 2 * PC_VBUF;
  const char* const img = c.smem + 2 * PC_VBUF;
  const u32x4 xdesc = pc_desc(p.x);
  const float rtw = 1.0f / (float)p.TW, rth = 1.0f / (float)p.TH, rsp = 1.0f / (float)g.Sp;

  // DMA sources of this wave's pieces i = 4 ii + pw: unit i * 64 + lane <- byte offset in x at chunk 0
  int xoff[PC_HPW];
#pragma unroll
  for (int ii = 0; ii < PC_HPW; ++ii) {
    const int u = (4 * ii + pw) * 64 + lane;
    int sg = 0;
    if (g.nseg > 1 && u >= g.base1) sg = min(1 + pc_div(u - g.base1, rsp), g.nseg - 1);
    const int base = sg == 0 ? 0 : g.base1 + (sg - 1) * g.Sp;
    const int pitch = sg == 0 ? g.pitch0 : (sg == g.nseg - 1 ? g.pitchl : g.pitchm);
    const int lo = sg == 0 ? g.lo0 : 0;
    const int local = u - base;
    const int row = pc_div(local, 1.0f / (float)pitch);
    const int uu = local - row * pitch;
    const int g9 = pc_div(uu, 1.0f / 9.0f);
    const int e = uu - 9 * g9;
    const int px = 4 * g9 + (e >> 1), hh = e & 1;
    const int R = g.R0 + sg;
    const int im = pc_div(R, rth), ty = R - im * p.TH;
    const int iy = 4 * ty - 1 + row, ix = 4 * lo - 1 + px;
    const bool ok = u < g.units && row < 6 && e != 8 && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
    xoff[ii] = ok ? (((im * p.H + iy) * p.W + ix) * p.C + 4 * hh) * 4 : (int)PC_OOB;
  }
  auto issue = [&](int kc, int buf) {
#pragma unroll
    for (int ii = 0; ii < PC_HPW; ++ii)
      if (4 * ii + pw < c.pieces) pc_dma(xoff[ii], xdesc, kc * 32, img_lds + buf * IMGB + (4 * ii + pw) * 1024);
  };

  // this lane's tile (block tile tl) and chunk channel ch: patch pixel (dy, dx) at rd + dy * prs + 16 dxu(dx)
  const int tl = 16 * (pw & 1) + (lane >> 2);
  const int ch = 4 * (pw >> 1) + (lane & 3);
  const int t = g.tw0 + tl;
  int rd = 0, prs = 0;
  if (t <= g.tlast) {
    const int R = pc_div(t, rtw), sg = R - g.R0;
    const int base = sg == 0 ? 0 : g.base1 + (sg - 1) * g.Sp;
    const int pitch = sg == 0 ? g.pitch0 : (sg == g.nseg - 1 ? g.pitchl : g.pitchm);
    const int cgl = t - R * p.TW - (sg == 0 ? g.lo0 : 0);
    rd = (base + 9 * cgl + (ch >> 2)) * 16 + (ch & 3) * 4;
    prs = pitch * 16;
  }
  // V[pos][s][q][t ^ 16 (q & 1)], channel ch = 2 q + s
  const int q = ch >> 1, s = ch & 1;
  const int vw = ((s * 4 + q) * 32 + (tl ^ (16 * (q & 1)))) * 4;

  auto produce = [&](int buf, int vbuf) {
    const char* src = img + buf * IMGB + rd;
    float d[36];
#pragma unroll
    for (int dy = 0; dy < 6; ++dy)
#pragma unroll
      for (int dx = 0; dx < 6; ++dx) d[dy * 6 + dx] = *(const float*)(src + dy * prs + 16 * pc_dxu(dx));
    if constexpr (!(EXP & 2)) {
#pragma unroll
      for (int dy = 0; dy < 6; ++dy)
        pc_bt(d[dy * 6 + 0], d[dy * 6 + 1], d[dy * 6 + 2], d[dy * 6 + 3], d[dy * 6 + 4], d[dy * 6 + 5]);
#pragma unroll
      for (int pb = 0; pb < 6; ++pb) pc_bt(d[pb], d[6 + pb], d[12 + pb], d[18 + pb], d[24 + pb], d[30 + pb]);
    }
    char* dst = c.smem + vbuf * PC_VBUF + vw;
#pragma unroll
    for (int pos = 0; pos < 36; ++pos) *(float*)(dst + pos * 1024) = d[pos];
  };

  // prologue: chunk k0's image (buffer 0) and k0 + 1's (buffer 1; kper >= 2), every producer's pieces landed
  // (barrier), then V(k0)
  issue(c.k0, 0);
  issue(c.k0 + 1, 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  produce(0, 0);
  pc_stamp(c.dbg, 1);
  // chunk j: the consumers multiply V(j); the image of j + 2 refills buffer j & 1 (read during j - 1), and
  // V(j + 1) is built from image buffer (j + 1) & 1 into V buffer (j + 1) & 1 (read during j - 1)
  for (int j = 0; j < c.kper; ++j) {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (!(EXP & 1) && j + 2 < c.kper) issue(c.k0 + j + 2, j & 1);
    if (!(EXP & 16) && j + 1 < c.kper) produce((j + 1) & 1, (j + 1) & 1);
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  pc_stamp(c.dbg, 2);
}

// ------------------------------------------------------------------ consumer (waves 0-3)
template <int HA, int HB, int EXP>
__device__ __forceinline__ void pc_consumer_loop(PcCtx& c, f32x4 (&acc)[9][2][2]) {
  const WinoF32Params& p = *c.p;
  const int lane = threadIdx.x & 63;
  const int i = lane & 15, q = lane >> 4;
  const int KC = p.C / 8;
  const __amdgpu_buffer_rsrc_t ur = pc_rsrc(p.u + (size_t)c.cg * KC * PC_WCH);
  const int uvo = lane * 16 + (18 * HA + 3 * HB) * 1024;     // position (3 HA, 3 HB) of this lane
  // A operand: V[pos][s][q][(16 tb + i) ^ 16 (q & 1)]
  const int va0 = (q * 32 + ((0 ^ (q & 1)) * 16 + i)) * 4;
  const int va1 = (q * 32 + ((1 ^ (q & 1)) * 16 + i)) * 4;

  auto load_u = [&](f32x4 (&bu)[9], int kc) {
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
      for (int b = 0; b < 3; ++b)
        bu[3 * a + b] = __builtin_bit_cast(
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                       ur, uvo, __builtin_amdgcn_readfirstlane(kc * (PC_WCH * 4) + (6 * a + b) * 1024), 0));
  };
  auto step = [&](int j, f32x4 (&bc)[9], f32x4 (&bn)[9]) {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (!(EXP & 4) && j + 1 < c.kper) load_u(bn, c.k0 + j + 1);
    const char* vb = c.smem + (j & 1) * PC_VBUF;
    // 18 groups g = (k = 3 a + b, tb): the A pair of group g + 1 is read while group g's 4 MFMAs run
    auto rd = [&](int g, float (&av)[2]) {
      const int k = g >> 1, tb = g & 1;
      const int pos = 6 * (3 * HA + k / 3) + 3 * HB + k % 3;
      const char* va = vb + (tb ? va1 : va0) + pos * 1024;
      av[0] = *(const float*)(va);
      av[1] = *(const float*)(va + 512);
    };
    float av[2][2];
    rd(0, av[0]);
#pragma unroll
    for (int g = 0; g < 18; ++g) {
      if (g < 17) rd(g + 1, av[(g + 1) & 1]);
      const int k = g >> 1, tb = g & 1;
      if constexpr (EXP & 8) {
        acc[k][tb][0][0] += av[g & 1][0] + av[g & 1][1];
      } else {
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int jj = 0; jj < 2; ++jj)
            acc[k][tb][jj] =
                __builtin_amdgcn_mfma_f32_16x16x4f32(av[g & 1][s], bc[k][2 * jj + s], acc[k][tb][jj], 0, 0, 0);
      }
      // one group per scheduling region: left free, the scheduler (at ~240 registers) sinks each read to
      // just before its MFMAs and exposes the LDS latency every group
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  f32x4 bA[9], bB[9];
  load_u(bA, c.k0);
  __builtin_amdgcn_s_barrier();                      // the prologue barrier (the producers' image has landed)
  pc_stamp(c.dbg, 1);
  for (int j = 0; j < c.kper; j += 2) {              // kper even (host)
    step(j, bA, bB);
    step(j + 1, bB, bA);
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  pc_stamp(c.dbg, 2);
}

// partial output transform of the quadrant for 16-tile half tb, staged as [w][px][tile][2 n + j]
template <int HA, int HB>
__device__ __forceinline__ void pc_consumer_stage(PcCtx& c, const f32x4 (&acc)[9][2][2], int tb, int w) {
  const int lane = threadIdx.x & 63;
  const int r = lane & 15, q = lane >> 4;
  char* const st = c.smem + w * 32768;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float o[2][16];
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      float wv[3][4];                                 // pb direction: wv[a][x]
#pragma unroll
      for (int a = 0; a < 3; ++a)
        pc_at3<HB>(acc[3 * a][tb][jj][i], acc[3 * a + 1][tb][jj][i], acc[3 * a + 2][tb][jj][i], wv[a]);
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        float col[4];
        pc_at3<HA>(wv[0][x], wv[1][x], wv[2][x], col);
#pragma unroll
        for (int y = 0; y < 4; ++y) o[jj][4 * y + x] = col[y];
      }
    }
#pragma unroll
    for (int px = 0; px < 16; ++px) {
      typedef float f32x2_t __attribute__((ext_vector_type(2)));
      *(f32x2_t*)(st + ((px * 16 + 4 * q + i) * 32 + 2 * r) * 4) = (f32x2_t){o[0][px], o[1][px]};
    }
  }
}

}  // namespace

// EXP (measurement variants only, tools/wino4_timeline.py --cfg 210 --exp; outputs wrong by design): bit 0 no
// image DMA in the K loop, 1 no input transform, 2 no weight loads in the loop, 3 no MFMAs, 4 producers skip
// the patch reads / transform / V stores
template <int EXP>
__global__ __launch_bounds__(512, 1) void conv_wino4pc_f32_kernel(WinoF32Params p) {
  __shared__ __attribute__((aligned(16))) char smem[PC_LDS];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  PcCtx c;
  c.p = &p;
  c.smem = smem;
  c.cg = blockIdx.y;
  c.zs = blockIdx.z;
  c.ns = gridDim.z;
  const int KC = p.C / 8;
  c.kper = KC / c.ns;
  c.k0 = c.zs * c.kper;
  pc_geom(blockIdx.x, p.T, p.TW, c.g);
  c.pieces = (c.g.units + 63) >> 6;
  c.dbg = p.dbg ? p.dbg + 8 * (wave + 8 * (blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z))) : nullptr;
  pc_stamp(c.dbg, 0);
  if (c.dbg && (threadIdx.x & 63) == 0) c.dbg[6] = __builtin_amdgcn_s_memrealtime();

  // ---- main loop + half-0 staging (consumers) / idle (producers); barriers: prologue, kper, E0, E1
  f32x4 acc[9][2][2];
  if (wave < 4) {
#pragma unroll
    for (int k = 0; k < 9; ++k)
#pragma unroll
      for (int tb = 0; tb < 2; ++tb)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) acc[k][tb][jj] = (f32x4){0.f, 0.f, 0.f, 0.f};
    switch (wave) {
      case 0: pc_consumer_loop<0, 0, EXP>(c, acc); break;
      case 1: pc_consumer_loop<1, 0, EXP>(c, acc); break;
      case 2: pc_consumer_loop<0, 1, EXP>(c, acc); break;
      default: pc_consumer_loop<1, 1, EXP>(c, acc); break;
    }
  } else {
    pc_producer<EXP>(c, wave - 4);
  }
  __builtin_amdgcn_s_barrier();                      // E0: every wave is done with the V / image buffers
  asm volatile("" ::: "memory");
  pc_stamp(c.dbg, 4);

  const bool split = c.ns > 1;
  const bool fused = split && p.counters != nullptr;
  const int MN = p.B * p.H * p.W * p.N;
  const __amdgpu_buffer_rsrc_t wsr = pc_rsrc(p.ws);
  auto finish = [&](int o, f32x4 v, int ch) {
    v += *(const f32x4*)(p.bias + c.cg * 32 + ch);
    if (p.res) v += *(const f32x4*)(p.res + o + ch);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = act_relu(v[e], p.relu);
    *(f32x4*)(p.out + o + ch) = v;
  };
  auto emit = [&](int o, int c4, f32x4 v0, f32x4 v1) {
    if (o < 0) return;
    if (!split) {
      finish(o, v0, 4 * c4);
      finish(o, v1, 16 + 4 * c4);
    } else if (!fused) {
      *(f32x4*)(p.ws + (size_t)c.zs * MN + o + 4 * c4) = v0;
      *(f32x4*)(p.ws + (size_t)c.zs * MN + o + 16 + 4 * c4) = v1;
    } else {
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v0), wsr, (c.zs * MN + o + 4 * c4) * 4, 0,
                                             PC_CPOL_SC1);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v1), wsr, (c.zs * MN + o + 16 + 4 * c4) * 4,
                                             0, PC_CPOL_SC1);
    }
  };
#pragma unroll
  for (int tb = 0; tb < 2; ++tb) {
    if (wave < 4) {
      switch (wave) {
        case 0: pc_consumer_stage<0, 0>(c, acc, tb, 0); break;
        case 1: pc_consumer_stage<1, 0>(c, acc, tb, 1); break;
        case 2: pc_consumer_stage<0, 1>(c, acc, tb, 2); break;
        default: pc_consumer_stage<1, 1>(c, acc, tb, 3); break;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();                    // half tb staged
    asm volatile("" ::: "memory");
    pc_readback(c, tb, emit);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();                    // the staging is free again
    asm volatile("" ::: "memory");
    if (tb == 0) pc_stamp(c.dbg, 5);
  }
  pc_stamp(c.dbg, 3);
  if (c.dbg && (threadIdx.x & 63) == 0) c.dbg[7] = __builtin_amdgcn_s_memrealtime();
  if (!fused) return;
  // fused split-K: this split's slab is published (sc1); the last arriving split of the block adds every
  // slab in split order (deterministic whoever arrives last), then bias / residual / ReLU
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* const flag = (int*)(smem + PC_LDS - 16);
  if (threadIdx.x == 0) {
    int* ctr = p.counters + blockIdx.x + gridDim.x * blockIdx.y;
    const int old = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == c.ns - 1;
    if (last) __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = last;
  }
  __syncthreads();
  if (!*flag) return;
#pragma unroll
  for (int tb = 0; tb < 2; ++tb)
#pragma unroll
    for (int rep = 0; rep < 2; ++rep) {
      const int tk = threadIdx.x + 512 * rep;
      const int c4 = tk & 3, px = (tk >> 2) & 15, tile = tk >> 6;
      const int o = pc_out_off(c, 16 * tb + tile, px);
      if (o < 0) continue;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int ch = 16 * h + 4 * c4;
        f32x4 v = (f32x4){0.f, 0.f, 0.f, 0.f};
        for (int z = 0; z < c.ns; ++z)
          v += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(wsr, (z * MN + o + ch) * 4, 0,
                                                                               PC_CPOL_SC1));
        finish(o, v, ch);
      }
    }
}

// image pieces (1 KiB) of the widest block of an F(4x4) producer / consumer launch; 0: not supported
int conv_wino4pc_pieces(int B, int H, int W) {
  const int TH = (H + 3) / 4, TW = (W + 3) / 4, T = B * TH * TW;
  if (T >= (1 << 20) || TH * TW >= 4096 || 6 * (9 * TW + 4) + 8 >= 4096) return 0;
  int mx = 0;
  for (int bx = 0; bx * 32 < T; ++bx) {
    PcGeom g;
    pc_geom(bx, T, TW, g);
    mx = g.units > mx ? g.units : mx;
  }
  const int pieces = (mx + 63) / 64;
  return pieces <= PC_MAXP ? pieces : 0;
}

hipError_t conv_wino4pc_f32_launch(const WinoF32Params& p_in, hipStream_t s) {
  WinoF32Params p = p_in;
  p.dbg = wino4_debug_buffer();
  const int KC = p.C / 8;
  const int ns = p.ksplit;
  if (p.C % 16 || p.N % 32 || ns < 1 || KC % ns || (KC / ns) % 2 || p.sk_iters > 0) return hipErrorInvalidValue;
  if (p.TH != (p.H + 3) / 4 || p.TW != (p.W + 3) / 4 || p.T != p.B * p.TH * p.TW) return hipErrorInvalidValue;
  if (ns > 1 && (!p.ws || (size_t)ns * p.B * p.H * p.W * p.N * 4 > 0x7fffffffu)) return hipErrorInvalidValue;
  if ((size_t)p.B * p.H * p.W * p.C * 4 >= 0x7fffffffu) return hipErrorInvalidValue;   // 31-bit DMA offsets
  if (conv_wino4pc_pieces(p.B, p.H, p.W) == 0) return hipErrorInvalidValue;
  const dim3 grid((p.T + 31) / 32, p.N / 32, ns), block(512);
  switch (wino4_exp_flags()) {
    case 0: hipLaunchKernelGGL(conv_wino4pc_f32_kernel<0>, grid, block, 0, s, p); break;
    case 1: hipLaunchKernelGGL(conv_wino4pc_f32_kernel<1>, grid, block, 0, s, p); break;
    case 4: hipLaunchKernelGGL(conv_wino4pc_f32_kernel<4>, grid, block, 0, s, p); break;
    case 17: hipLaunchKernelGGL(conv_wino4pc_f32_kernel<17>, grid, block, 0, s, p); break;
    case 12: hipLaunchKernelGGL(conv_wino4pc_f32_kernel<12>, grid, block, 0, s, p); break;
    case 21: hipLaunchKernelGGL(conv_wino4pc_f32_kernel<21>, grid, block, 0, s, p); break;
    case 13: hipLaunchKernelGGL(conv_wino4pc_f32_kernel<13>, grid, block, 0, s, p); break;
    case 14: hipLaunchKernelGGL(conv_wino4pc_f32_kernel<14>, grid, block, 0, s, p); break;
    case 5: hipLaunchKernelGGL(conv_wino4pc_f32_kernel<5>, grid, block, 0, s, p); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace adapt
