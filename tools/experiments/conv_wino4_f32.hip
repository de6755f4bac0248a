// fp32 3x3 / stride-1 / pad-1 convolution by Winograd F(4x4, 3x3) on the fp32 matrix cores
// (v_mfma_f32_16x16x4_f32), transforms fused: one launch reads the NHWC input and writes the NHWC
// output (BN folded, bias, residual, ReLU).
//
// Why: F(2x2, 3x3) (conv_wino_f32.hip) does 16 multiplies per 2x2 output tile and (cin, cout), i.e.
// 4 per output; F(4x4, 3x3) does 36 per 4x4 tile, 2.25 per output -- 1.78x less matrix work on the
// layers that are 37 % of the fp32 ResNet-50 forward.  It is the algorithm cuDNN runs for float32 3x3
// convs under TensorFlow (the reference's Keras model, `/root/reference/test/test.py:13`, float32
// `model.predict` at `/root/reference/test/local_infer.py:22`).  Everything stays fp32: the weight
// transform (1/4, 1/6, 1/24 factors) is done on the host in fp64 and rounded once; the input / output
// transforms use small integer coefficients (B^T: 4, 5, 2; A^T: 2, 4, 8).
//
//   V_p[t][c] = (B^T d_t,c B)_p   (d = the 6x6 input patch of tile t, p = pa * 6 + pb, 36 positions)
//   M_p[t][n] = sum_c V_p[t][c] U_p[c][n]           U = G g G^T  (host, ops/conv.py wino4_pack_np)
//   y_t[n]    = A^T M[t][n] A + bias[n]   (4x4 outputs)
//
// Layout (MI355X-first, one wave per SIMD, 512 registers each):
//  * block = 4 waves = 2 tile groups x a wave pair.  Both waves of a pair own the same 16 tiles (the MFMA
//    rows) x 32 output channels (two 16-channel fragments); wave h of the pair accumulates the positions
//    of rows pa = 3h .. 3h + 2 only: 18 positions x 2 fragments = 144 accumulators, within the 256 AGPRs
//    an MFMA can address (all 36 positions would be 288 and spill).  The split also halves the input
//    transform: B^T's rows 0-2 read patch rows 0-4 and rows 3-5 read rows 1-5, so wave h row-transforms
//    5 patch rows and applies 3 of the 6 column rows (3.3 / 2.9 VALU per MFMA instead of 4.7).
//  * K walks the input channels in chunks of 8: MFMA step s of a chunk takes channel 2q + s from lane
//    group q, so a lane's share of the patch is 30 float2 (its tile, its 2 channels), transformed in
//    registers; the A operand never exists as a matrix.  Two patch register sets: the NEXT chunk's patch
//    is read and transformed while the current chunk's 72 MFMAs run.
//  * transformed weights, host-packed [N/32][C/8][36 positions][64 lanes][2 fragments][2 steps]: one
//    contiguous 36 KiB run per (channel group, chunk), streamed into a two-slot LDS ring by LDS-DMA
//    (9 pieces per wave) and read back as one lane-linear ds_read_b128 per position (conflict-free).
//  * each tile group's input patches are staged by LDS-DMA (the pair splits the pieces) in a double-
//    buffered image: per tile-row segment of n tiles, 6 input rows of 4n + 2 pixels, 8 channels (two 16-B
//    halves) per pixel, laid out as column groups of 4 pixels + one 16-B pad (9 units): tiles 4 pixels
//    apart land 9 units apart, i.e. on 16 different 16-B bank slots, so a patch read (ds_read_b64) is
//    conflict-free, and every pixel of a tile's patch sits at the lane's row base + an immediate offset.
//  * the output transform is linear, so each wave transforms its 18 positions into a partial 4x4 output
//    (lane-local: all positions of a (tile, channel) sit in one lane); the pair's partials meet in LDS,
//    are added in a fixed order and leave as 16-B stores (8 lanes per 128-B line).
// Split-K (gridDim.z, ksplit): > 1 writes partial outputs to fp32 slabs for splitk_reduce_f32; < 0 (the
// host passes counters) fuses the fixup: the last split of each block adds the slabs in split order.
#include "kernels.h"

namespace adapt {

namespace {

typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int W4_NW = 4;                        // waves per block (one per SIMD): 2 tile groups x 2 halves
constexpr int W4_FN = 2;                        // 16-channel output fragments per wave
constexpr int W4_WPW = 9;                       // weight pieces per wave per chunk
constexpr int W4_SLOT = 36 * 64 * 16;           // bytes of one chunk's weights (36 KiB)
constexpr int W4_WCH = W4_SLOT / 4;             // floats of one chunk's weights
constexpr int W4_CPOL_SC1 = 16;                 // gfx950 cache policy: sc1
constexpr int W4_MAXSEG = 8;                    // tile-row segments per wave (TW >= 2)

// measurement only (tools/wino4_timeline.py): per wave 8 words -- shader clock at start / table built /
// first patch transformed / K loop done / partial outputs staged / stores issued, and the 100 MHz wall
// clock at start and end; lane 0 writes them with vector stores
__device__ __forceinline__ void w4_stamp(unsigned long long* d, int i) {
  if (d != nullptr && (threadIdx.x & 63) == 0) d[i] = __builtin_amdgcn_s_memtime();
}

// floor(a / b) for 0 <= a < 2^20, 1 <= b < 2^12 with rb = 1.0f / b (exact: conv_wino_f32.hip wino_div)
__device__ __forceinline__ int w4_div(int a, float rb) { return (int)(((float)a + 0.5f) * rb); }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t w4_rsrc(const float* base) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, 0x7fffffff, 0x00020000);
}

// one 1 KiB LDS-DMA piece (16 B per lane, lane-linear at LDS byte address `lds`) by a raw buffer load:
// source = descriptor base + voff (per lane) + soff (scalar: the chunk, the piece).  A lane whose voff is
// out of the descriptor's range (W4_OOB) writes zeros -- the image's padding -- with no dummy buffer, and
// the chunk offset is scalar, so no 64-bit address VALU.  Issued from inline asm: the compiler's
// wait-count model (which counts an LDS DMA as an LDS access too) never sees it, so the loop's LDS waits
// stay partial; the kernel waits for its DMA itself (vmcnt at the chunk barrier).  M0 is written in the
// same statement (the compiler keeps nothing in M0 across it).
constexpr unsigned W4_OOB = 0x80000000u;
__device__ __forceinline__ void w4_dma(int voff, u32x4 rsrc, int soff, unsigned lds) {
  asm volatile("s_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds" ::"v"(voff), "s"(rsrc),
               "s"(soff), "s"(lds)
               : "memory");
}
__device__ __forceinline__ u32x4 w4_desc(const float* base) {
  const unsigned long long a = (unsigned long long)(uintptr_t)base;
  return (u32x4){(unsigned)a, (unsigned)(a >> 32) & 0xffffu, 0x7fffffffu, 0x00020000u};
}

// B^T of F(4x4, 3x3) on 6 values (14 VALU): rows [4 0 -5 0 1 0], [0 -4 -4 1 1 0], [0 4 -4 -1 1 0],
// [0 -2 -1 2 1 0], [0 2 -1 -2 1 0], [0 4 0 -5 0 1]
__device__ __forceinline__ void w4_bt(float& d0, float& d1, float& d2, float& d3, float& d4, float& d5) {
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

// B^T row transform (over dx) of patch row `row` (local index) of a lane's 2 channels, in place
__device__ __forceinline__ void w4_row(f32x2 (&d)[30], int row) {
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    float v0 = d[row * 6 + 0][c], v1 = d[row * 6 + 1][c], v2 = d[row * 6 + 2][c];
    float v3 = d[row * 6 + 3][c], v4 = d[row * 6 + 4][c], v5 = d[row * 6 + 5][c];
    w4_bt(v0, v1, v2, v3, v4, v5);
    d[row * 6 + 0][c] = v0; d[row * 6 + 1][c] = v1; d[row * 6 + 2][c] = v2;
    d[row * 6 + 3][c] = v3; d[row * 6 + 4][c] = v4; d[row * 6 + 5][c] = v5;
  }
}

// the same on one channel
__device__ __forceinline__ void w4_row1(f32x2 (&d)[30], int row, int c) {
  float v0 = d[row * 6 + 0][c], v1 = d[row * 6 + 1][c], v2 = d[row * 6 + 2][c];
  float v3 = d[row * 6 + 3][c], v4 = d[row * 6 + 4][c], v5 = d[row * 6 + 5][c];
  w4_bt(v0, v1, v2, v3, v4, v5);
  d[row * 6 + 0][c] = v0; d[row * 6 + 1][c] = v1; d[row * 6 + 2][c] = v2;
  d[row * 6 + 3][c] = v3; d[row * 6 + 4][c] = v4; d[row * 6 + 5][c] = v5;
}

// B^T column rows 3h .. 3h + 2 applied to column pb of the row-transformed patch (5 rows: patch rows
// h .. h + 4) -> V[3h + a][pb], a = 0..2.  h = 0: [4 0 -5 0 1], [0 -4 -4 1 1], [0 4 -4 -1 1] on rows 0-4
// (8 VALU); h = 1: [-2 -1 2 1 0], [2 -1 -2 1 0], [4 0 -5 0 1] on rows 1-5 (6 VALU)
template <int H>
__device__ __forceinline__ void w4_colh(const f32x2 (&d)[30], f32x2 (&v)[18], int pb) {
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const float e0 = d[0 * 6 + pb][c], e1 = d[1 * 6 + pb][c], e2 = d[2 * 6 + pb][c];
    const float e3 = d[3 * 6 + pb][c], e4 = d[4 * 6 + pb][c];
    if constexpr (H == 0) {        // e_k = row k
      v[0 * 6 + pb][c] = fmaf(4.f, e0, fmaf(-5.f, e2, e4));
      v[1 * 6 + pb][c] = fmaf(-4.f, e1 + e2, e3 + e4);
      v[2 * 6 + pb][c] = fmaf(4.f, e1 - e2, e4 - e3);
    } else {                       // e_k = row k + 1
      const float m13 = e0 - e2, m42 = e3 - e1;
      v[0 * 6 + pb][c] = fmaf(-2.f, m13, m42);
      v[1 * 6 + pb][c] = fmaf(2.f, m13, m42);
      v[2 * 6 + pb][c] = fmaf(4.f, e0, fmaf(-5.f, e2, e4));
    }
  }
}

// A^T of F(4x4, 3x3) on 6 values -> 4 (10 VALU): rows [1 1 1 1 1 0], [0 1 -1 2 -2 0], [0 1 1 4 4 0],
// [0 1 -1 8 -8 1]
__device__ __forceinline__ void w4_at(const float (&m)[6], float (&o)[4]) {
  const float s12 = m[1] + m[2], d12 = m[1] - m[2], s34 = m[3] + m[4], d34 = m[3] - m[4];
  o[0] = m[0] + s12 + s34;
  o[1] = fmaf(2.f, d34, d12);
  o[2] = fmaf(4.f, s34, s12);
  o[3] = fmaf(8.f, d34, d12) + m[5];
}

// pixel offsets (in 16-B units) of patch column dx inside a 9-unit column group layout
__device__ __forceinline__ constexpr int w4_dxu(int dx) { return dx < 4 ? 2 * dx : 2 * dx + 1; }

template <int PIECES, int H, int EXP>
__device__ __forceinline__ void wino4_wave(const WinoF32Params& p, char* smem, int wave) {
  constexpr int NW = W4_NW, WPW = W4_WPW, SLOT = W4_SLOT, WCH = W4_WCH;
  constexpr int IMG = PIECES * 1024;                 // one image buffer of a tile group
  constexpr int HP = (PIECES + 1) / 2;               // image pieces a wave of the pair issues (at most)
  constexpr int TAB = HP * 256;                      // a wave's DMA source table (one int per unit)
  constexpr int LDS = 2 * SLOT + 4 * IMG + NW * TAB;
  const unsigned smem_lds = (unsigned)(uintptr_t)smem;
  const int lane = threadIdx.x & 63;
  const int r = lane & 15, q = lane >> 4;
  const int tgl = wave >> 1;                         // tile group of the block
  char* const imgb = smem + 2 * SLOT + tgl * 2 * IMG;           // its two image buffers
  const unsigned imgb_lds = smem_lds + 2 * SLOT + tgl * 2 * IMG;
  int* const tab = (int*)(smem + 2 * SLOT + 4 * IMG + wave * TAB);
  const int cg = blockIdx.y, zs = blockIdx.z;
  const int ns = gridDim.z;                          // splits of K
  const int KC = p.C / 8;
  const int kper = KC / ns;                          // host: even, ns divides KC
  const int k0 = zs * kper, k1 = k0 + kper;
  const u32x4 xdesc = w4_desc(p.x);
  const u32x4 udesc = w4_desc(p.u + (size_t)cg * KC * WCH);
  unsigned long long* const dbg =
      p.dbg ? p.dbg + 8 * (wave + W4_NW * (blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z))) : nullptr;
  w4_stamp(dbg, 0);
  if (dbg && lane == 0) dbg[6] = __builtin_amdgcn_s_memrealtime();

  // ---- the tile group's tile-row segments (wave-uniform)
  const int tw0 = (blockIdx.x * 2 + tgl) * 16;
  const int tlast = min(tw0 + 15, p.T - 1);
  const float rtw = 1.0f / (float)p.TW, rth = 1.0f / (float)p.TH;
  const int R0 = w4_div(tw0, rtw);
  const int nseg = tw0 < p.T ? w4_div(tlast, rtw) - R0 + 1 : 0;
  int seg_lo[W4_MAXSEG], seg_pitch[W4_MAXSEG], seg_base[W4_MAXSEG + 1];
  float seg_rp[W4_MAXSEG];
  seg_base[0] = 0;
  int r0 = 0;                                        // tiles of the group before the segment
#pragma unroll
  for (int sg = 0; sg < W4_MAXSEG; ++sg) {
    const int lo = sg == 0 ? tw0 - R0 * p.TW : 0;
    const int hi = sg == nseg - 1 ? tlast - (R0 + sg) * p.TW : p.TW - 1;
    const int n = sg < nseg ? hi - lo + 1 : 0;
    seg_lo[sg] = lo;
    seg_pitch[sg] = n ? 9 * n + 4 : 0;              // units per image row: n column groups of 9 + 2 pixels
    seg_rp[sg] = n ? 1.0f / (float)(9 * n + 4) : 0.f;
    r0 += n;
    // flags & 1: start the next segment on the 16-B bank slot 9 r0 (mod 16), so the group's 16 tiles take
    // 16 distinct slots whenever the segments' pitches agree (full tile rows: stages 4 / 5 at bs 32)
    const int b = seg_base[sg] + 6 * seg_pitch[sg];
    seg_base[sg + 1] = ((p.flags & 1) && sg + 1 < nseg) ? b + ((9 * r0 - b) & 15) : b;
  }
  const int units = seg_base[W4_MAXSEG];

  // ---- DMA source table: this wave's pieces i = 2 ii + H of the image; unit i * 64 + l <- byte offset in
  // x at chunk 0 (W4_OOB: zeros).  Built once, read back per chunk by the same lane (no barrier): the
  // offsets would otherwise hold 8 VGPRs through the K loop
#pragma unroll
  for (int ii = 0; ii < HP; ++ii) {
    const int u = (2 * ii + H) * 64 + lane;
    int sg = 0;
#pragma unroll
    for (int k = 1; k < W4_MAXSEG; ++k) sg += u >= seg_base[k] ? 1 : 0;
    int base = seg_base[0], pitch = seg_pitch[0], lo = seg_lo[0];
    float rp = seg_rp[0];
#pragma unroll
    for (int k = 1; k < W4_MAXSEG; ++k) {
      base = sg == k ? seg_base[k] : base;
      pitch = sg == k ? seg_pitch[k] : pitch;
      lo = sg == k ? seg_lo[k] : lo;
      rp = sg == k ? seg_rp[k] : rp;
    }
    const int local = u - base;
    const int row = pitch ? w4_div(local, rp) : 0;
    const int uu = local - row * pitch;
    const int g9 = w4_div(uu, 1.0f / 9.0f);
    const int e = uu - 9 * g9;
    const int px = 4 * g9 + (e >> 1), hh = e & 1;
    const int R = R0 + sg;
    const int im = w4_div(R, rth), ty = R - im * p.TH;
    const int iy = 4 * ty - 1 + row, ix = 4 * lo - 1 + px;
    const bool ok = u < units && e != 8 && R < p.B * p.TH && (unsigned)iy < (unsigned)p.H &&
                    (unsigned)ix < (unsigned)p.W;
    tab[ii * 64 + lane] = ok ? (((im * p.H + iy) * p.W + ix) * p.C + 4 * hh) * 4 : (int)W4_OOB;
  }

  w4_stamp(dbg, 1);
  // ---- this lane's tile (A row r): unit of patch pixel (dy, dx) = u0 + dy * pitch + w4_dxu(dx); the
  // wave reads patch rows H .. H + 4
  const int t = tw0 + r;
  const bool tok = t < p.T;
  const int tsg = tok ? w4_div(t, rtw) - R0 : 0;
  int pitch_t = seg_pitch[0], lo_t = seg_lo[0], base_t = seg_base[0];
#pragma unroll
  for (int k = 1; k < W4_MAXSEG; ++k) {
    pitch_t = tsg == k ? seg_pitch[k] : pitch_t;
    lo_t = tsg == k ? seg_lo[k] : lo_t;
    base_t = tsg == k ? seg_base[k] : base_t;
  }
  const int cgl = tok ? t - (R0 + tsg) * p.TW - lo_t : 0;
  const int prs = pitch_t * 16;                                        // bytes per patch row
  const int prd = (base_t + 9 * cgl + (q >> 1)) * 16 + 8 * (q & 1) + H * prs;

  auto read_patch = [&](f32x2 (&d)[30], int buf, int pix) {   // pix = local row * 6 + dx
    const int row = pix / 6, dx = pix - 6 * (pix / 6);
    d[pix] = *(const f32x2*)(imgb + buf * IMG + prd + row * prs + 16 * w4_dxu(dx));
  };
  const int wvoff = (wave * WPW * 256 + lane * 4) * 4; // this lane's bytes in the wave's weight pieces
  auto issue_w = [&](int kc, int slot, int i) {       // weight piece i of chunk kc -> ring slot
    w4_dma(wvoff, udesc, kc * (WCH * 4) + i * 1024, smem_lds + slot * SLOT + (wave * WPW + i) * 1024);
  };
  auto issue_x = [&](int kc, int buf, int ii, int off) {   // this wave's image piece ii of chunk kc
    w4_dma(off, xdesc, kc * 32, imgb_lds + buf * IMG + (2 * ii + H) * 1024);
  };
  constexpr bool LAST_SHORT = (PIECES & 1) && H == 1; // the pair's odd piece belongs to wave 0
  auto issue_img = [&](int kc, int buf) {
#pragma unroll
    for (int ii = 0; ii < HP; ++ii)
      if (!(LAST_SHORT && ii == HP - 1)) issue_x(kc, buf, ii, tab[ii * 64 + lane]);
  };
  // the transform of a fresh patch (30 float2: patch rows H .. H + 4) into this wave's 18 positions
  auto transform = [&](f32x2 (&d)[30], f32x2 (&v)[18]) {
#pragma unroll
    for (int row = 0; row < 5; ++row) w4_row(d, row);
#pragma unroll
    for (int pb = 0; pb < 6; ++pb) w4_colh<H>(d, v, pb);
  };

  f32x4 acc[18][W4_FN];
#pragma unroll
  for (int i = 0; i < 18; ++i)
#pragma unroll
    for (int j = 0; j < W4_FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  f32x2 vA[18], vB[18];

  // ---- prologue: chunk k0's weights (slot 0) and image (buffer 0), chunk k0 + 1's image (buffer 1)
  {
#pragma unroll
    for (int i = 0; i < WPW; ++i) issue_w(k0, 0, i);
    issue_img(k0, 0);
    issue_img(k0 + 1, 1);                            // kper >= 2
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();                                 // the partner's image pieces too
    f32x2 d[30];
#pragma unroll
    for (int pix = 0; pix < 30; ++pix) read_patch(d, 0, pix);
    transform(d, vA);
    if (dbg) {
#pragma unroll
      for (int i = 0; i < 18; ++i) asm volatile("" : "+v"(vA[i]));
      w4_stamp(dbg, 2);
    }
  }

  // ---- one chunk: MFMAs on vc (chunk kc, transformed) with ring slot kc & 1; meanwhile the weights of
  // kc + 1 go to the other slot, the image buffer kc & 1 (read during chunk kc - 1) refills with kc + 2,
  // and the patch of kc + 1 (buffer (kc + 1) & 1) is read and transformed into vn.  Past the split's last
  // chunk the DMAs reload chunk kc (harmless, in bounds).
  const char* const ringr = smem + lane * 16 + H * 18 * 1024;   // this wave's positions 18 H ..
  auto body = [&](f32x2 (&vc)[18], f32x2 (&vn)[18], int kc, int slot) {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();                   // every wave's pieces of kc (weights) and of kc + 1
    asm volatile("" ::: "memory");                  // (image) have landed; slot kc + 1 & image kc are free
    const int kw = kc + 1 < k1 ? kc + 1 : kc;
    const int kx = kc + 2 < k1 ? kc + 2 : kc;
    const char* sl = ringr + slot * SLOT;
    f32x4 u[2];
    int toff[HP];
    f32x2 d[30];
    u[0] = *(const f32x4*)(sl);
#pragma unroll
    for (int g = 0; g < 18; ++g) {
      if (g < 17) u[(g + 1) & 1] = *(const f32x4*)(sl + (g + 1) * 1024);
      if (g < HP) toff[g] = tab[g * 64 + lane];
      if constexpr (EXP & 8) {
        // one DMA per group: weight piece i in group 2 i, image piece ii in group 2 ii + 1 (the 9th / 10th
        // image pieces double up in groups 16 / 14); patch reads 3 per group (groups 0-9); row r's
        // transform in groups 2 r + 3 (channel 0) and 2 r + 4 (channel 1), column pb in group 12 + pb
        if (!(EXP & 1) && (g & 1) == 0 && g / 2 < WPW) issue_w(kw, slot ^ 1, g / 2);
        constexpr int ii_of[18] = {-1, 0, -1, 1, -1, 2, -1, 3, -1, 4, -1, 5, -1, 6, 9, 7, 8, -1};
        const int ii = ii_of[g];
        if (!(EXP & 2) && ii >= 0 && ii < HP && !(LAST_SHORT && ii == HP - 1)) issue_x(kx, slot, ii, toff[ii]);
        if (g < 10) {
#pragma unroll
          for (int e = 0; e < 3; ++e) read_patch(d, slot ^ 1, 3 * g + e);
        }
        if (!(EXP & 4) && g >= 3 && g < 13) {
          const int row = (g - 3) >> 1, c = (g - 3) & 1;
          w4_row1(d, row, c);
#pragma unroll
          for (int k = 0; k < 6; ++k) {
            float t = d[row * 6 + k][c];
            asm volatile("" : "+v"(t));
            d[row * 6 + k][c] = t;
          }
        }
      } else {
        if (!(EXP & 1) && g < WPW) issue_w(kw, slot ^ 1, g);
        if (!(EXP & 2) && g >= 2 && g < 2 + HP && !(LAST_SHORT && g - 2 == HP - 1))
          issue_x(kx, slot, g - 2, toff[g - 2]);
        if (g < 8) {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (4 * g + e < 30) read_patch(d, slot ^ 1, 4 * g + e);
        }
        if (!(EXP & 4) && g >= 3 && g < 8) w4_row(d, g - 3);
      }
      constexpr int COL0 = (EXP & 8) ? 12 : 9;
      if (g >= COL0 && g < COL0 + 6) {
        const int pb = g - COL0;
        if constexpr (EXP & 4) {
#pragma unroll
          for (int a = 0; a < 3; ++a) vn[a * 6 + pb] = d[a * 6 + pb] + d[(a + 2) * 6 + pb];
        } else {
          w4_colh<H>(d, vn, pb);
        }
        // pin the finished column here: left alone, the compiler sinks the transform into the next
        // chunk (where vn is consumed), i.e. behind the barrier, in front of its MFMAs
#pragma unroll
        for (int a = 0; a < 3; ++a) asm volatile("" : "+v"(vn[a * 6 + pb]));
      }
      const f32x2 a = vc[g];
      const f32x4 b = u[g & 1];
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int j = 0; j < W4_FN; ++j)
          acc[g][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b[2 * j + s], acc[g][j], 0, 0, 0);
      // one group per scheduling region: left free, the scheduler hoists the chunk's fragment reads to
      // its top (VGPRs the accumulators need)
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  for (int kc = k0; kc < k1; kc += 2) {
    body(vA, vB, kc, 0);
    body(vB, vA, kc + 1, 1);
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");   // the last chunk's spare DMA has landed
  w4_stamp(dbg, 3);
  __syncthreads();                                   // every wave is done with the ring and the images

  // ---- partial output transform: Y_H = A^T[:, 3H..3H+2] M[3H..3H+2][:] A, staged per wave as
  // [16 tiles][16 pixels][32 channels] (32 KiB)
  float* const st = (float*)(smem + wave * 32768);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < W4_FN; ++j) {
      float w[4][6];
#pragma unroll
      for (int pb = 0; pb < 6; ++pb) {
        const float m0 = acc[0 * 6 + pb][j][i], m1 = acc[1 * 6 + pb][j][i], m2 = acc[2 * 6 + pb][j][i];
        if constexpr (H == 0) {      // A^T columns 0-2: (1 0 0 0), (1 1 1 1), (1 -1 1 -1)
          const float s12 = m1 + m2, d12 = m1 - m2;
          w[0][pb] = m0 + s12;
          w[1][pb] = d12;
          w[2][pb] = s12;
          w[3][pb] = d12;
        } else {                     // A^T columns 3-5: (1 2 4 8), (1 -2 4 -8), (0 0 0 1)
          const float s34 = m0 + m1, d34 = m0 - m1;
          w[0][pb] = s34;
          w[1][pb] = 2.f * d34;
          w[2][pb] = 4.f * s34;
          w[3][pb] = fmaf(8.f, d34, m2);
        }
      }
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        float o[4];
        w4_at(w[a], o);
#pragma unroll
        for (int b = 0; b < 4; ++b) st[((4 * q + i) * 16 + a * 4 + b) * 32 + 16 * j + r] = o[b];
      }
    }
  w4_stamp(dbg, 4);
  __syncthreads();                                   // the pair's partials are both staged
  // read-back: wave H of the pair takes passes it = 16 H .. 16 H + 15 of its tile group; pass it covers
  // tile it / 2, pixels 8 (it & 1) .. + 7, 8 lanes (16 B each) per pixel; Y = Y_0 + Y_1 in that order
  const float* const st0 = (const float*)(smem + (wave & ~1) * 32768);
  const float* const st1 = st0 + 8192;
  const int c8 = lane & 7, pxl = lane >> 3;
  int bidx = cg * 32 + c8 * 4;
  asm volatile("" : "+v"(bidx));                     // keep the bias load below the K loop
  const bool split = ns > 1;
  const bool fused = split && p.counters != nullptr;
  const int MN = p.B * p.H * p.W * p.N;
  const f32x4 bsv = *(const f32x4*)(p.bias + bidx);   // finish(): whole K, or the fused split's last block
  const int tpi = p.TH * p.TW;
  int oo[16];                                        // NHWC offset of each float4 this lane owns (-1: outside)
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int it = 16 * H + k;
    const int tl = it >> 1, px = (it & 1) * 8 + pxl;
    const int tt = tw0 + tl;                         // wave-uniform
    const int im = tt / tpi, rr = tt - im * tpi;
    const int ty = rr / p.TW, tx = rr - ty * p.TW;
    const int oy = 4 * ty + (px >> 2), ox = 4 * tx + (px & 3);
    oo[k] = (tt < p.T && oy < p.H && ox < p.W) ? ((im * p.H + oy) * p.W + ox) * p.N + bidx : -1;
  }
  auto own = [&](int k) -> f32x4 {
    const int it = 16 * H + k;
    const int o = ((it >> 1) * 16 + (it & 1) * 8 + pxl) * 32 + c8 * 4;
    return *(const f32x4*)(st0 + o) + *(const f32x4*)(st1 + o);
  };
  auto finish = [&](int k, f32x4 v) {
    const int o = oo[k];
    v += bsv;
    if (p.res) v += *(const f32x4*)(p.res + o);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = act_relu(v[e], p.relu);
    *(f32x4*)(p.out + o) = v;
  };
  if (!split) {
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (oo[k] >= 0) finish(k, own(k));
    if (dbg) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      w4_stamp(dbg, 5);
      if (lane == 0) dbg[7] = __builtin_amdgcn_s_memrealtime();
    }
    return;
  }
  const __amdgpu_buffer_rsrc_t wsr = w4_rsrc(p.ws);
  if (!fused) {                                      // plain split-K: slab zs, splitk_reduce_f32 finishes
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (oo[k] >= 0) *(f32x4*)(p.ws + (size_t)zs * MN + oo[k]) = own(k);
    return;
  }
  // fused split-K: publish this split's partials write-through (sc1), count the arrival; the last split
  // of the block adds every slab in split order (deterministic whoever arrives last), then bias /
  // residual / ReLU (MI355X_MICROARCH.md inter-workgroup hand-off, first table row)
#pragma unroll
  for (int k = 0; k < 16; ++k)
    if (oo[k] >= 0)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, own(k)), wsr, (zs * MN + oo[k]) * 4, 0,
                                             W4_CPOL_SC1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* const flag = (int*)(smem + LDS - 16);         // past the staging regions (static_assert in the kernel)
  if (threadIdx.x == 0) {
    int* ctr = p.counters + blockIdx.x + gridDim.x * blockIdx.y;
    const int old = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == ns - 1;
    if (last) __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = last;
  }
  __syncthreads();
  if (!*flag) return;
#pragma unroll 4
  for (int k = 0; k < 16; ++k) {
    const int o = oo[k];
    f32x4 v = (f32x4){0.f, 0.f, 0.f, 0.f};
    for (int z = 0; z < ns; ++z)
      v += z == zs ? own(k)
                   : __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(wsr, (z * MN + max(o, 0)) * 4,
                                                                                     0, W4_CPOL_SC1));
    if (o >= 0) finish(k, v);
  }
}

// EXP (measurement variants, tools/wino4_timeline.py --exp): bit 0 no weight DMA in the K loop, bit 1 no image
// DMA, bit 2 no input transform (wrong results: timing attribution only); bit 3 the spread schedule
template <int PIECES, int EXP>
__global__ __launch_bounds__(256, 1) void conv_wino4_f32_kernel(WinoF32Params p) {
  constexpr int HP = (PIECES + 1) / 2;
  constexpr int LDS = 2 * W4_SLOT + 4 * PIECES * 1024 + W4_NW * HP * 256;
  static_assert(LDS >= W4_NW * 32768 + 16, "the output staging needs 32 KiB per wave (+ the fixup flag)");
  static_assert(LDS <= 163840, "LDS: at most 19 image pieces");
  __shared__ __attribute__((aligned(16))) char smem[LDS];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (wave & 1) wino4_wave<PIECES, 1, EXP>(p, smem, wave);
  else wino4_wave<PIECES, 0, EXP>(p, smem, wave);
}

// 16-B units of a tile group's image for tiles tw0 .. tw0 + 15 (host mirror of the kernel's layout)
int w4_wave_units(int tw0, int T, int TW, bool align) {
  if (tw0 >= T) return 0;
  const int tlast = tw0 + 15 < T - 1 ? tw0 + 15 : T - 1;
  const int R0 = tw0 / TW, R1 = tlast / TW;
  int units = 0, r0 = 0;
  for (int R = R0; R <= R1; ++R) {
    const int lo = R == R0 ? tw0 - R0 * TW : 0;
    const int hi = R == R1 ? tlast - R1 * TW : TW - 1;
    units += 6 * (9 * (hi - lo + 1) + 4);
    r0 += hi - lo + 1;
    if (align && R < R1) units += (9 * r0 - units) & 15;
  }
  return units;
}

template <int PIECES, int EXP = 0>
hipError_t launch_wino4(const WinoF32Params& p, int ns, hipStream_t s) {
  const dim3 grid((p.T + 31) / 32, p.N / (16 * W4_FN), ns), block(W4_NW * 64);   // 2 tile groups per block
  hipLaunchKernelGGL((conv_wino4_f32_kernel<PIECES, EXP>), grid, block, 0, s, p);
  return hipGetLastError();
}

}  // namespace

// image pieces (1 KiB each) the widest tile group of a Winograd F(4x4) launch stages, and whether its
// segment bases are bank-aligned (preferred when it still fits); 0: the geometry is not supported (a tile
// row narrower than 2 tiles, or more than 19 pieces)
int conv_wino4_pieces(int B, int H, int W, int* align) {
  const int TH = (H + 3) / 4, TW = (W + 3) / 4, T = B * TH * TW;
  if (TW < 2 || T >= (1 << 20)) return 0;
  for (int a = 1; a >= 0; --a) {
    int mx = 0;
    for (int tw0 = 0; tw0 < T; tw0 += 16) {
      const int u = w4_wave_units(tw0, T, TW, a);
      mx = u > mx ? u : mx;
    }
    const int pieces = (mx + 63) / 64 < 15 ? 15 : (mx + 63) / 64;
    if (pieces <= 19) {
      if (align) *align = a;
      return pieces;
    }
  }
  return 0;
}

bool conv_wino4_f32_ok(int C, int N) { return C % 16 == 0 && N % 32 == 0; }

// F(4x4, 3x3): p.TH / TW / T count 4x4 tiles; ksplit: |splits| (the fused fixup when p.counters is set)
static unsigned long long* g_wino4_dbg = nullptr;
static int g_wino4_exp = 0;
unsigned long long* wino4_debug_buffer() { return g_wino4_dbg; }
int wino4_exp_flags() { return g_wino4_exp; }
void wino4_set_debug(unsigned long long* buf, int exp) {
  g_wino4_dbg = buf;
  g_wino4_exp = exp;
}

template <int PIECES>
hipError_t launch_wino4_exp(const WinoF32Params& p, int ns, hipStream_t s, int exp) {
  switch (exp) {
    case 1: return launch_wino4<PIECES, 1>(p, ns, s);
    case 2: return launch_wino4<PIECES, 2>(p, ns, s);
    case 3: return launch_wino4<PIECES, 3>(p, ns, s);
    case 4: return launch_wino4<PIECES, 4>(p, ns, s);
    case 7: return launch_wino4<PIECES, 7>(p, ns, s);
    case 8: return launch_wino4<PIECES, 8>(p, ns, s);
    case 9: return launch_wino4<PIECES, 9>(p, ns, s);
    case 10: return launch_wino4<PIECES, 10>(p, ns, s);
    case 12: return launch_wino4<PIECES, 12>(p, ns, s);
  }
  return hipErrorInvalidValue;
}

hipError_t conv_wino4_f32_launch(const WinoF32Params& p_in, hipStream_t s) {
  WinoF32Params p = p_in;
  p.dbg = g_wino4_dbg;
  const int KC = p.C / 8;
  const int ns = p.ksplit;
  if (p.C % 16 || p.N % 32 || ns < 1 || KC % ns || (KC / ns) % 2 || p.sk_iters > 0) return hipErrorInvalidValue;
  if (p.TH != (p.H + 3) / 4 || p.TW != (p.W + 3) / 4 || p.T != p.B * p.TH * p.TW) return hipErrorInvalidValue;
  if (ns > 1 && (!p.ws || (size_t)ns * p.B * p.H * p.W * p.N * 4 > 0x7fffffffu)) return hipErrorInvalidValue;
  if ((size_t)p.B * p.H * p.W * p.C * 4 >= 0x7fffffffu) return hipErrorInvalidValue;   // 31-bit DMA offsets
  int align = 0;
  const int pieces = conv_wino4_pieces(p.B, p.H, p.W, &align);
  p.flags = align;
  if (g_wino4_exp) {                                 // measurement variants: stages 1 / 2 geometries only
    if (pieces == 15) return launch_wino4_exp<15>(p, ns, s, g_wino4_exp);
    if (pieces == 16) return launch_wino4_exp<16>(p, ns, s, g_wino4_exp);
    return hipErrorInvalidValue;
  }
  switch (pieces) {
    case 15: return launch_wino4<15>(p, ns, s);
    case 16: return launch_wino4<16>(p, ns, s);
    case 17: return launch_wino4<17>(p, ns, s);
    case 18: return launch_wino4<18>(p, ns, s);
    case 19: return launch_wino4<19>(p, ns, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace adapt
