// 3x3 / stride-1 / pad-1 convolution with an LDS halo patch ("v3").
//
// The implicit-GEMM kernels (conv_glds.hip) fetch the im2col A operand: every
// input pixel is gathered 9 times, once per filter tap, and on MI355X the 3x3
// layers are bound by that L2 -> LDS traffic (profiles/pmc_conv3_3x3_cfg22.txt:
// TCC 72 % busy, MFMA ~25 %).  Here a block owns TH whole output rows of one
// image (M tile = TH*OW pixels) and, per 64-channel input slice, stages the
// (TH+2) x (OW+2) input patch in LDS ONCE; the 9 taps then read shifted windows
// of it.  Only the weights still stream per (slice, tap).  A traffic drops ~6x.
//
// * patch rows/cols outside the image are fetched from a 16-byte zero page, so
//   the padding is implicit and the DMA needs no mask;
// * patch image: pixel q at q*128 B, its eight 16-byte channel chunks XOR-
//   swizzled by (q >> 1) & 7 (conflict-free MFMA fragment reads: consecutive
//   output pixels are consecutive patch pixels within a row);
// * LDS-DMA (`global_load_lds`, 16 B/lane) for both the patch (double
//   buffered across slices) and the STAGES-deep weight ring; the wait counts
//   are compile-time constants (the A issue sits at tap 0 of every slice);
// * fused epilogue of the other conv kernels (bias = folded BN, residual, ReLU).
#include "epilogue.h"
#include "kernels.h"

namespace adapt {

typedef __attribute__((address_space(3))) void lds3_void;

namespace {
__device__ __forceinline__ int swzq(int q, int c) { return q * 128 + ((c ^ ((q >> 1) & 7)) << 4); }
template <int N> __device__ __forceinline__ void hwait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
}  // namespace

// WM x WN waves, each FM x FN 16x16 fragments; LA patch pieces (8 pixels each)
// per wave per slice; STAGES-deep weight ring.
template <int WM, int WN, int FM, int FN, int LA, int STAGES, bool ILV, bool OUT_F32>
__global__ __launch_bounds__(WM * WN * 64, 1) void conv_halo_kernel(ConvParams p, const bf16* __restrict__ zero) {
  constexpr int NW = WM * WN, NT = NW * 64;
  constexpr int BM = WM * FM * 16, BN = WN * FN * 16;
  constexpr int LB = BN / (8 * NW);                 // weight pieces per wave per (slice, tap)
  // The next slice's patch is spread over the last NTA = 10 - STAGES taps of the
  // current slice (iterations that run after the last read of the buffer it
  // overwrites, the slice before), LT pieces per tap; the other taps issue
  // dummy zero-page pieces into a landing zone, so every iteration issues the
  // same LB + LT pieces, the loop body stays one basic block, and the whole
  // patch is older than the weight tile waited for at the next slice's tap 0.
  constexpr int NTA = 10 - STAGES;
  constexpr int LT = (LA + NTA - 1) / NTA;
  constexpr int LPI = LB + LT;                      // pieces per wave per iteration
  constexpr int PATCH_PIX = LA * NW * 8;            // patch capacity (pixels)
  constexpr int PATCH_BYTES = (NTA + 1) * LT * NW * 1024;   // incl. one shared landing zone for dummies
  constexpr int B_BYTES = BN * 128;
  constexpr int EPI_LD = BN + 4;
  constexpr int MAIN_BYTES = 2 * PATCH_BYTES + STAGES * B_BYTES;
  constexpr int EPI_BYTES = BM * EPI_LD * 4;
  constexpr int LDS_BYTES = MAIN_BYTES > EPI_BYTES ? MAIN_BYTES : EPI_BYTES;
  static_assert(LB * 8 * NW == BN && LB >= 1, "weight tile split");
  static_assert(LDS_BYTES <= 160 * 1024, "LDS");
  static_assert(STAGES >= 2 && STAGES <= 8, "stages (A issue must be older than the waited B)");
  static_assert((STAGES - 2) * LPI <= 63, "vmcnt range");
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
  char* patch0 = smem;
  char* ring = smem + 2 * PATCH_BYTES;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int fr = lane & 15, fq = lane >> 4;

  // ---- tile: TH output rows of one image x BN output channels (n fastest)
  const int TH = p.th;
  const int rtiles = (p.OH + TH - 1) / TH;
  const int tilesN = (p.N + BN - 1) / BN;
  const int tile = xcd_remap(blockIdx.x, p.B * rtiles * tilesN);
  const int tn = tile % tilesN, tmr = tile / tilesN;
  const int img = tmr / rtiles, oh0 = (tmr - img * rtiles) * TH;
  const int n0 = tn * BN;
  const int PW = p.OW + 2;                            // patch row pitch (pixels)
  const int rows_here = min(TH, p.OH - oh0);
  const int npix = (rows_here + 2) * PW;              // patch pixels in use
  const int m0 = (img * p.OH + oh0) * p.OW;
  const int m_end = m0 + rows_here * p.OW;
  const int nslices = p.Cin >> 6;
  const int total = nslices * 9;                      // (slice, tap) iterations

  // ---- patch DMA bookkeeping: lane -> (patch pixel, physical chunk)
  const int lpix = lane >> 3, pchunk = lane & 7;
  const bf16* a_src[LA];                              // slice-0 source (or null = zero page)
#pragma unroll
  for (int i = 0; i < LA; ++i) {
    const int q = (wave + NW * i) * 8 + lpix;
    const int c = pchunk ^ ((q >> 1) & 7);
    a_src[i] = nullptr;
    if (q < npix) {
      const int pr = q / PW, pc = q - pr * PW;
      const int ih = oh0 - 1 + pr, iw = pc - 1;
      if ((unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W)
        a_src[i] = p.x + (((size_t)img * p.H + ih) * p.W + iw) * p.Cin + c * 8;
    }
  }
  // the LT pieces that iteration (slice', tap) issues for the patch of `slice`
  // (= slice' + 1) into buffer `buf`: live pieces at taps >= STAGES-1
  auto issue_patch_part = [&](int slice, int buf, int tap) {
    char* dst = patch0 + buf * PATCH_BYTES;
    const bool live = slice < nslices && tap >= STAGES - 1;
    const int i0 = tap >= STAGES - 1 ? (tap - (STAGES - 1)) * LT : NTA * LT;
#pragma unroll
    for (int k = 0; k < LT; ++k) {
      const int i = i0 + k;                           // wave-uniform piece index
      const bf16* s = zero;
#pragma unroll
      for (int ii = 0; ii < LA; ++ii)
        if (ii == i && live && a_src[ii] != nullptr) s = a_src[ii] + slice * 64;   // i >= LA: dummy
      __builtin_amdgcn_global_load_lds((const void*)s, (lds3_void*)(dst + (wave + NW * i) * 1024), 16, 0, 0);
    }
  };
  const bf16* b_src[LB];
#pragma unroll
  for (int i = 0; i < LB; ++i) {
    const int r = (wave * LB + i) * 8 + lpix;
    b_src[i] = p.w + (size_t)(n0 + r) * p.Kpad + (pchunk ^ ((r >> 1) & 7)) * 8;
  }
  // weights of iteration `it` = (slice, tap): k offset tap*Cin + slice*64
  auto issue_b = [&](int it, int slot) {
    char* dst = ring + slot * B_BYTES;
    const bool live = it < total;
    const int slice = it / 9, tap = it - slice * 9;
    const int koff = tap * p.Cin + slice * 64;
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const bf16* s = live ? b_src[i] + koff : zero;
      __builtin_amdgcn_global_load_lds((const void*)s, (lds3_void*)(dst + (wave * LB + i) * 1024), 16, 0, 0);
    }
  };

  // ---- A fragment rows: output pixel -> patch pixel of the (0,0) tap
  int qbase[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int pix = wm * FM * 16 + i * 16 + fr;
    const int r = pix / p.OW, col = pix - r * p.OW;
    qbase[i] = pix < rows_here * p.OW ? r * PW + col : 0;
  }

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // prologue: the whole patch of slice 0, then the first STAGES-1 weight tiles
  // (each with its LT companion pieces: dummies, taps 0..STAGES-2)
#pragma unroll
  for (int i = 0; i < LA; ++i) {
    const bf16* s = a_src[i] != nullptr ? a_src[i] : zero;
    __builtin_amdgcn_global_load_lds((const void*)s, (lds3_void*)(patch0 + (wave + NW * i) * 1024), 16, 0, 0);
  }
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s) {
    issue_b(s, s);
    issue_patch_part(1, 1, s);
  }

  constexpr int MT = 2 * FM * FN;
  for (int it = 0; it < total; ++it) {
    const int slice = it / 9, tap = it - slice * 9;
    // B(it) must have landed (and with it everything issued earlier: the
    // patch of this slice); STAGES-2 later iterations' pieces stay in flight
    hwait_vm<(STAGES - 2) * LPI>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int nit = it + STAGES - 1;                  // iteration whose pieces are issued now
    const int nslice = nit / 9, ntap = nit - nslice * 9;
    if constexpr (!ILV) {
      issue_b(nit, nit % STAGES);
      issue_patch_part(nslice + 1, (nslice + 1) & 1, ntap);
    }
    const char* pa = patch0 + (slice & 1) * PATCH_BYTES;
    const char* pb = ring + (it % STAGES) * B_BYTES;
    const int kh = tap / 3, kw = tap - kh * 3;
    const int toff = kh * PW + kw;
    bf16x8 af[2][FM], bfr[2][FN];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int i = 0; i < FM; ++i) af[ks][i] = *(const bf16x8*)(pa + swzq(qbase[i] + toff, ks * 4 + fq));
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int r = wn * FN * 16 + j * 16 + fr;
        bfr[ks][j] = *(const bf16x8*)(pb + r * 128 + (((ks * 4 + fq) ^ ((r >> 1) & 7)) << 4));
      }
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks][i], bfr[ks][j], acc[i][j], 0, 0, 0);
    if constexpr (ILV) {
      issue_b(nit, nit % STAGES);
      issue_patch_part(nslice + 1, (nslice + 1) & 1, ntap);
      constexpr int MPP = MT / LPI > 0 ? MT / LPI : 1;
      __builtin_amdgcn_sched_group_barrier(0x100, 2 * (FM + FN), 0);   // ds_read
#pragma unroll
      for (int q = 0; q < LPI; ++q) {
        __builtin_amdgcn_sched_group_barrier(0x008, MPP, 0);          // MFMA
        __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);            // VMEM (LDS-DMA piece)
      }
      __builtin_amdgcn_sched_group_barrier(0x008, MT, 0);
    }
  }
  hwait_vm<0>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  float* epi = (float*)smem;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int col = wn * FN * 16 + j * 16 + fr;
#pragma unroll
      for (int r = 0; r < 4; ++r) epi[(wm * FM * 16 + i * 16 + fq * 4 + r) * EPI_LD + col] = acc[i][j][r];
    }
  __syncthreads();
  fused_epilogue<BM, BN, NT, EPI_LD, OUT_F32>(p, epi, m0, n0, tid, m_end);
}

__device__ __attribute__((aligned(64))) bf16 g_halo_zero[64];

// v3 configs: id -> WM, WN, FM, FN, LA, STAGES  (tile BM = WM*FM*16 pixels, BN = WN*FN*16)
#define ADAPT_HALO_CFGS(X)              \
  X(40, 2, 2, 7, 2, 11, 4, false)       \
  X(41, 1, 4, 7, 2, 6, 4, false)        \
  X(42, 2, 2, 7, 2, 9, 4, false)        \
  X(43, 1, 4, 4, 2, 3, 4, false)        \
  X(44, 1, 2, 7, 2, 9, 4, false)        \
  X(45, 2, 4, 7, 1, 6, 4, false)        \
  X(46, 2, 2, 7, 2, 11, 4, true)        \
  X(47, 1, 4, 7, 2, 6, 4, true)         \
  X(48, 2, 4, 7, 1, 6, 4, true)         \
  X(49, 1, 4, 4, 2, 3, 4, true)         \
  X(50, 2, 4, 7, 1, 5, 4, true)         \
  X(51, 2, 2, 7, 2, 9, 4, true)         \
  X(52, 1, 2, 7, 2, 9, 4, true)

bool conv_halo_cfg(int cfg, int* bm, int* bn, int* patch_pix) {
  switch (cfg) {
#define X(id, WM_, WN_, FM_, FN_, LA_, S_, I_)                 \
  case id:                                                     \
    *bm = WM_ * FM_ * 16;                                      \
    *bn = WN_ * FN_ * 16;                                      \
    *patch_pix = LA_ * WM_ * WN_ * 8;                          \
    return true;
    ADAPT_HALO_CFGS(X)
#undef X
  }
  return false;
}

template <int WM, int WN, int FM, int FN, int LA, int S, bool ILV>
static hipError_t launch_halo(const ConvParams& p, hipStream_t s, bool out_f32) {
  static bf16* zero = nullptr;
  if (!zero) {
    hipError_t e = hipGetSymbolAddress((void**)&zero, HIP_SYMBOL(g_halo_zero));
    if (e != hipSuccess) return e;
  }
  constexpr int BM = WM * FM * 16, BN = WN * FN * 16, PATCH_PIX = LA * WM * WN * 8;
  if (p.KH != 3 || p.KW != 3 || p.stride != 1 || p.pad_t != 1 || p.pad_l != 1 || p.Cin % 64 || p.th < 1 ||
      p.th * p.OW > BM || (p.th + 2) * (p.OW + 2) > PATCH_PIX || p.OH != p.H || p.OW != p.W || p.ksplit != 1)
    return hipErrorInvalidValue;
  const int tiles = p.B * ((p.OH + p.th - 1) / p.th) * ((p.N + BN - 1) / BN);
  dim3 grid(tiles), block(WM * WN * 64);
  if (out_f32) hipLaunchKernelGGL((conv_halo_kernel<WM, WN, FM, FN, LA, S, ILV, true>), grid, block, 0, s, p, zero);
  else hipLaunchKernelGGL((conv_halo_kernel<WM, WN, FM, FN, LA, S, ILV, false>), grid, block, 0, s, p, zero);
  return hipGetLastError();
}

hipError_t conv_halo_launch(const ConvParams& p, int cfg, hipStream_t s, bool out_f32) {
  switch (cfg) {
#define X(id, WM_, WN_, FM_, FN_, LA_, S_, I_) case id: return launch_halo<WM_, WN_, FM_, FN_, LA_, S_, I_>(p, s, out_f32);
    ADAPT_HALO_CFGS(X)
#undef X
  }
  return hipErrorInvalidValue;
}

}  // namespace adapt
