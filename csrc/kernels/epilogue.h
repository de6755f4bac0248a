// Fused conv epilogue shared by the implicit-GEMM kernels:
//   out[m][n] = act(tile[m][n] + bias[n] (+ res[m][n]))   (bf16 or fp32 out)
// over a BM x BN fp32 tile staged in LDS (row stride EPI_LD), written as 16-byte
// row segments; rows m >= m_end are not written.
//
// Latency: one block per CU is the common case, so nothing hides a dependent
// global load here.  A thread's column chunk is the same for all its
// iterations (NT % (BN/8) == 0): the bias is loaded once, and the residual
// loads of a group of EPI_G iterations are all issued before the first one is
// used — EPI_G round trips collapse into one (the serial loop used to pay one
// HBM latency per 16-byte chunk).
#pragma once
#include "kernels.h"

namespace adapt {

// Residual chunks of this thread's epilogue iterations, loaded BEFORE the main
// loop so their HBM latency overlaps the GEMM (the small-K 1x1 "_3" convs of
// ResNet spend a large share of each block in that epilogue round trip).
template <int BM, int BN, int NT>
struct EpiRes {
  static constexpr int CPR = BN / 8, NCH = BM * CPR, RPI = NT / CPR, IT = (NCH + NT - 1) / NT;
  V8 r[IT];
  __device__ __forceinline__ void prefetch(const ConvParams& p, int m0, int n0, int tid, int m_end) {
    const int cc = tid % CPR, row0 = tid / CPR;
    const int n = n0 + cc * 8;
#pragma unroll
    for (int u = 0; u < IT; ++u) {
      const int row = row0 + u * RPI, m = m0 + row;
      r[u].u = (u32x4){0u, 0u, 0u, 0u};
      if (p.res && n < p.N && row < BM && m < m_end) r[u].u = *(const u32x4*)(p.res + (size_t)m * p.N + n);
    }
  }
};

template <int BM, int BN, int NT, int EPI_LD, bool OUT_F32>
__device__ __forceinline__ void fused_epilogue(const ConvParams& p, const float* epi, int m0, int n0, int tid,
                                               int m_end, const EpiRes<BM, BN, NT>* rp = nullptr,
                                               bool use_pre = false) {
  constexpr int CPR = BN / 8;                 // 8-wide chunks per row
  constexpr int NCH = BM * CPR;
  constexpr int RPI = NT / CPR;               // rows covered per iteration
  constexpr int IT = (NCH + NT - 1) / NT;
  constexpr int EPI_G = IT < 4 ? IT : 4;
  static_assert(NT % CPR == 0, "column chunk must be iteration-invariant");
  const int cc = tid % CPR, row0 = tid / CPR;
  const int n = n0 + cc * 8;
  if (n >= p.N) return;
  const EpiDst d = epi_dst(p, n);             // n_split is a multiple of 8: one destination per chunk
  float b[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) b[t] = 0.f;
  if (p.bias) {
    const f32x4 b0 = *(const f32x4*)(p.bias + n), b1 = *(const f32x4*)(p.bias + n + 4);
    b[0] = b0[0]; b[1] = b0[1]; b[2] = b0[2]; b[3] = b0[3];
    b[4] = b1[0]; b[5] = b1[1]; b[6] = b1[2]; b[7] = b1[3];
  }
#pragma unroll
  for (int g = 0; g < IT; g += EPI_G) {
    V8 r[EPI_G];
#pragma unroll
    for (int u = 0; u < EPI_G; ++u) {
      const int row = row0 + (g + u) * RPI;
      const int m = m0 + row;
      r[u].u = (u32x4){0u, 0u, 0u, 0u};
      if (use_pre) {
        if (g + u < IT) r[u] = rp->r[g + u];       // compile-time index: stays in registers
      } else if (p.res && g + u < IT && row < BM && m < m_end) {
        r[u].u = *(const u32x4*)(p.res + (size_t)m * p.N + n);
      }
    }
#pragma unroll
    for (int u = 0; u < EPI_G; ++u) {
      const int row = row0 + (g + u) * RPI;
      const int m = m0 + row;
      if (g + u >= IT || row >= BM || m >= m_end) continue;
      const float* e = epi + row * EPI_LD + cc * 8;
      const f32x4 v0 = *(const f32x4*)e, v1 = *(const f32x4*)(e + 4);
      float v[8] = {v0[0] + b[0], v0[1] + b[1], v0[2] + b[2], v0[3] + b[3],
                    v1[0] + b[4], v1[1] + b[5], v1[2] + b[6], v1[3] + b[7]};
      if (p.res) {
#pragma unroll
        for (int t = 0; t < 8; ++t) v[t] += bf2f(r[u].e[t]);
      }
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
}

}  // namespace adapt
