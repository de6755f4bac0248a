// Layers beyond the ResNet set, for the other Keras model families the
// DEFER API can be handed (models/zoo.py: MobileNetV2's DepthwiseConv2D,
// DenseNet's Concatenate + AveragePooling2D).  All three are memory-bound
// streams over bf16 NHWC activations whose channel dim is padded to Cp (a
// multiple of 8, the runtime's 16-byte vector layout): one thread per
// 8-channel chunk of one output pixel, 16-byte loads and stores, fp32 math.
#include "kernels.h"

namespace adapt {

namespace {
__device__ __forceinline__ size_t gstride() { return (size_t)gridDim.x * blockDim.x; }
__device__ __forceinline__ size_t gtid() { return blockIdx.x * (size_t)blockDim.x + threadIdx.x; }
inline unsigned grid_of(size_t n) {
  size_t g = (n + 255) / 256;
  return (unsigned)(g < 8192 ? (g ? g : 1) : 8192);
}
}  // namespace

// Depthwise KHxKW conv (depth multiplier 1): y[b,oh,ow,c] = act(sum_taps x * w[kh][kw][c] + bias[c]),
// BN folded into w/bias on the host; zero padding is implicit (pad_t / pad_l, Keras 'same' or a folded
// ZeroPadding2D).  w: fp32 [KH][KW][Cp].
template <bool GEN>
__global__ __launch_bounds__(256) void dwconv_kernel(const bf16* __restrict__ x, const float* __restrict__ w,
                                                     const float* __restrict__ bias, bf16* __restrict__ y, int B,
                                                     int H, int W, int Cp, int OH, int OW, int KH, int KW,
                                                     int stride, int pad_t, int pad_l, int act) {
  const int cpr = Cp / 8;
  const size_t total = (size_t)B * OH * OW * cpr;
  for (size_t i = gtid(); i < total; i += gstride()) {
    const int c0 = (int)(i % cpr) * 8;
    size_t pix = i / cpr;
    const int ow = (int)(pix % OW);
    pix /= OW;
    const int oh = (int)(pix % OH);
    const int b = (int)(pix / OH);
    float acc[8];
    const f32x4 b0 = *(const f32x4*)(bias + c0), b1 = *(const f32x4*)(bias + c0 + 4);
    acc[0] = b0[0]; acc[1] = b0[1]; acc[2] = b0[2]; acc[3] = b0[3];
    acc[4] = b1[0]; acc[5] = b1[1]; acc[6] = b1[2]; acc[7] = b1[3];
    const int ih0 = oh * stride - pad_t, iw0 = ow * stride - pad_l;
    for (int kh = 0; kh < KH; ++kh) {
      const int ih = ih0 + kh;
      if ((unsigned)ih >= (unsigned)H) continue;
      for (int kw = 0; kw < KW; ++kw) {
        const int iw = iw0 + kw;
        if ((unsigned)iw >= (unsigned)W) continue;
        V8 v;
        v.u = *(const u32x4*)(x + (((size_t)b * H + ih) * W + iw) * Cp + c0);
        const float* wt = w + ((size_t)kh * KW + kw) * Cp + c0;
        const f32x4 w0 = *(const f32x4*)wt, w1 = *(const f32x4*)(wt + 4);
        float xf[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) xf[t] = bf2f(v.e[t]);
        acc[0] += xf[0] * w0[0]; acc[1] += xf[1] * w0[1];
        acc[2] += xf[2] * w0[2]; acc[3] += xf[3] * w0[3];
        acc[4] += xf[4] * w1[0]; acc[5] += xf[5] * w1[1];
        acc[6] += xf[6] * w1[2]; acc[7] += xf[7] * w1[3];
      }
    }
    V8 o;
#pragma unroll
    for (int t = 0; t < 8; ++t) o.e[t] = f2bf(actx<GEN>(acc[t], act));
    *(u32x4*)(y + i * 8) = o.u;
  }
}

// 3x3 specialisation: a thread owns OWG consecutive output pixels of one row and one 8-channel chunk, so
// each input column of the (OWG-1)*S+3 it touches is loaded once per filter row (6 loads per row instead of
// 12 at stride 1, 9 instead of 12 at stride 2) and the row's three weight vectors stay in registers.
template <int S, int OWG, bool GEN>
__global__ __launch_bounds__(256) void dwconv3_kernel(const bf16* __restrict__ x, const float* __restrict__ w,
                                                      const float* __restrict__ bias, bf16* __restrict__ y, int B,
                                                      int H, int W, int Cp, int OH, int OW, int pad_t, int pad_l,
                                                      int act) {
  constexpr int COLS = (OWG - 1) * S + 3;
  const int cpr = Cp / 8;
  const int owg = (OW + OWG - 1) / OWG;
  const size_t total = (size_t)B * OH * owg * cpr;
  for (size_t i = gtid(); i < total; i += gstride()) {
    const int c0 = (int)(i % cpr) * 8;
    size_t pix = i / cpr;
    const int ow0 = (int)(pix % owg) * OWG;
    pix /= owg;
    const int oh = (int)(pix % OH);
    const int b = (int)(pix / OH);
    float acc[OWG][8];
    {
      const f32x4 b0 = *(const f32x4*)(bias + c0), b1 = *(const f32x4*)(bias + c0 + 4);
#pragma unroll
      for (int j = 0; j < OWG; ++j) {
        acc[j][0] = b0[0]; acc[j][1] = b0[1]; acc[j][2] = b0[2]; acc[j][3] = b0[3];
        acc[j][4] = b1[0]; acc[j][5] = b1[1]; acc[j][6] = b1[2]; acc[j][7] = b1[3];
      }
    }
    const int iw0 = ow0 * S - pad_l;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int ih = oh * S - pad_t + kh;
      if ((unsigned)ih >= (unsigned)H) continue;
      float wk[3][8];
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const float* wt = w + ((size_t)kh * 3 + kw) * Cp + c0;
        const f32x4 w0 = *(const f32x4*)wt, w1 = *(const f32x4*)(wt + 4);
        wk[kw][0] = w0[0]; wk[kw][1] = w0[1]; wk[kw][2] = w0[2]; wk[kw][3] = w0[3];
        wk[kw][4] = w1[0]; wk[kw][5] = w1[1]; wk[kw][6] = w1[2]; wk[kw][7] = w1[3];
      }
      const bf16* row = x + ((size_t)b * H + ih) * W * Cp + c0;
#pragma unroll
      for (int c = 0; c < COLS; ++c) {
        const int iw = iw0 + c;
        if ((unsigned)iw >= (unsigned)W) continue;
        V8 v;
        v.u = *(const u32x4*)(row + (size_t)iw * Cp);
        float xf[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) xf[t] = bf2f(v.e[t]);
#pragma unroll
        for (int j = 0; j < OWG; ++j) {
          const int kw = c - j * S;
          if (kw < 0 || kw > 2) continue;      // compile-time after unrolling
#pragma unroll
          for (int t = 0; t < 8; ++t) acc[j][t] += xf[t] * wk[kw][t];
        }
      }
    }
#pragma unroll
    for (int j = 0; j < OWG; ++j) {
      if (ow0 + j >= OW) break;
      V8 o;
#pragma unroll
      for (int t = 0; t < 8; ++t) o.e[t] = f2bf(actx<GEN>(acc[j][t], act));
      *(u32x4*)(y + (((size_t)b * OH + oh) * OW + ow0 + j) * Cp + c0) = o.u;
    }
  }
}

// Average pool; padded positions are excluded from the count (TF/Keras 'same'), 'valid' has none.
__global__ __launch_bounds__(256) void avgpool_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, int B, int H,
                                                      int W, int Cp, int OH, int OW, int KH, int KW, int S,
                                                      int pad_t, int pad_l) {
  const int cpr = Cp / 8;
  const size_t total = (size_t)B * OH * OW * cpr;
  for (size_t i = gtid(); i < total; i += gstride()) {
    const int c0 = (int)(i % cpr) * 8;
    size_t pix = i / cpr;
    const int ow = (int)(pix % OW);
    pix /= OW;
    const int oh = (int)(pix % OH);
    const int b = (int)(pix / OH);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int n = 0;
    for (int kh = 0; kh < KH; ++kh) {
      const int ih = oh * S - pad_t + kh;
      if ((unsigned)ih >= (unsigned)H) continue;
      for (int kw = 0; kw < KW; ++kw) {
        const int iw = ow * S - pad_l + kw;
        if ((unsigned)iw >= (unsigned)W) continue;
        V8 v;
        v.u = *(const u32x4*)(x + (((size_t)b * H + ih) * W + iw) * Cp + c0);
#pragma unroll
        for (int t = 0; t < 8; ++t) acc[t] += bf2f(v.e[t]);
        ++n;
      }
    }
    const float inv = n ? 1.f / (float)n : 0.f;
    V8 o;
#pragma unroll
    for (int t = 0; t < 8; ++t) o.e[t] = f2bf(acc[t] * inv);
    *(u32x4*)(y + i * 8) = o.u;
  }
}

// One input of a channel concat: y[p][off + c] = x[p][c] for c < Cx; channels [zero_from, Cpy) of y are
// zeroed (the padding of the last input).  Aligned inputs (off, Cx, Cpx multiples of 8) move 16-byte chunks.
__global__ __launch_bounds__(256) void concat_vec_kernel(const bf16* __restrict__ x, int Cpx, bf16* __restrict__ y,
                                                         int Cpy, int off, int nchunk, size_t pixels) {
  const size_t total = pixels * nchunk;
  for (size_t i = gtid(); i < total; i += gstride()) {
    const size_t p = i / nchunk;
    const int c = (int)(i % nchunk) * 8;
    *(u32x4*)(y + p * Cpy + off + c) = *(const u32x4*)(x + p * Cpx + c);
  }
}

__global__ __launch_bounds__(256) void concat_scalar_kernel(const bf16* __restrict__ x, int Cx, int Cpx,
                                                            bf16* __restrict__ y, int Cpy, int off, int zero_from,
                                                            size_t pixels) {
  const int span = Cx + (zero_from < Cpy ? Cpy - zero_from : 0);
  const size_t total = pixels * span;
  for (size_t i = gtid(); i < total; i += gstride()) {
    const size_t p = i / span;
    const int c = (int)(i % span);
    if (c < Cx) y[p * Cpy + off + c] = x[p * Cpx + c];
    else y[p * Cpy + zero_from + (c - Cx)] = f2bf(0.f);
  }
}

// Standalone activation (any ActMode, LeakyReLU slope alpha) over bf16 chunks.
template <bool GEN>
__global__ __launch_bounds__(256) void act_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, size_t chunks,
                                                  int mode, float alpha) {
  for (size_t i = gtid(); i < chunks; i += gstride()) {
    V8 v, o;
    v.u = ((const u32x4*)x)[i];
#pragma unroll
    for (int t = 0; t < 8; ++t) o.e[t] = f2bf(actx<GEN>(bf2f(v.e[t]), mode, alpha));
    ((u32x4*)y)[i] = o.u;
  }
}

// Element-wise binary op (Keras Multiply / Subtract / Maximum / Minimum / Average / Add) of a [P][Cp] tensor
// with b, where b is either the same shape or one [Cp] row per image (bcast_hw = H*W pixels share it: the
// squeeze-excite Multiply of EfficientNet, x * se[b, 1, 1, c]).
enum BinOp { BIN_ADD = 0, BIN_SUB, BIN_MUL, BIN_MAX, BIN_MIN, BIN_AVG };
template <bool GEN>
__global__ __launch_bounds__(256) void binary_kernel(const bf16* __restrict__ a, const bf16* __restrict__ b,
                                                     bf16* __restrict__ y, size_t chunks, int cpr, int bcast_hw,
                                                     int op, int act) {
  for (size_t i = gtid(); i < chunks; i += gstride()) {
    size_t bi = i;
    if (bcast_hw) {
      const size_t pix = i / cpr;
      bi = (pix / bcast_hw) * cpr + (i % cpr);
    }
    V8 va, vb, o;
    va.u = ((const u32x4*)a)[i];
    vb.u = ((const u32x4*)b)[bi];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const float p = bf2f(va.e[t]), q = bf2f(vb.e[t]);
      float r;
      switch (op) {
        case BIN_SUB: r = p - q; break;
        case BIN_MUL: r = p * q; break;
        case BIN_MAX: r = fmaxf(p, q); break;
        case BIN_MIN: r = fminf(p, q); break;
        case BIN_AVG: r = 0.5f * (p + q); break;
        default: r = p + q;
      }
      o.e[t] = f2bf(actx<GEN>(r, act));
    }
    ((u32x4*)y)[i] = o.u;
  }
}

// Global max pool: block (image, 64 chunks), 4 pixel groups, LDS combine (as head.hip's GAP).
__global__ __launch_bounds__(256) void gmp_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, int HW, int Cp) {
  __shared__ float part[4][64][9];
  const int b = blockIdx.y;
  const int ch = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int cc = blockIdx.x * 64 + ch;
  const bool ok = cc * 8 < Cp;
  float m[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) m[t] = -INFINITY;
  if (ok) {
    const bf16* base = x + (size_t)b * HW * Cp + cc * 8;
    for (int i = grp; i < HW; i += 4) {
      V8 v;
      v.u = *(const u32x4*)(base + (size_t)i * Cp);
#pragma unroll
      for (int t = 0; t < 8; ++t) m[t] = fmaxf(m[t], bf2f(v.e[t]));
    }
  }
#pragma unroll
  for (int t = 0; t < 8; ++t) part[grp][ch][t] = m[t];
  __syncthreads();
  if (grp != 0 || !ok) return;
  V8 o;
#pragma unroll
  for (int t = 0; t < 8; ++t)
    o.e[t] = f2bf(fmaxf(fmaxf(part[0][ch][t], part[1][ch][t]), fmaxf(part[2][ch][t], part[3][ch][t])));
  *(u32x4*)(y + (size_t)b * Cp + cc * 8) = o.u;
}

// Global average pool over LARGE maps (EfficientNet's squeeze-excite at 112x112 .. 28x28), where head.hip's
// one-block-per-image GAP leaves most of the chip idle.  Pass 1: grid (S pixel slices, B); a block sums its
// slice for a group of up to 256 channel chunks (lane = chunk, the remaining threads stride the pixels) and
// reduces in LDS to one fp32 partial per channel.  Pass 2: sum of the S partials / HW -> bf16.
__global__ __launch_bounds__(256) void gap_part_kernel(const bf16* __restrict__ x, float* __restrict__ part,
                                                       int HW, int Cp, int S) {
  __shared__ float red[256][9];
  const int b = blockIdx.y, sl = blockIdx.x;
  const int cpr = Cp / 8;
  const int p0 = (int)((long long)HW * sl / S), p1 = (int)((long long)HW * (sl + 1) / S);
  for (int cg = 0; cg < cpr; cg += 256) {
    const int nc = min(256, cpr - cg);
    const int lanes = 256 / nc;                      // pixel lanes per chunk
    const int ch = threadIdx.x % nc, pl = threadIdx.x / nc;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (pl < lanes) {
      const bf16* base = x + (size_t)b * HW * Cp + (size_t)(cg + ch) * 8;
      for (int p = p0 + pl; p < p1; p += lanes) {
        V8 v;
        v.u = *(const u32x4*)(base + (size_t)p * Cp);
#pragma unroll
        for (int t = 0; t < 8; ++t) acc[t] += bf2f(v.e[t]);
      }
    }
#pragma unroll
    for (int t = 0; t < 8; ++t) red[threadIdx.x][t] = acc[t];
    __syncthreads();
    if (threadIdx.x < nc) {
      float sum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int l = 0; l < lanes; ++l)
#pragma unroll
        for (int t = 0; t < 8; ++t) sum[t] += red[l * nc + threadIdx.x][t];
      float* d = part + ((size_t)b * S + sl) * Cp + (size_t)(cg + threadIdx.x) * 8;
#pragma unroll
      for (int t = 0; t < 8; ++t) d[t] = sum[t];
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void gap_finish_kernel(const float* __restrict__ part, bf16* __restrict__ y,
                                                         float* __restrict__ y32, int B, int HW, int Cp, int S) {
  const size_t total = (size_t)B * Cp;
  const float inv = 1.f / (float)HW;
  for (size_t i = gtid(); i < total; i += gstride()) {
    const size_t b = i / Cp, c = i % Cp;
    float sum = 0.f;
    for (int sl = 0; sl < S; ++sl) sum += part[(b * S + sl) * Cp + c];
    if (y) y[i] = f2bf(sum * inv);
    if (y32) y32[i] = sum * inv;
  }
}

int gap_large_slices(int B, int HW) {
  int s = (512 + B - 1) / B;                       // ~2 blocks per CU in all
  const int cap = HW / 64 > 0 ? HW / 64 : 1;       // >= 64 pixels per slice
  return s < 1 ? 1 : (s > cap ? cap : s);
}

hipError_t gap_large(const bf16* x, bf16* y, float* y32, float* part, int B, int HW, int Cp, hipStream_t s) {
  if (Cp % 8) return hipErrorInvalidValue;
  const int S = gap_large_slices(B, HW);
  hipLaunchKernelGGL(gap_part_kernel, dim3(S, B), dim3(256), 0, s, x, part, HW, Cp, S);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(gap_finish_kernel, dim3(grid_of((size_t)B * Cp)), dim3(256), 0, s, part, y, y32, B, HW, Cp, S);
  return hipGetLastError();
}

hipError_t act(const bf16* x, bf16* y, size_t elems, int mode, float alpha, hipStream_t s) {
  if (elems % 8) return hipErrorInvalidValue;
  if (mode > ACT_RELU6) hipLaunchKernelGGL(act_kernel<true>, dim3(grid_of(elems / 8)), dim3(256), 0, s, x, y, elems / 8, mode, alpha);
  else hipLaunchKernelGGL(act_kernel<false>, dim3(grid_of(elems / 8)), dim3(256), 0, s, x, y, elems / 8, mode, alpha);
  return hipGetLastError();
}

hipError_t binary(const bf16* a, const bf16* b, bf16* y, size_t elems, int Cp, int bcast_hw, int op, int act_mode,
                  hipStream_t s) {
  if (elems % 8 || Cp % 8) return hipErrorInvalidValue;
  if (act_mode > ACT_RELU6)
    hipLaunchKernelGGL(binary_kernel<true>, dim3(grid_of(elems / 8)), dim3(256), 0, s, a, b, y, elems / 8, Cp / 8,
                       bcast_hw, op, act_mode);
  else
    hipLaunchKernelGGL(binary_kernel<false>, dim3(grid_of(elems / 8)), dim3(256), 0, s, a, b, y, elems / 8, Cp / 8,
                       bcast_hw, op, act_mode);
  return hipGetLastError();
}

hipError_t gmp(const bf16* x, bf16* y, int B, int HW, int Cp, hipStream_t s) {
  if (Cp % 8) return hipErrorInvalidValue;
  hipLaunchKernelGGL(gmp_kernel, dim3((Cp / 8 + 63) / 64, B), dim3(256), 0, s, x, y, HW, Cp);
  return hipGetLastError();
}

hipError_t dwconv(const bf16* x, const float* w, const float* bias, bf16* y, int B, int H, int W, int Cp, int OH,
                  int OW, int KH, int KW, int stride, int pad_t, int pad_l, int act, hipStream_t s) {
  if (Cp % 8) return hipErrorInvalidValue;
  // The register-blocked 3x3 kernel pays off at stride 1 on large maps; measured on MobileNetV2 bs=32
  // (profiles/mbv2_bs32_steps_v*.json) it lost at stride 2 and on grids under ~512 blocks, where the
  // thread-per-pixel kernel keeps 4x more loads in flight.
  constexpr int OWG = 4;
  const size_t t3 = (size_t)B * OH * ((OW + OWG - 1) / OWG) * (Cp / 8);
  if (KH == 3 && KW == 3 && stride == 1 && t3 >= 512 * 256) {
    if (act > ACT_RELU6)
      hipLaunchKernelGGL((dwconv3_kernel<1, OWG, true>), dim3(grid_of(t3)), dim3(256), 0, s, x, w, bias, y, B, H, W, Cp,
                         OH, OW, pad_t, pad_l, act);
    else
      hipLaunchKernelGGL((dwconv3_kernel<1, OWG, false>), dim3(grid_of(t3)), dim3(256), 0, s, x, w, bias, y, B, H, W, Cp,
                         OH, OW, pad_t, pad_l, act);
    return hipGetLastError();
  }
  const size_t total = (size_t)B * OH * OW * (Cp / 8);
  if (act > ACT_RELU6)
    hipLaunchKernelGGL(dwconv_kernel<true>, dim3(grid_of(total)), dim3(256), 0, s, x, w, bias, y, B, H, W, Cp, OH, OW,
                       KH, KW, stride, pad_t, pad_l, act);
  else
    hipLaunchKernelGGL(dwconv_kernel<false>, dim3(grid_of(total)), dim3(256), 0, s, x, w, bias, y, B, H, W, Cp, OH, OW,
                       KH, KW, stride, pad_t, pad_l, act);
  return hipGetLastError();
}

hipError_t avgpool(const bf16* x, bf16* y, int B, int H, int W, int Cp, int OH, int OW, int KH, int KW, int S,
                   int pad_t, int pad_l, hipStream_t s) {
  if (Cp % 8) return hipErrorInvalidValue;
  const size_t total = (size_t)B * OH * OW * (Cp / 8);
  hipLaunchKernelGGL(avgpool_kernel, dim3(grid_of(total)), dim3(256), 0, s, x, y, B, H, W, Cp, OH, OW, KH, KW, S,
                     pad_t, pad_l);
  return hipGetLastError();
}

hipError_t concat_into(const bf16* x, int Cx, int Cpx, bf16* y, int Cpy, int off, int zero_from, size_t pixels,
                       hipStream_t s) {
  if (off + Cx > Cpy || Cx > Cpx || zero_from > Cpy) return hipErrorInvalidValue;
  if (off % 8 == 0 && Cx % 8 == 0 && Cpx % 8 == 0 && Cpy % 8 == 0 && zero_from >= Cpy) {
    const int nchunk = Cx / 8;
    hipLaunchKernelGGL(concat_vec_kernel, dim3(grid_of(pixels * nchunk)), dim3(256), 0, s, x, Cpx, y, Cpy, off,
                       nchunk, pixels);
  } else {
    const size_t span = (size_t)Cx + (zero_from < Cpy ? Cpy - zero_from : 0);
    hipLaunchKernelGGL(concat_scalar_kernel, dim3(grid_of(pixels * span)), dim3(256), 0, s, x, Cx, Cpx, y, Cpy,
                       off, zero_from, pixels);
  }
  return hipGetLastError();
}

}  // namespace adapt
