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
        acc[0] += bf2f(v.e[0]) * w0[0]; acc[1] += bf2f(v.e[1]) * w0[1];
        acc[2] += bf2f(v.e[2]) * w0[2]; acc[3] += bf2f(v.e[3]) * w0[3];
        acc[4] += bf2f(v.e[4]) * w1[0]; acc[5] += bf2f(v.e[5]) * w1[1];
        acc[6] += bf2f(v.e[6]) * w1[2]; acc[7] += bf2f(v.e[7]) * w1[3];
      }
    }
    V8 o;
#pragma unroll
    for (int t = 0; t < 8; ++t) o.e[t] = f2bf(act_f(acc[t], act));
    *(u32x4*)(y + i * 8) = o.u;
  }
}

// 3x3 specialisation: a thread owns OWG consecutive output pixels of one row and one 8-channel chunk, so
// each input column of the (OWG-1)*S+3 it touches is loaded once per filter row (6 loads per row instead of
// 12 at stride 1, 9 instead of 12 at stride 2) and the row's three weight vectors stay in registers.
template <int S, int OWG>
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
      for (int t = 0; t < 8; ++t) o.e[t] = f2bf(act_f(acc[j][t], act));
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

hipError_t dwconv(const bf16* x, const float* w, const float* bias, bf16* y, int B, int H, int W, int Cp, int OH,
                  int OW, int KH, int KW, int stride, int pad_t, int pad_l, int act, hipStream_t s) {
  if (Cp % 8) return hipErrorInvalidValue;
  // The register-blocked 3x3 kernel pays off at stride 1 on large maps; measured on MobileNetV2 bs=32
  // (profiles/mbv2_bs32_steps_v*.json) it lost at stride 2 and on grids under ~512 blocks, where the
  // thread-per-pixel kernel keeps 4x more loads in flight.
  constexpr int OWG = 4;
  const size_t t3 = (size_t)B * OH * ((OW + OWG - 1) / OWG) * (Cp / 8);
  if (KH == 3 && KW == 3 && stride == 1 && t3 >= 512 * 256) {
    hipLaunchKernelGGL((dwconv3_kernel<1, OWG>), dim3(grid_of(t3)), dim3(256), 0, s, x, w, bias, y, B, H, W, Cp, OH,
                       OW, pad_t, pad_l, act);
    return hipGetLastError();
  }
  const size_t total = (size_t)B * OH * OW * (Cp / 8);
  hipLaunchKernelGGL(dwconv_kernel, dim3(grid_of(total)), dim3(256), 0, s, x, w, bias, y, B, H, W, Cp, OH, OW, KH,
                     KW, stride, pad_t, pad_l, act);
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
