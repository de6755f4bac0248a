// Memory-bound NHWC kernels for the ResNet graph (gfx950).
//
// Every kernel moves 16-byte vectors (8 x bf16) per lane
// (cdna_hip_programming.md Guideline 13) and grid-strides over the tensor.
//
//  * input_pack    fp32 NHWC (C=3) -> bf16 NHWC padded to Cp channels (stem input)
//  * bn_act        y = x*scale[c] + shift[c] (+ReLU)          (unfused Keras BN)
//  * add_act       y = a + b (+ReLU)                          (unfused Keras Add)
//  * relu          y = max(x, 0)
//  * maxpool       KxK/s with explicit zero padding (Keras ZeroPadding2D + MaxPooling2D)
//  * gap           -> head.hip
//  * softmax_rows  fp32 row softmax (Dense activation='softmax')
//  * cast          bf16 <-> fp32 for frontier / host I/O
#include "kernels.h"

namespace adapt {

static inline int grid_for(size_t work, int block = 256, int cap = 8192) {
  size_t g = (work + block - 1) / block;
  if (g < 1) g = 1;
  if (g > (size_t)cap) g = cap;
  return (int)g;
}

__global__ __launch_bounds__(256) void input_pack_kernel(const float* __restrict__ x, bf16* __restrict__ y,
                                                         size_t pixels, int C, int Cp) {
  for (size_t p = blockIdx.x * (size_t)blockDim.x + threadIdx.x; p < pixels; p += (size_t)gridDim.x * blockDim.x) {
    V8 o;
#pragma unroll
    for (int t = 0; t < 8; ++t) o.e[t] = f2bf(0.f);
    const float* src = x + p * C;
    for (int c = 0; c < C && c < 8; ++c) o.e[c] = f2bf(src[c]);
    *(u32x4*)(y + p * Cp) = o.u;
    for (int c = 8; c < Cp; c += 8) {
      V8 z;
      for (int t = 0; t < 8; ++t) z.e[t] = f2bf((c + t) < C ? src[c + t] : 0.f);
      *(u32x4*)(y + p * Cp + c) = z.u;
    }
  }
}

template <bool GEN>
__global__ __launch_bounds__(256) void bn_act_kernel(const bf16* __restrict__ x, bf16* __restrict__ y,
                                                     const float* __restrict__ scale, const float* __restrict__ shift,
                                                     size_t chunks, int C, int relu) {
  const int cpr = C / 8;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < chunks; i += (size_t)gridDim.x * blockDim.x) {
    const int c0 = (int)(i % cpr) * 8;
    V8 v, o;
    v.u = ((const u32x4*)x)[i];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      float f = bf2f(v.e[t]) * scale[c0 + t] + shift[c0 + t];
      o.e[t] = f2bf(actx<GEN>(f, relu));
    }
    ((u32x4*)y)[i] = o.u;
  }
}

template <bool GEN>
__global__ __launch_bounds__(256) void add_act_kernel(const bf16* __restrict__ a, const bf16* __restrict__ b,
                                                      bf16* __restrict__ y, size_t chunks, int relu) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < chunks; i += (size_t)gridDim.x * blockDim.x) {
    V8 va, vb, o;
    va.u = ((const u32x4*)a)[i];
    vb.u = ((const u32x4*)b)[i];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      float f = bf2f(va.e[t]) + bf2f(vb.e[t]);
      o.e[t] = f2bf(actx<GEN>(f, relu));
    }
    ((u32x4*)y)[i] = o.u;
  }
}

template <bool GEN>
__global__ __launch_bounds__(256) void relu_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, size_t chunks,
                                                   int mode) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < chunks; i += (size_t)gridDim.x * blockDim.x) {
    V8 v, o;
    v.u = ((const u32x4*)x)[i];
#pragma unroll
    for (int t = 0; t < 8; ++t) o.e[t] = f2bf(actx<GEN>(bf2f(v.e[t]), mode));
    ((u32x4*)y)[i] = o.u;
  }
}

// Max pool over an implicitly zero-padded input: Keras pads with zeros
// (ZeroPadding2D) and the zeros take part in the max.
__global__ __launch_bounds__(256) void maxpool_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, int B, int H,
                                                      int W, int C, int OH, int OW, int K, int S, int pad_t, int pad_l,
                                                      int pad_zero) {
  const int cpr = C / 8;
  const size_t total = (size_t)B * OH * OW * cpr;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int cc = (int)(i % cpr);
    size_t r = i / cpr;
    const int ow = (int)(r % OW);
    r /= OW;
    const int oh = (int)(r % OH);
    const int b = (int)(r / OH);
    float m[8];
    bool any_pad = false;
#pragma unroll
    for (int t = 0; t < 8; ++t) m[t] = -INFINITY;
    for (int kh = 0; kh < K; ++kh) {
      const int ih = oh * S - pad_t + kh;
      for (int kw = 0; kw < K; ++kw) {
        const int iw = ow * S - pad_l + kw;
        if ((unsigned)ih >= (unsigned)H || (unsigned)iw >= (unsigned)W) {
          any_pad = true;
          continue;
        }
        V8 v;
        v.u = *(const u32x4*)(x + (((size_t)b * H + ih) * W + iw) * C + cc * 8);
#pragma unroll
        for (int t = 0; t < 8; ++t) m[t] = fmaxf(m[t], bf2f(v.e[t]));
      }
    }
    V8 o;
#pragma unroll
    for (int t = 0; t < 8; ++t) o.e[t] = f2bf((any_pad && pad_zero) ? fmaxf(m[t], 0.f) : m[t]);
    *(u32x4*)(y + i * 8) = o.u;
  }
}

// one block (256 threads) per row
__global__ __launch_bounds__(256) void softmax_rows_kernel(const float* __restrict__ x, float* __restrict__ y, int N,
                                                           int ldx) {
  __shared__ float red[8];
  const int row = blockIdx.x;
  const float* xr = x + (size_t)row * ldx;
  float* yr = y + (size_t)row * N;
  float mx = -INFINITY;
  for (int i = threadIdx.x; i < N; i += blockDim.x) mx = fmaxf(mx, xr[i]);
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) red[w] = mx;
  __syncthreads();
  mx = red[0];
  for (int i = 1; i < (int)(blockDim.x >> 6); ++i) mx = fmaxf(mx, red[i]);
  __syncthreads();
  float sum = 0.f;
  for (int i = threadIdx.x; i < N; i += blockDim.x) sum += __expf(xr[i] - mx);
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
  if (l == 0) red[w] = sum;
  __syncthreads();
  sum = 0.f;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) sum += red[i];
  const float inv = 1.f / sum;
  for (int i = threadIdx.x; i < N; i += blockDim.x) yr[i] = __expf(xr[i] - mx) * inv;
}

__global__ __launch_bounds__(256) void cast_bf16_f32_kernel(const bf16* __restrict__ x, float* __restrict__ y, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    y[i] = bf2f(x[i]);
}
__global__ __launch_bounds__(256) void cast_f32_bf16_kernel(const float* __restrict__ x, bf16* __restrict__ y, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    y[i] = f2bf(x[i]);
}


// materialised ZeroPadding2D (only when a cut exposes the padded tensor)
__global__ __launch_bounds__(256) void pad_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, int B, int H, int W,
                                                  int C, int OH, int OW, int pad_t, int pad_l) {
  const int cpr = C / 8;
  const size_t total = (size_t)B * OH * OW * cpr;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int cc = (int)(i % cpr);
    size_t r = i / cpr;
    const int ow = (int)(r % OW);
    r /= OW;
    const int oh = (int)(r % OH);
    const int b = (int)(r / OH);
    const int ih = oh - pad_t, iw = ow - pad_l;
    u32x4 v = {0u, 0u, 0u, 0u};
    if ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W)
      v = *(const u32x4*)(x + (((size_t)b * H + ih) * W + iw) * C + cc * 8);
    *(u32x4*)(y + i * 8) = v;
  }
}

// ---------------------------------------------------------------- launchers
hipError_t input_pack(const float* x, bf16* y, size_t pixels, int C, int Cp, hipStream_t s) {
  hipLaunchKernelGGL(input_pack_kernel, dim3(grid_for(pixels)), dim3(256), 0, s, x, y, pixels, C, Cp);
  return hipGetLastError();
}
hipError_t bn_act(const bf16* x, bf16* y, const float* scale, const float* shift, size_t elems, int C, int relu,
                  hipStream_t s) {
  size_t chunks = elems / 8;
  if (relu > ACT_RELU6)
    hipLaunchKernelGGL(bn_act_kernel<true>, dim3(grid_for(chunks)), dim3(256), 0, s, x, y, scale, shift, chunks, C, relu);
  else
    hipLaunchKernelGGL(bn_act_kernel<false>, dim3(grid_for(chunks)), dim3(256), 0, s, x, y, scale, shift, chunks, C, relu);
  return hipGetLastError();
}
hipError_t add_act(const bf16* a, const bf16* b, bf16* y, size_t elems, int relu, hipStream_t s) {
  size_t chunks = elems / 8;
  if (relu > ACT_RELU6) hipLaunchKernelGGL(add_act_kernel<true>, dim3(grid_for(chunks)), dim3(256), 0, s, a, b, y, chunks, relu);
  else hipLaunchKernelGGL(add_act_kernel<false>, dim3(grid_for(chunks)), dim3(256), 0, s, a, b, y, chunks, relu);
  return hipGetLastError();
}
hipError_t relu(const bf16* x, bf16* y, size_t elems, int mode, hipStream_t s) {
  size_t chunks = elems / 8;
  if (mode > ACT_RELU6) hipLaunchKernelGGL(relu_kernel<true>, dim3(grid_for(chunks)), dim3(256), 0, s, x, y, chunks, mode);
  else hipLaunchKernelGGL(relu_kernel<false>, dim3(grid_for(chunks)), dim3(256), 0, s, x, y, chunks, mode);
  return hipGetLastError();
}
hipError_t maxpool(const bf16* x, bf16* y, int B, int H, int W, int C, int OH, int OW, int K, int S, int pad_t,
                   int pad_l, int pad_zero, hipStream_t s) {
  size_t total = (size_t)B * OH * OW * (C / 8);
  hipLaunchKernelGGL(maxpool_kernel, dim3(grid_for(total)), dim3(256), 0, s, x, y, B, H, W, C, OH, OW, K, S, pad_t,
                     pad_l, pad_zero);
  return hipGetLastError();
}
hipError_t softmax_rows(const float* x, float* y, int rows, int N, int ldx, hipStream_t s) {
  hipLaunchKernelGGL(softmax_rows_kernel, dim3(rows), dim3(256), 0, s, x, y, N, ldx);
  return hipGetLastError();
}
hipError_t cast_bf16_f32(const bf16* x, float* y, size_t n, hipStream_t s) {
  hipLaunchKernelGGL(cast_bf16_f32_kernel, dim3(grid_for(n)), dim3(256), 0, s, x, y, n);
  return hipGetLastError();
}
hipError_t cast_f32_bf16(const float* x, bf16* y, size_t n, hipStream_t s) {
  hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3(grid_for(n)), dim3(256), 0, s, x, y, n);
  return hipGetLastError();
}

hipError_t pad(const bf16* x, bf16* y, int B, int H, int W, int C, int OH, int OW, int pad_t, int pad_l,
               hipStream_t s) {
  size_t total = (size_t)B * OH * OW * (C / 8);
  hipLaunchKernelGGL(pad_kernel, dim3(grid_for(total)), dim3(256), 0, s, x, y, B, H, W, C, OH, OW, pad_t, pad_l);
  return hipGetLastError();
}

}  // namespace adapt
