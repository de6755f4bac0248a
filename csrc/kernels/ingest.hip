// Serving ingest: uint8 NHWC images -> fp32 model input, with the Keras
// `preprocess_input` modes applied on the device.  The reference runs
// `preprocess_input` (caffe: RGB -> BGR, minus the ImageNet BGR mean) in
// numpy on the host and ships fp32 pixels (`test/test.py:20-23`, 19.3 MB per
// bs=32 batch); here 4.8 MB of uint8 cross to the GPU and this kernel writes
// the stem's fp32 input:
//   y[p][c] = x[p][src(c)] * scale[c] + shift[c],  src(c) = reverse ? C-1-c : c
// Each thread handles 4 consecutive bytes of the flat input (one dword load).
#include "kernels.h"

namespace adapt {

namespace {
struct IngestAffine {
  float scale[4], shift[4];
};

__global__ __launch_bounds__(256) void ingest_u8_kernel(const uint8_t* __restrict__ x, float* __restrict__ y,
                                                        size_t n, int C, int reverse, IngestAffine a) {
  const size_t n4 = n / 4;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4 + (n % 4 ? 1 : 0);
       i += (size_t)gridDim.x * blockDim.x) {
    const size_t base = i * 4;
    uint32_t w;
    if (base + 4 <= n) {
      w = *(const uint32_t*)(x + base);          // n % 4 == 0 for any batch of 3-channel 224x224 images
    } else {
      w = 0;
      for (size_t t = base; t < n; ++t) w |= (uint32_t)x[t] << (8 * (t - base));
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const size_t e = base + t;
      if (e >= n) break;
      const int c = (int)(e % C);
      const int sc = reverse ? C - 1 - c : c;     // the source channel of output channel c
      const size_t src = e - c + sc;
      const uint32_t v = (src >= base && src < base + 4) ? (w >> (8 * (src - base))) & 0xFF : x[src];
      y[e] = (float)v * a.scale[c] + a.shift[c];
    }
  }
}
}  // namespace

hipError_t ingest_u8(const uint8_t* x, float* y, size_t n, int C, int reverse, const float* scale,
                     const float* shift, hipStream_t s) {
  if (C < 1 || C > 4) return hipErrorInvalidValue;
  IngestAffine a;
  for (int c = 0; c < 4; ++c) {
    a.scale[c] = c < C ? scale[c] : 1.f;
    a.shift[c] = c < C ? shift[c] : 0.f;
  }
  size_t blocks = (n / 4 + 256) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(ingest_u8_kernel, dim3((unsigned)blocks), dim3(256), 0, s, x, y, n, C, reverse, a);
  return hipGetLastError();
}

}  // namespace adapt
