// Shared CDNA4 (gfx950) helpers for the ADAPT MI355X kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define ADAPT_WAVE 64

__device__ __forceinline__ float bf2f(bf16 v) { return (float)v; }
__device__ __forceinline__ bf16 f2bf(float v) { return (bf16)v; }  // RNE, v_cvt_pk_bf16_f32

// 16-byte vector of 8 bf16 held as 4 dwords (keeps loads/stores dwordx4).
union V8 {
  u32x4 u;
  bf16x8 h;
  bf16 e[8];
};

// Fused activation of the epilogues and eltwise kernels: 0 none, 1 ReLU,
// 2 ReLU6 (Keras ReLU(max_value=6), MobileNetV2).
__device__ __forceinline__ float act_f(float v, int mode) {
  v = mode ? fmaxf(v, 0.f) : v;
  return mode == 2 ? fminf(v, 6.f) : v;
}

// Bijective XCD-aware remap (cdna_hip_programming.md §5 "XCD swizzle must be
// bijective"): consecutive logical tiles land on the same XCD so neighbouring
// tiles that share an A panel hit the same L2.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int nx = 8;
  if (nwg < nx) return orig;
  int q = nwg / nx, r = nwg % nx;
  int xcd = orig % nx, loc = orig / nx;
  int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + loc;
}
