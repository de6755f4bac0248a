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

// Activations of the fused epilogues and the eltwise kernels (Keras names):
//   0 linear, 1 relu, 2 relu6 (ReLU(max_value=6)), 3 swish / silu, 4 sigmoid, 5 tanh,
//   6 hard_sigmoid (Keras 2: clip(0.2x + 0.5)), 7 hard_swish (x * relu6(x + 3) / 6),
//   8 gelu (erf form), 9 elu, 10 selu, 11 softplus, 12 leaky_relu (slope alpha)
enum ActMode { ACT_LINEAR = 0, ACT_RELU, ACT_RELU6, ACT_SWISH, ACT_SIGMOID, ACT_TANH, ACT_HARD_SIGMOID,
               ACT_HARD_SWISH, ACT_GELU, ACT_ELU, ACT_SELU, ACT_SOFTPLUS, ACT_LEAKY_RELU };
// The MFMA conv epilogues take the ReLU family only (two selects; the wider
// switch below, inlined into every tile config, doubled their code and compile
// time): runtime/plan.py runs other activations after a conv as their own step.
__device__ __forceinline__ float act_relu(float v, int mode) {
  v = mode ? fmaxf(v, 0.f) : v;
  return mode == ACT_RELU6 ? fminf(v, 6.f) : v;
}

__device__ __forceinline__ float act_f(float v, int mode, float alpha = 0.3f) {
  if (mode <= ACT_RELU6) return act_relu(v, mode);
  switch (mode) {
    case ACT_SWISH: return v / (1.f + __expf(-v));
    case ACT_SIGMOID: return 1.f / (1.f + __expf(-v));
    case ACT_TANH: return tanhf(v);
    case ACT_HARD_SIGMOID: return fminf(fmaxf(0.2f * v + 0.5f, 0.f), 1.f);
    case ACT_HARD_SWISH: return v * fminf(fmaxf(v + 3.f, 0.f), 6.f) * (1.f / 6.f);
    case ACT_GELU: return 0.5f * v * (1.f + erff(v * 0.70710678f));
    case ACT_ELU: return v > 0.f ? v : __expf(v) - 1.f;
    case ACT_SELU: return 1.0507009873554805f * (v > 0.f ? v : 1.6732632423543772f * (__expf(v) - 1.f));
    case ACT_SOFTPLUS: return v > 20.f ? v : log1pf(__expf(v));
    case ACT_LEAKY_RELU: return v > 0.f ? v : alpha * v;
    default: return v;
  }
}

// Activation with the mode range fixed at compile time: GEN = false keeps a
// kernel's inner loop to the ReLU family's two selects (the full switch of
// act_f, expanded per element, made the memory-bound bn / add / dwconv
// kernels instruction-bound: DenseNet121's unfused BN 5x slower);
// launchers pick GEN = mode > ACT_RELU6.
template <bool GEN>
__device__ __forceinline__ float actx(float v, int mode, float alpha = 0.3f) {
  if constexpr (GEN) return act_f(v, mode, alpha);
  else return act_relu(v, mode);
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
