// Native CPU execution path (pybind11 module `_cpu`): the ops of a compiled
// fp32 launch plan (runtime/plan.py, `target="cpu"`) on NHWC float32 tensors,
// parallelised with OpenMP and vectorised over channels.
//
// The reference's single-chunk baseline runs ResNet-50 through TF's CPU
// kernels (`/root/reference/test/local_infer.py:18-28`, `model.predict` in
// float32) and its workers run whatever TF device they have
// (`/root/reference/src/node.py:177`).  Here a CPU stage executes the same
// fused steps as a GPU slice -- conv with BN folded into the weights at load,
// bias + residual + activation in the conv's own epilogue, pools with TF
// padding semantics, GAP, dense + softmax -- so PyTorch stays the test oracle
// only (ops/reference.py).
//
// Conv is a direct NHWC convolution blocked for registers: a task owns one
// output row segment of PIX pixels and a COB-wide slice of output channels,
// accumulates PIX x COB fp32 sums over (kh, kw, cin) with the filter row
// HWIO-contiguous in cout (one vector load feeds PIX FMAs), then applies the
// epilogue and stores.  1x1 convs and Dense are the same loop with kh = kw = 1.
// Each hot function is compiled for AVX-512, AVX2+FMA and baseline x86-64
// (`target_clones`); the loader picks the widest one the host CPU has, so the
// library runs on any x86-64 box.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <omp.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <vector>

namespace py = pybind11;

namespace {

#if defined(__x86_64__) && defined(__GNUC__) && !defined(__clang__)
#define ADAPT_CLONES __attribute__((target_clones("avx512f", "arch=haswell", "default")))
#else
#define ADAPT_CLONES
#endif

// Activations of the plan (graph/ir.py ACT_MODE; same formulas as
// csrc/kernels/common.h `act_f`, Keras 2 definitions).
enum Act { LINEAR = 0, RELU, RELU6, SWISH, SIGMOID, TANH, HARD_SIGMOID, HARD_SWISH, GELU, ELU, SELU, SOFTPLUS,
           LEAKY_RELU };

inline float act_f(float v, int mode, float alpha) {
  switch (mode) {
    case LINEAR: return v;
    case RELU: return v > 0.f ? v : 0.f;
    case RELU6: return std::min(std::max(v, 0.f), 6.f);
    case SWISH: return v / (1.f + std::exp(-v));
    case SIGMOID: return 1.f / (1.f + std::exp(-v));
    case TANH: return std::tanh(v);
    case HARD_SIGMOID: return std::min(std::max(0.2f * v + 0.5f, 0.f), 1.f);
    case HARD_SWISH: return v * std::min(std::max(v + 3.f, 0.f), 6.f) * (1.f / 6.f);
    case GELU: return 0.5f * v * (1.f + std::erf(v * 0.70710678f));
    case ELU: return v > 0.f ? v : std::exp(v) - 1.f;
    case SELU: return 1.0507009873554805f * (v > 0.f ? v : 1.6732632423543772f * (std::exp(v) - 1.f));
    case SOFTPLUS: return v > 20.f ? v : std::log1p(std::exp(v));
    case LEAKY_RELU: return v > 0.f ? v : alpha * v;
    default: throw std::invalid_argument("cpu_ops: unknown activation mode");
  }
}

template <typename T>
using Arr = py::array_t<T, py::array::c_style | py::array::forcecast>;

const float* cptr(const Arr<float>& a) { return a.data(); }
float* mptr(Arr<float>& a) { return a.mutable_data(); }

void need(bool ok, const char* what) {
  if (!ok) throw std::invalid_argument(std::string("cpu_ops: ") + what);
}

// ------------------------------------------------------------------ conv
constexpr int COB = 64;   // output channels per task (4 zmm / 8 ymm)
constexpr int PIX = 4;    // output pixels per task

struct ConvGeom {
  int N, H, W, C, OH, OW, CO, COP, KH, KW, S, PT, PL, act;
  float alpha;
};

// One task: pixels [ow0, ow0 + np) of output row (n, oh), channels [co0, co0 + COB).
// w is HWIO with cout padded to COP (a multiple of COB, zero filters).
ADAPT_CLONES
void conv_task(const ConvGeom& g, const float* __restrict x, const float* __restrict w, const float* __restrict bias,
               const float* __restrict res, float* __restrict y, int n, int oh, int ow0, int np, int co0) {
  float acc[PIX][COB];
  for (int p = 0; p < PIX; ++p)
    for (int j = 0; j < COB; ++j) acc[p][j] = 0.f;
  for (int kh = 0; kh < g.KH; ++kh) {
    const int ih = oh * g.S - g.PT + kh;
    if (ih < 0 || ih >= g.H) continue;
    for (int kw = 0; kw < g.KW; ++kw) {
      const float* xp[PIX];
      for (int p = 0; p < PIX; ++p) {
        const int iw = (ow0 + p) * g.S - g.PL + kw;
        xp[p] = (p < np && iw >= 0 && iw < g.W) ? x + (((size_t)n * g.H + ih) * g.W + iw) * g.C : nullptr;
      }
      const float* wr = w + ((size_t)(kh * g.KW + kw) * g.C) * g.COP + co0;
      if (xp[0] && xp[1] && xp[2] && xp[3]) {          // interior: no per-pixel checks in the K loop
        for (int c = 0; c < g.C; ++c) {
          const float* wv = wr + (size_t)c * g.COP;
          const float x0 = xp[0][c], x1 = xp[1][c], x2 = xp[2][c], x3 = xp[3][c];
#pragma omp simd
          for (int j = 0; j < COB; ++j) {
            const float wj = wv[j];
            acc[0][j] += x0 * wj;
            acc[1][j] += x1 * wj;
            acc[2][j] += x2 * wj;
            acc[3][j] += x3 * wj;
          }
        }
      } else {
        for (int c = 0; c < g.C; ++c) {
          const float* wv = wr + (size_t)c * g.COP;
          float xv[PIX];
          for (int p = 0; p < PIX; ++p) xv[p] = xp[p] ? xp[p][c] : 0.f;
#pragma omp simd
          for (int j = 0; j < COB; ++j) {
            const float wj = wv[j];
            acc[0][j] += xv[0] * wj;
            acc[1][j] += xv[1] * wj;
            acc[2][j] += xv[2] * wj;
            acc[3][j] += xv[3] * wj;
          }
        }
      }
    }
  }
  const int nco = std::min(COB, g.CO - co0);
  for (int p = 0; p < np; ++p) {
    const size_t o = (((size_t)n * g.OH + oh) * g.OW + ow0 + p) * g.CO + co0;
    float* yo = y + o;
    const float* ro = res ? res + o : nullptr;
    for (int j = 0; j < nco; ++j) {
      float v = acc[p][j] + bias[co0 + j];
      if (ro) v += ro[j];
      yo[j] = g.act == RELU ? (v > 0.f ? v : 0.f) : act_f(v, g.act, g.alpha);
    }
  }
}

// x [N,H,W,C]; w [KH,KW,C,COP] (cout padded to COP); bias [CO]; y [N,OH,OW,CO];
// residual (optional) [N,OH,OW,CO] added before the activation.
void conv2d(const Arr<float>& x, const Arr<float>& w, const Arr<float>& bias, Arr<float>& y, int stride, int pad_t,
            int pad_l, int act, float alpha, py::object residual) {
  need(x.ndim() == 4 && w.ndim() == 4 && y.ndim() == 4 && bias.ndim() == 1, "conv2d ranks");
  ConvGeom g{(int)x.shape(0), (int)x.shape(1), (int)x.shape(2), (int)x.shape(3), (int)y.shape(1), (int)y.shape(2),
             (int)y.shape(3), (int)w.shape(3), (int)w.shape(0), (int)w.shape(1), stride, pad_t, pad_l, act, alpha};
  need(w.shape(2) == g.C && g.COP % COB == 0 && g.COP >= g.CO && y.shape(0) == g.N && bias.shape(0) >= g.CO,
       "conv2d shapes");
  Arr<float> r;
  const float* rp = nullptr;
  if (!residual.is_none()) {
    r = residual.cast<Arr<float>>();
    need(r.size() == y.size(), "conv2d residual shape");
    rp = r.data();
  }
  const float *xp = cptr(x), *wp = cptr(w), *bp = cptr(bias);
  float* yp = mptr(y);
  const int segs = (g.OW + PIX - 1) / PIX, cob = g.COP / COB;
  const long tasks = (long)g.N * g.OH * segs * cob;
  py::gil_scoped_release nogil;
#pragma omp parallel for schedule(static)
  for (long t = 0; t < tasks; ++t) {
    // channel slice innermost: the tasks of one thread share their input row segment
    const int cb = (int)(t % cob);
    long r2 = t / cob;
    const int sg = (int)(r2 % segs);
    r2 /= segs;
    const int oh = (int)(r2 % g.OH), n = (int)(r2 / g.OH);
    const int ow0 = sg * PIX;
    conv_task(g, xp, wp, bp, rp, yp, n, oh, ow0, std::min(PIX, g.OW - ow0), cb * COB);
  }
}

// ------------------------------------------------------------------ depthwise
// x [N,H,W,C]; w [KH,KW,C]; bias [C]; y [N,OH,OW,C]
ADAPT_CLONES
void dw_row(const float* __restrict x, const float* __restrict w, const float* __restrict b, float* __restrict y,
            int n, int oh, int H, int W, int C, int OW, int KH, int KW, int S, int PT, int PL, int act, float alpha,
            int OH) {
  std::vector<float> acc(C);
  for (int ow = 0; ow < OW; ++ow) {
    std::copy(b, b + C, acc.begin());
    for (int kh = 0; kh < KH; ++kh) {
      const int ih = oh * S - PT + kh;
      if (ih < 0 || ih >= H) continue;
      for (int kw = 0; kw < KW; ++kw) {
        const int iw = ow * S - PL + kw;
        if (iw < 0 || iw >= W) continue;
        const float* xv = x + (((size_t)n * H + ih) * W + iw) * C;
        const float* wv = w + (size_t)(kh * KW + kw) * C;
        float* a = acc.data();
#pragma omp simd
        for (int c = 0; c < C; ++c) a[c] += xv[c] * wv[c];
      }
    }
    float* yo = y + (((size_t)n * OH + oh) * OW + ow) * C;
    for (int c = 0; c < C; ++c) yo[c] = act_f(acc[c], act, alpha);
  }
}

void dwconv2d(const Arr<float>& x, const Arr<float>& w, const Arr<float>& bias, Arr<float>& y, int stride, int pad_t,
              int pad_l, int act, float alpha) {
  need(x.ndim() == 4 && w.ndim() == 3 && y.ndim() == 4, "dwconv ranks");
  const int N = x.shape(0), H = x.shape(1), W = x.shape(2), C = x.shape(3), OH = y.shape(1), OW = y.shape(2);
  need(w.shape(2) == C && y.shape(3) == C && bias.shape(0) == C, "dwconv shapes");
  const float *xp = cptr(x), *wp = cptr(w), *bp = cptr(bias);
  float* yp = mptr(y);
  const int KH = w.shape(0), KW = w.shape(1);
  py::gil_scoped_release nogil;
#pragma omp parallel for collapse(2) schedule(static)
  for (int n = 0; n < N; ++n)
    for (int oh = 0; oh < OH; ++oh) dw_row(xp, wp, bp, yp, n, oh, H, W, C, OW, KH, KW, stride, pad_t, pad_l, act, alpha, OH);
}

// ------------------------------------------------------------------ pools
// kind 0 max, 1 avg.  pad_zero (max): padded positions take part as zeros (a
// folded ZeroPadding2D); otherwise they are excluded (Keras 'same').  avg
// always excludes them (TF).
void pool2d(const Arr<float>& x, Arr<float>& y, int kind, int kh_, int kw_, int stride, int pad_t, int pad_l,
            bool pad_zero) {
  need(x.ndim() == 4 && y.ndim() == 4, "pool ranks");
  const int N = x.shape(0), H = x.shape(1), W = x.shape(2), C = x.shape(3), OH = y.shape(1), OW = y.shape(2);
  need(y.shape(3) == C, "pool channels");
  const float* xp = cptr(x);
  float* yp = mptr(y);
  py::gil_scoped_release nogil;
#pragma omp parallel for collapse(2) schedule(static)
  for (int n = 0; n < N; ++n)
    for (int oh = 0; oh < OH; ++oh) {
      std::vector<float> acc(C);
      for (int ow = 0; ow < OW; ++ow) {
        std::fill(acc.begin(), acc.end(), kind == 0 ? -INFINITY : 0.f);
        int cnt = 0;
        bool padded = false;
        for (int i = 0; i < kh_; ++i) {
          const int ih = oh * stride - pad_t + i;
          for (int j = 0; j < kw_; ++j) {
            const int iw = ow * stride - pad_l + j;
            if (ih < 0 || ih >= H || iw < 0 || iw >= W) {
              padded = true;
              continue;
            }
            ++cnt;
            const float* xv = xp + (((size_t)n * H + ih) * W + iw) * C;
            float* a = acc.data();
            if (kind == 0) {
#pragma omp simd
              for (int c = 0; c < C; ++c) a[c] = std::max(a[c], xv[c]);
            } else {
#pragma omp simd
              for (int c = 0; c < C; ++c) a[c] += xv[c];
            }
          }
        }
        float* yo = yp + (((size_t)n * OH + oh) * OW + ow) * C;
        if (kind == 0) {
          for (int c = 0; c < C; ++c) yo[c] = (padded && pad_zero) ? std::max(acc[c], 0.f) : acc[c];
        } else {
          const float inv = cnt ? 1.f / cnt : 0.f;
          for (int c = 0; c < C; ++c) yo[c] = acc[c] * inv;
        }
      }
    }
}

// global average / max pool: x [N, P, C] -> y [N, C]
void global_pool(const Arr<float>& x, Arr<float>& y, int kind) {
  const int N = x.shape(0), C = x.shape(x.ndim() - 1);
  const long P = x.size() / ((long)N * C);
  need(y.size() == (long)N * C, "global pool shape");
  const float* xp = cptr(x);
  float* yp = mptr(y);
  py::gil_scoped_release nogil;
#pragma omp parallel for schedule(static)
  for (int n = 0; n < N; ++n) {
    std::vector<double> acc(C, kind == 0 ? 0.0 : -INFINITY);
    for (long p = 0; p < P; ++p) {
      const float* xv = xp + ((size_t)n * P + p) * C;
      if (kind == 0)
        for (int c = 0; c < C; ++c) acc[c] += xv[c];
      else
        for (int c = 0; c < C; ++c) acc[c] = std::max(acc[c], (double)xv[c]);
    }
    for (int c = 0; c < C; ++c) yp[(size_t)n * C + c] = kind == 0 ? (float)(acc[c] / P) : (float)acc[c];
  }
}

// ------------------------------------------------------------------ eltwise
// y = act(x * scale[c] + shift[c])   (standalone BN, Rescaling, Normalization)
void affine(const Arr<float>& x, const Arr<float>& scale, const Arr<float>& shift, Arr<float>& y, int act,
            float alpha) {
  const int C = x.shape(x.ndim() - 1);
  const long rows = x.size() / C;
  need(scale.size() == C && shift.size() == C && y.size() == x.size(), "affine shapes");
  const float *xp = cptr(x), *sp = cptr(scale), *hp = cptr(shift);
  float* yp = mptr(y);
  py::gil_scoped_release nogil;
#pragma omp parallel for schedule(static)
  for (long r = 0; r < rows; ++r)
    for (int c = 0; c < C; ++c) yp[r * C + c] = act_f(xp[r * C + c] * sp[c] + hp[c], act, alpha);
}

// y = act(x)
void activation(const Arr<float>& x, Arr<float>& y, int act, float alpha) {
  need(y.size() == x.size(), "act shapes");
  const float* xp = cptr(x);
  float* yp = mptr(y);
  const long n = x.size();
  py::gil_scoped_release nogil;
#pragma omp parallel for schedule(static)
  for (long i = 0; i < n; ++i) yp[i] = act_f(xp[i], act, alpha);
}

// y = act(a (op) b); b is either a's shape or one channel row per image
// ([N, C] broadcast over a's pixels).  op: 0 add, 1 mul, 2 sub, 3 max, 4 min, 5 avg
void binary(const Arr<float>& a, const Arr<float>& b, Arr<float>& y, int op, int act, float alpha) {
  need(y.size() == a.size(), "binary shapes");
  const int N = a.shape(0), C = a.shape(a.ndim() - 1);
  const long per = a.size() / N;
  const bool bcast = b.size() != a.size();
  need(!bcast || b.size() == (long)N * C, "binary broadcast shape");
  const float *ap = cptr(a), *bp = cptr(b);
  float* yp = mptr(y);
  const long n = a.size();
  py::gil_scoped_release nogil;
#pragma omp parallel for schedule(static)
  for (long i = 0; i < n; ++i) {
    const float u = ap[i];
    const float v = bcast ? bp[(i / per) * C + i % C] : bp[i];
    float r;
    switch (op) {
      case 0: r = u + v; break;
      case 1: r = u * v; break;
      case 2: r = u - v; break;
      case 3: r = std::max(u, v); break;
      case 4: r = std::min(u, v); break;
      default: r = 0.5f * (u + v); break;
    }
    yp[i] = act_f(r, act, alpha);
  }
}

// row softmax over the last axis (in place allowed)
void softmax(const Arr<float>& x, Arr<float>& y) {
  const int C = x.shape(x.ndim() - 1);
  const long rows = x.size() / C;
  need(y.size() == x.size(), "softmax shapes");
  const float* xp = cptr(x);
  float* yp = mptr(y);
  py::gil_scoped_release nogil;
#pragma omp parallel for schedule(static)
  for (long r = 0; r < rows; ++r) {
    const float* xr = xp + r * C;
    float* yr = yp + r * C;
    float m = -INFINITY;
    for (int c = 0; c < C; ++c) m = std::max(m, xr[c]);
    double s = 0.0;
    for (int c = 0; c < C; ++c) {
      const float e = std::exp(xr[c] - m);
      yr[c] = e;
      s += e;
    }
    const float inv = (float)(1.0 / s);
    for (int c = 0; c < C; ++c) yr[c] *= inv;
  }
}

// copy x [N,H,W,C] into y [N,H+t+b,W+l+r,C] at (t, l), zeros around
void zero_pad(const Arr<float>& x, Arr<float>& y, int t, int l) {
  const int N = x.shape(0), H = x.shape(1), W = x.shape(2), C = x.shape(3), OH = y.shape(1), OW = y.shape(2);
  const float* xp = cptr(x);
  float* yp = mptr(y);
  py::gil_scoped_release nogil;
  std::memset(yp, 0, sizeof(float) * y.size());
#pragma omp parallel for collapse(2) schedule(static)
  for (int n = 0; n < N; ++n)
    for (int h = 0; h < H; ++h)
      std::memcpy(yp + (((size_t)n * OH + h + t) * OW + l) * C, xp + (((size_t)n * H + h) * W) * C,
                  sizeof(float) * W * C);
}

// channel concat of equal-pixel tensors: y [..., sum C_i]
void concat(const py::list& xs, Arr<float>& y) {
  const int CT = y.shape(y.ndim() - 1);
  const long rows = y.size() / CT;
  std::vector<Arr<float>> ins;
  for (auto h : xs) ins.push_back(h.cast<Arr<float>>());
  float* yp = mptr(y);
  int off = 0;
  for (auto& a : ins) {
    const int C = a.shape(a.ndim() - 1);
    need(a.size() == rows * C, "concat shapes");
    const float* ap = a.data();
#pragma omp parallel for schedule(static)
    for (long r = 0; r < rows; ++r) std::memcpy(yp + r * CT + off, ap + r * C, sizeof(float) * C);
    off += C;
  }
  need(off == CT, "concat channel total");
}

int threads() { return omp_get_max_threads(); }
void set_threads(int n) { omp_set_num_threads(n); }

}  // namespace

PYBIND11_MODULE(_cpu, m) {
  m.doc() = "ADAPT native CPU ops (OpenMP, NHWC fp32): the CPU stage / local_infer execution path";
  m.attr("COB") = COB;
  m.def("conv2d", &conv2d, py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("y"), py::arg("stride"),
        py::arg("pad_t"), py::arg("pad_l"), py::arg("act") = 0, py::arg("alpha") = 0.3f,
        py::arg("residual") = py::none());
  m.def("dwconv2d", &dwconv2d, py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("y"), py::arg("stride"),
        py::arg("pad_t"), py::arg("pad_l"), py::arg("act") = 0, py::arg("alpha") = 0.3f);
  m.def("pool2d", &pool2d, py::arg("x"), py::arg("y"), py::arg("kind"), py::arg("kh"), py::arg("kw"),
        py::arg("stride"), py::arg("pad_t"), py::arg("pad_l"), py::arg("pad_zero"));
  m.def("global_pool", &global_pool, py::arg("x"), py::arg("y"), py::arg("kind") = 0);
  m.def("affine", &affine, py::arg("x"), py::arg("scale"), py::arg("shift"), py::arg("y"), py::arg("act") = 0,
        py::arg("alpha") = 0.3f);
  m.def("activation", &activation, py::arg("x"), py::arg("y"), py::arg("act"), py::arg("alpha") = 0.3f);
  m.def("binary", &binary, py::arg("a"), py::arg("b"), py::arg("y"), py::arg("op"), py::arg("act") = 0,
        py::arg("alpha") = 0.3f);
  m.def("softmax", &softmax, py::arg("x"), py::arg("y"));
  m.def("zero_pad", &zero_pad, py::arg("x"), py::arg("y"), py::arg("t"), py::arg("l"));
  m.def("concat", &concat, py::arg("xs"), py::arg("y"));
  m.def("threads", &threads);
  m.def("set_threads", &set_threads, py::arg("n"));
}
