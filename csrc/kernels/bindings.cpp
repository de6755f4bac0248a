// pybind11 bindings for the gfx950 kernels.  Tensors cross the boundary as
// raw device pointers (uintptr_t) plus the HIP stream handle of the caller's
// current torch stream, so launches are captured by hipGraphs the runtime
// records (runtime/executor.py).  Shape checks happen on the host in
// ops/*.py before any launch.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "kernels.h"



namespace py = pybind11;
using u64 = uintptr_t;

static void check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
template <typename T>
static T* P(u64 v) { return reinterpret_cast<T*>(v); }
static hipStream_t S(u64 v) { return reinterpret_cast<hipStream_t>(v); }

PYBIND11_MODULE(_C, m) {
  m.doc() = "ADAPT MI355X (gfx950) HIP kernels";
  m.def("conv_num_cfgs", &adapt::conv_num_cfgs);
  m.def("conv_halo_cfg", [](int cfg) -> py::object {
    int bm, bn, pp;
    if (!adapt::conv_halo_cfg(cfg, &bm, &bn, &pp)) return py::none();
    return py::make_tuple(bm, bn, pp);
  });
  m.def("conv_sk_plan", [](int tiles, int kt, int mult) {
    int g, it;
    adapt::conv_sk_plan(tiles, kt, mult, &g, &it);
    return py::make_tuple(g, it);
  });
  m.def("conv_cfg_tile", [](int cfg) {
    int bm, bn;
    adapt::conv_cfg_tile(cfg, &bm, &bn);
    return py::make_tuple(bm, bn);
  });
  m.def(
      "conv_forward",
      [](u64 x, u64 w, u64 bias, u64 res, u64 out, u64 ws, u64 counters, int sk_iters, int th, int B, int H, int W,
         int Cin, int OH, int OW, int N, int KH, int KW, int stride, int pad_t, int pad_l, int K, int Kpad, int ldo,
         int relu, int ksplit, int cfg, bool out_f32, u64 stream, u64 out2, int n_split, int relu2) {
        adapt::ConvParams p;
        p.x = P<const bf16>(x);
        p.w = P<const bf16>(w);
        p.bias = P<const float>(bias);
        p.res = P<const bf16>(res);
        p.out = P<void>(out);
        p.ws = P<float>(ws);
        p.counters = P<int>(counters);
        p.sk_iters = sk_iters;
        p.th = th;
        p.B = B; p.H = H; p.W = W; p.Cin = Cin;
        p.OH = OH; p.OW = OW; p.N = N;
        p.KH = KH; p.KW = KW; p.stride = stride; p.pad_t = pad_t; p.pad_l = pad_l;
        p.M = B * OH * OW; p.K = K; p.Kpad = Kpad; p.ldo = ldo;
        // ksplit > 1: split-K slabs; < 0: stream-K over -ksplit x 256 blocks (v2 configs)
        p.relu = relu; p.ksplit = ksplit == 0 ? 1 : ksplit;
        p.n_split = n_split; p.out2 = P<void>(out2); p.relu2 = relu2; p.ldo2 = N - n_split;
        py::gil_scoped_release nogil;
        check(adapt::conv_forward(p, cfg, S(stream), out_f32), "conv_forward");
      },
      py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("res"), py::arg("out"), py::arg("ws"), py::arg("counters"),
      py::arg("sk_iters"), py::arg("th"), py::arg("B"), py::arg("H"), py::arg("W"), py::arg("Cin"), py::arg("OH"),
      py::arg("OW"), py::arg("N"), py::arg("KH"), py::arg("KW"), py::arg("stride"), py::arg("pad_t"), py::arg("pad_l"),
      py::arg("K"), py::arg("Kpad"), py::arg("ldo"), py::arg("relu"), py::arg("ksplit"), py::arg("cfg"),
      py::arg("out_f32"), py::arg("stream"), py::arg("out2") = 0, py::arg("n_split") = 0, py::arg("relu2") = 0);
  m.def("zvc_seg", &adapt::zvc_seg);
  m.def("zvc_scratch_bytes", &adapt::zvc_scratch_bytes);
  m.def("zvc_max_stream", &adapt::zvc_max_stream);
  m.def("zvc_gpu_compress", [](u64 in, size_t n, int esz, u64 scratch, u64 sizes, u64 offs, u64 out, u64 total,
                               u64 s) {
    check(adapt::zvc_gpu_compress(P<const void>(in), n, esz, P<uint8_t>(scratch), P<uint32_t>(sizes),
                                  P<uint32_t>(offs), P<uint8_t>(out), P<uint64_t>(total), S(s)),
          "zvc_gpu_compress");
  });
  m.def("zvc_gpu_decompress", [](u64 stream, u64 offs, int nseg, size_t n, int esz, u64 out, u64 s) {
    check(adapt::zvc_gpu_decompress(P<const uint8_t>(stream), P<const uint32_t>(offs), nseg, n, esz, P<void>(out),
                                    S(s)),
          "zvc_gpu_decompress");
  });
  m.def("lz4_gpu_chunk", &adapt::lz4_gpu_chunk);
  m.def("lz4_gpu_scratch_bytes", &adapt::lz4_gpu_scratch_bytes);
  m.def("lz4_gpu_max_frame", &adapt::lz4_gpu_max_frame);
  m.def("lz4_gpu_compress", [](u64 in, size_t n, u64 scratch, u64 sizes, u64 offs, u64 out, u64 total, u64 s) {
    check(adapt::lz4_gpu_compress(P<const uint8_t>(in), n, P<uint8_t>(scratch), P<uint32_t>(sizes),
                                  P<uint32_t>(offs), P<uint8_t>(out), P<uint64_t>(total), S(s)),
          "lz4_gpu_compress");
  });
  m.def("lz4_gpu_decompress", [](u64 frame, u64 offs, u64 sizes, int nchunks, u64 out, size_t n, u64 err, u64 s) {
    check(adapt::lz4_gpu_decompress(P<const uint8_t>(frame), P<const uint32_t>(offs), P<const uint32_t>(sizes),
                                    nchunks, P<uint8_t>(out), n, P<int>(err), S(s)),
          "lz4_gpu_decompress");
  });
  m.def("lz4_gpu_decompress_dev", [](u64 frame, u64 sizes, int nchunks, u64 offs, u64 out, size_t n, u64 err, u64 s) {
    check(adapt::lz4_gpu_decompress_dev(P<const uint8_t>(frame), P<const uint32_t>(sizes), nchunks, P<uint32_t>(offs),
                                        P<uint8_t>(out), n, P<int>(err), S(s)),
          "lz4_gpu_decompress_dev");
  });
  m.def("zvc_gpu_decompress_dev", [](u64 stream, int nseg, size_t n, int esz, u64 out, u64 offs, u64 s) {
    check(adapt::zvc_gpu_decompress_dev(P<const uint8_t>(stream), nseg, n, esz, P<void>(out), P<uint32_t>(offs), S(s)),
          "zvc_gpu_decompress_dev");
  });
  m.def("stem_set_debug", [](u64 buf, int exp) { adapt::stem_set_debug(reinterpret_cast<unsigned long long*>(buf), exp); },
        py::arg("buf"), py::arg("exp") = 0);
  m.def("stem_forward", [](u64 x, u64 w, u64 bias, u64 out, int B, int H, int W, int C, int OH, int OW, int pad_t,
                           int pad_l, int pool, int PH, int PW, int pool_pad, u64 s) {
    check(adapt::stem_forward(P<const float>(x), P<const bf16>(w), P<const float>(bias), P<bf16>(out), B, H, W, C,
                              OH, OW, pad_t, pad_l, pool, PH, PW, pool_pad, S(s)),
          "stem_forward");
  });
  m.def("lb_wait", [](u64 ctr, unsigned long long target, u64 abort_word, u64 status, double timeout_ms, u64 s) {
    check(adapt::lb_wait(P<const unsigned long long>(ctr), target, P<const int>(abort_word), P<int>(status),
                         timeout_ms, S(s)),
          "lb_wait");
  });
  m.def("lb_signal", [](u64 ctr, unsigned long long value, u64 s) {
    check(adapt::lb_signal(P<unsigned long long>(ctr), value, S(s)), "lb_signal");
  });
  // page-lock a host range for the GPU (mapped, portable) and return its device address
  m.def("host_register", [](u64 ptr, size_t n) {
    check(hipHostRegister(reinterpret_cast<void*>(ptr), n, hipHostRegisterMapped | hipHostRegisterPortable),
          "host_register");
    void* d = nullptr;
    check(hipHostGetDevicePointer(&d, reinterpret_cast<void*>(ptr), 0), "host_register: device pointer");
    return reinterpret_cast<u64>(d);
  });
  m.def("host_unregister", [](u64 ptr) { check(hipHostUnregister(reinterpret_cast<void*>(ptr)), "host_unregister"); });
  m.def("spin_flag", [](u64 flag, u64 out, double timeout_ms, u64 s) {
    check(adapt::spin_flag(P<const int>(flag), P<int>(out), timeout_ms, S(s)), "spin_flag");
  });
  m.def("input_pack", [](u64 x, u64 y, size_t pixels, int C, int Cp, u64 s) {
    check(adapt::input_pack(P<const float>(x), P<bf16>(y), pixels, C, Cp, S(s)), "input_pack");
  });
  m.def("bn_act", [](u64 x, u64 y, u64 scale, u64 shift, size_t elems, int C, int relu, u64 s) {
    check(adapt::bn_act(P<const bf16>(x), P<bf16>(y), P<const float>(scale), P<const float>(shift), elems, C, relu,
                        S(s)), "bn_act");
  });
  m.def("add_act", [](u64 a, u64 b, u64 y, size_t elems, int relu, u64 s) {
    check(adapt::add_act(P<const bf16>(a), P<const bf16>(b), P<bf16>(y), elems, relu, S(s)), "add_act");
  });
  m.def("relu", [](u64 x, u64 y, size_t elems, int mode, u64 s) {
    check(adapt::relu(P<const bf16>(x), P<bf16>(y), elems, mode, S(s)), "relu");
  });
  m.def("dwconv", [](u64 x, u64 w, u64 bias, u64 y, int B, int H, int W, int Cp, int OH, int OW, int KH, int KW,
                     int stride, int pad_t, int pad_l, int act, u64 s) {
    check(adapt::dwconv(P<const bf16>(x), P<const float>(w), P<const float>(bias), P<bf16>(y), B, H, W, Cp, OH, OW,
                        KH, KW, stride, pad_t, pad_l, act, S(s)), "dwconv");
  });
  m.def("avgpool", [](u64 x, u64 y, int B, int H, int W, int Cp, int OH, int OW, int KH, int KW, int Sd, int pad_t,
                      int pad_l, u64 s) {
    check(adapt::avgpool(P<const bf16>(x), P<bf16>(y), B, H, W, Cp, OH, OW, KH, KW, Sd, pad_t, pad_l, S(s)),
          "avgpool");
  });
  m.def("act", [](u64 x, u64 y, size_t elems, int mode, float alpha, u64 s) {
    check(adapt::act(P<const bf16>(x), P<bf16>(y), elems, mode, alpha, S(s)), "act");
  });
  m.def("binary", [](u64 a, u64 b, u64 y, size_t elems, int Cp, int bcast_hw, int op, int act_mode, u64 s) {
    check(adapt::binary(P<const bf16>(a), P<const bf16>(b), P<bf16>(y), elems, Cp, bcast_hw, op, act_mode, S(s)),
          "binary");
  });
  m.def("gap_large_slices", &adapt::gap_large_slices);
  m.def("gap_large", [](u64 x, u64 y, u64 y32, u64 part, int B, int HW, int Cp, u64 s) {
    check(adapt::gap_large(P<const bf16>(x), P<bf16>(y), P<float>(y32), P<float>(part), B, HW, Cp, S(s)),
          "gap_large");
  });
  m.def("gmp", [](u64 x, u64 y, int B, int HW, int Cp, u64 s) {
    check(adapt::gmp(P<const bf16>(x), P<bf16>(y), B, HW, Cp, S(s)), "gmp");
  });
  m.def("concat_into", [](u64 x, int Cx, int Cpx, u64 y, int Cpy, int off, int zero_from, size_t pixels, u64 s) {
    check(adapt::concat_into(P<const bf16>(x), Cx, Cpx, P<bf16>(y), Cpy, off, zero_from, pixels, S(s)),
          "concat_into");
  });
  m.def("maxpool", [](u64 x, u64 y, int B, int H, int W, int C, int OH, int OW, int K, int Sd, int pad_t, int pad_l,
                      int pad_zero, u64 s) {
    check(adapt::maxpool(P<const bf16>(x), P<bf16>(y), B, H, W, C, OH, OW, K, Sd, pad_t, pad_l, pad_zero, S(s)),
          "maxpool");
  });
  m.def("dense_small_kslices", &adapt::dense_small_kslices);
  m.def("dense_small", [](u64 x, u64 w, u64 bias, u64 part, u64 logits, u64 probs, int M, int N, int K, int Kpad,
                          u64 s) {
    check(adapt::dense_small(P<const bf16>(x), P<const bf16>(w), P<const float>(bias), P<float>(part),
                             P<float>(logits), P<float>(probs), M, N, K, Kpad, S(s)),
          "dense_small");
  });
  m.def("pw_f32_supported", &adapt::pw_f32_supported);
  m.def("pw_f32_forward", [](u64 x, u64 w, u64 bias, u64 res, u64 out, int M, int K, int N, int relu, int bm, u64 s,
                             int B, int H, int W, int OH, int OW, int stride, u64 out2, int n_split, int relu2) {
    adapt::PwF32Params p{P<const float>(x), P<const float>(w), P<const float>(bias), P<const float>(res), P<float>(out),
                         M, K, N, relu, B, H, W, OH, OW, stride, P<float>(out2), n_split, relu2};
    check(adapt::pw_f32_forward(p, bm, S(s)), "pw_f32_forward");
  }, py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("res"), py::arg("out"), py::arg("M"), py::arg("K"),
     py::arg("N"), py::arg("relu"), py::arg("bm"), py::arg("s"), py::arg("B"), py::arg("H"), py::arg("W"),
     py::arg("OH"), py::arg("OW"), py::arg("stride"), py::arg("out2") = 0, py::arg("n_split") = 0,
     py::arg("relu2") = 0);
  m.def("pw_f32_fpw", &adapt::pw_f32_fpw);
  m.def("wino4s_forward", [](u64 x, u64 u, u64 bias, u64 out, u64 ws, int B, int H, int W, int C, int N, int relu,
                             int ksplit, int cfg, u64 s, u64 counters) {
    adapt::Wino4sParams p{};
    p.x = P<const float>(x);
    p.u = P<const float>(u);
    p.bias = P<const float>(bias);
    p.out = P<float>(out);
    p.ws = P<float>(ws);
    p.B = B; p.H = H; p.W = W; p.C = C; p.N = N; p.relu = relu; p.ksplit = ksplit;
    p.counters = P<int>(counters);
    check(adapt::wino4s_forward(p, cfg, S(s)), "wino4s_forward");
  }, py::arg("x"), py::arg("u"), py::arg("bias"), py::arg("out"), py::arg("ws"), py::arg("B"), py::arg("H"),
     py::arg("W"), py::arg("C"), py::arg("N"), py::arg("relu"), py::arg("ksplit"), py::arg("cfg"), py::arg("s"),
     py::arg("counters") = 0);
  m.def("wino4s_blocks", &adapt::wino4s_blocks);
  m.def("wino4s_set_debug", [](u64 buf) { adapt::wino4s_set_debug(P<unsigned long long>(buf)); });
  m.def("wino4s_ok", &adapt::wino4s_ok);
  m.def("wino4s_ws_floats", &adapt::wino4s_ws_floats);
  m.def("pw_f32_tail_plan", [](int M, int K, int N, int n_split, int bm) {
    int tail = 0, parts = 0;
    adapt::pw_f32_tail_plan(M, K, N, n_split, bm, &tail, &parts);
    return py::make_tuple(tail, parts);
  });
  m.def("pw_pair_f32_supported", &adapt::pw_pair_f32_supported);
  m.def("pw_pair_f32_forward", [](u64 x, u64 w3, u64 b3, u64 res, u64 w1, u64 b1, u64 y, u64 z, int M, int cin,
                                  int co, int cm, int bm, int grid, u64 s) {
    adapt::PwPairF32Params p{P<const float>(x), P<const float>(w3), P<const float>(b3), P<const float>(res),
                             P<const float>(w1), P<const float>(b1), P<float>(y), P<float>(z), M};
    check(adapt::pw_pair_f32_forward(p, cin, co, cm, bm, grid, S(s)), "pw_pair_f32_forward");
  });
  m.def("dense_small_f32_kslices", &adapt::dense_small_f32_kslices);
  m.def("dense_small_f32", [](u64 x, u64 w, u64 bias, u64 part, u64 logits, u64 probs, int M, int N, int K,
                              int Kpad, u64 s) {
    check(adapt::dense_small_f32(P<const float>(x), P<const float>(w), P<const float>(bias), P<float>(part),
                                 P<float>(logits), P<float>(probs), M, N, K, Kpad, S(s)),
          "dense_small_f32");
  });
  m.def("gap", [](u64 x, u64 y, u64 y32, int B, int HW, int C, u64 s) {
    check(adapt::gap(P<const bf16>(x), P<bf16>(y), P<float>(y32), B, HW, C, S(s)), "gap");
  });
  m.def("softmax_rows", [](u64 x, u64 y, int rows, int N, int ldx, u64 s) {
    check(adapt::softmax_rows(P<const float>(x), P<float>(y), rows, N, ldx, S(s)), "softmax_rows");
  });
  m.def("pad", [](u64 x, u64 y, int B, int H, int W, int C, int OH, int OW, int pt, int pl, u64 s) {
    check(adapt::pad(P<const bf16>(x), P<bf16>(y), B, H, W, C, OH, OW, pt, pl, S(s)), "pad");
  });
  m.def("cast_bf16_f32", [](u64 x, u64 y, size_t n, u64 s) {
    check(adapt::cast_bf16_f32(P<const bf16>(x), P<float>(y), n, S(s)), "cast_bf16_f32");
  });
  m.def("conv_f32_forward", [](u64 x, u64 w, u64 bias, u64 res, u64 out, u64 ws, int B, int H, int W, int Cin,
                               int OH, int OW, int N, int KH, int KW, int stride, int pad_t, int pad_l, int K,
                               int Kpad, int relu, int ksplit, int cfg, u64 s, u64 counters, u64 out2, int n_split,
                               int relu2) {
    py::gil_scoped_release nogil;
    check(adapt::conv_f32_forward(P<const float>(x), P<const float>(w), P<const float>(bias), P<const float>(res),
                                  P<float>(out), P<float>(ws), B, H, W, Cin, OH, OW, N, KH, KW, stride, pad_t, pad_l,
                                  K, Kpad, relu, ksplit, cfg, S(s), P<int>(counters), P<float>(out2), n_split, relu2),
          "conv_f32_forward");
  }, py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("res"), py::arg("out"), py::arg("ws"), py::arg("B"),
     py::arg("H"), py::arg("W"), py::arg("Cin"), py::arg("OH"), py::arg("OW"), py::arg("N"), py::arg("KH"),
     py::arg("KW"), py::arg("stride"), py::arg("pad_t"), py::arg("pad_l"), py::arg("K"), py::arg("Kpad"),
     py::arg("relu"), py::arg("ksplit"), py::arg("cfg"), py::arg("s"), py::arg("counters") = 0,
     py::arg("out2") = 0, py::arg("n_split") = 0, py::arg("relu2") = 0);
  m.def("conv_wino_sk_plan", [](int units, int kc, int mult) {
    int g, it, smax;
    adapt::conv_wino_sk_plan(units, kc, mult, &g, &it, &smax);
    return py::make_tuple(g, it, smax);
  });
  m.def("conv_f32g_sk_plan", [](int tiles, int kt, int mult) {
    int g = 0, it = 0;
    adapt::conv_f32g_sk_plan(tiles, kt, mult, &g, &it);
    return std::make_pair(g, it);
  });
  m.def("wino_set_debug", [](u64 buf) { adapt::wino_set_debug(P<unsigned long long>(buf)); });
  m.def("gemm_f32s_cfg", [](int cfg) {
    int bm = 0, bn = 0;
    const bool ok = adapt::gemm_f32s_cfg(cfg, &bm, &bn);
    return py::make_tuple(ok ? bm : 0, ok ? bn : 0);
  });
  m.def("gemm_f32s_ws_elems", &adapt::gemm_f32s_ws_elems);
  m.def("gemm_f32s_set_debug", [](u64 buf, int exp) { adapt::gemm_f32s_set_debug(P<unsigned long long>(buf), exp); },
        py::arg("buf"), py::arg("exp") = 0);
  m.def("pw_set_debug", [](u64 buf) { adapt::pw_set_debug(P<unsigned long long>(buf)); });
  m.def("stem_f32_forward", [](u64 x, u64 w, u64 bias, u64 out, int B, int H, int W, int C, int OH, int OW,
                               int pad_t, int pad_l, int PH, int PW, int pool_pad, u64 s, int variant) {
    py::gil_scoped_release nogil;
    check(adapt::stem_f32_forward(P<const float>(x), P<const float>(w), P<const float>(bias), P<float>(out), B, H, W,
                                  C, OH, OW, pad_t, pad_l, PH, PW, pool_pad, S(s), variant),
          "stem_f32_forward");
  });
  m.def("maxpool_f32", [](u64 x, u64 y, int B, int H, int W, int C, int OH, int OW, int K, int Sd, int pad_t,
                          int pad_l, int pad_zero, u64 s) {
    check(adapt::maxpool_f32(P<const float>(x), P<float>(y), B, H, W, C, OH, OW, K, Sd, pad_t, pad_l, pad_zero,
                             S(s)), "maxpool_f32");
  });
  m.def("gap_f32", [](u64 x, u64 y, int B, int HW, int C, u64 s) {
    check(adapt::gap_f32(P<const float>(x), P<float>(y), B, HW, C, S(s)), "gap_f32");
  });
  // a HIP stream of the caller's own: PyTorch's torch.cuda.Stream() hands out pool streams round-robin, so a
  // serving thread's copy stream could be the very stream another thread is capturing a graph on
  m.def("stream_create", []() {
    hipStream_t st = nullptr;
    check(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "stream_create");
    return (u64)(uintptr_t)st;
  });
  m.def("stream_destroy", [](u64 st) { check(hipStreamDestroy((hipStream_t)(uintptr_t)st), "stream_destroy"); });
  // device link slots (transport/shm.py DeviceLinkPool): one allocation per slot, exported by IPC handle
  m.def("dev_alloc", [](size_t n) {
    void* p = nullptr;
    check(hipMalloc(&p, n), "dev_alloc");
    return (u64)(uintptr_t)p;
  });
  m.def("dev_free", [](u64 p) { check(hipFree((void*)(uintptr_t)p), "dev_free"); });
  m.def("ipc_handle", [](u64 p) {
    hipIpcMemHandle_t h;
    check(hipIpcGetMemHandle(&h, (void*)(uintptr_t)p), "ipc_handle");
    return py::bytes(reinterpret_cast<const char*>(&h), sizeof(h));
  });
  // open a device link slot exported by another process; `peer` = the exporter's
  // device ordinal (-1 unknown): when it differs from this thread's device, peer
  // access to it is enabled explicitly first, so the copy out of the slot is a
  // direct xGMI peer read rather than whatever the lazy mapping falls back to
  m.def("ipc_open", [](py::bytes hb, int peer) {
    std::string b = hb;
    if (b.size() != sizeof(hipIpcMemHandle_t)) throw std::runtime_error("ipc_open: bad handle size");
    hipIpcMemHandle_t h;
    std::memcpy(&h, b.data(), sizeof(h));
    int cur = 0;
    check(hipGetDevice(&cur), "ipc_open: hipGetDevice");
    if (peer >= 0 && peer != cur) {
      int can = 0;
      check(hipDeviceCanAccessPeer(&can, cur, peer), "ipc_open: hipDeviceCanAccessPeer");
      if (!can) throw std::runtime_error("ipc_open: device " + std::to_string(cur) + " cannot access peer " +
                                         std::to_string(peer));
      hipError_t e = hipDeviceEnablePeerAccess(peer, 0);
      if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) check(e, "ipc_open: hipDeviceEnablePeerAccess");
      (void)hipGetLastError();               // clear a sticky "already enabled"
    }
    void* p = nullptr;
    check(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "ipc_open");
    return (u64)(uintptr_t)p;
  }, py::arg("handle"), py::arg("peer") = -1);
  m.def("device_of", [](u64 p) {
    hipPointerAttribute_t a;
    check(hipPointerGetAttributes(&a, (const void*)(uintptr_t)p), "device_of");
    return a.device;
  });
  m.def("ipc_close", [](u64 p) { check(hipIpcCloseMemHandle((void*)(uintptr_t)p), "ipc_close"); });
  m.def("memcpy_async", [](u64 dst, u64 src, size_t n, u64 st) {
    check(hipMemcpyAsync((void*)(uintptr_t)dst, (const void*)(uintptr_t)src, n, hipMemcpyDefault, S(st)),
          "memcpy_async");
  });
  m.def("pw_res_supported", [](int K, int N) { return adapt::pw_res_supported(K, N) != 0; });
  m.def("pw_res_forward", [](u64 x, u64 w, u64 bias, u64 res, u64 out, int M, int K, int N, int relu, int pt,
                             int blocks, u64 s) {
    adapt::PwParams p{P<const bf16>(x), P<const bf16>(w), P<const float>(bias), P<const bf16>(res), P<bf16>(out), M,
                      relu};
    check(adapt::pw_res_forward(p, K, N, pt, blocks, S(s)), "pw_res_forward");
  });
  m.def("pw_slice_supported", [](int K, int N, int code) { return adapt::pw_slice_supported(K, N, code) != 0; });
  m.def("pw_slice_forward", [](u64 x, u64 w, u64 bias, u64 res, u64 out, int M, int K, int N, int relu, int code,
                               int blocks, u64 s) {
    adapt::PwParams p{P<const bf16>(x), P<const bf16>(w), P<const float>(bias), P<const bf16>(res), P<bf16>(out), M,
                      relu};
    check(adapt::pw_slice_forward(p, K, N, code, blocks, S(s)), "pw_slice_forward");
  });
  m.def("gap_large_f32", [](u64 x, u64 y, u64 part, int B, int HW, int C, u64 s) {
    check(adapt::gap_large_f32(P<const float>(x), P<float>(y), P<float>(part), B, HW, C, S(s)), "gap_large_f32");
  });
  m.def("eltwise_f32", [](u64 a, u64 b, u64 scale, u64 shift, u64 y, size_t n, int C, int op, int relu, u64 s) {
    check(adapt::eltwise_f32(P<const float>(a), P<const float>(b), P<const float>(scale), P<const float>(shift),
                             P<float>(y), n, C, op, relu, S(s)), "eltwise_f32");
  });
  m.def("pad_f32", [](u64 x, u64 y, int B, int H, int W, int C, int OH, int OW, int pt, int pl, u64 s) {
    check(adapt::pad_f32(P<const float>(x), P<float>(y), B, H, W, C, OH, OW, pt, pl, S(s)), "pad_f32");
  });
  m.def("dwconv_f32", [](u64 x, u64 w, u64 b, u64 y, int B, int H, int W, int C, int OH, int OW, int KH, int KW,
                         int Sd, int pt, int pl, int act, float alpha, u64 s) {
    check(adapt::dwconv_f32(P<const float>(x), P<const float>(w), P<const float>(b), P<float>(y), B, H, W, C, OH, OW,
                            KH, KW, Sd, pt, pl, act, alpha, S(s)), "dwconv_f32");
  });
  m.def("avgpool_f32", [](u64 x, u64 y, int B, int H, int W, int C, int OH, int OW, int KH, int KW, int Sd, int pt,
                          int pl, u64 s) {
    check(adapt::avgpool_f32(P<const float>(x), P<float>(y), B, H, W, C, OH, OW, KH, KW, Sd, pt, pl, S(s)),
          "avgpool_f32");
  });
  m.def("concat_f32", [](u64 x, int Cx, u64 y, int Cy, int off, size_t pixels, u64 s) {
    check(adapt::concat_f32(P<const float>(x), Cx, P<float>(y), Cy, off, pixels, S(s)), "concat_f32");
  });
  m.def("binary_f32", [](u64 a, u64 b, u64 y, size_t n, int C, int bcast_hw, int op, int act, u64 s) {
    check(adapt::binary_f32(P<const float>(a), P<const float>(b), P<float>(y), n, C, bcast_hw, op, act, S(s)),
          "binary_f32");
  });
  m.def("affine_act_f32", [](u64 x, u64 sc, u64 sh, u64 y, size_t n, int C, int act, float alpha, u64 s) {
    check(adapt::affine_act_f32(P<const float>(x), P<const float>(sc), P<const float>(sh), P<float>(y), n, C, act,
                                alpha, S(s)), "affine_act_f32");
  });
  m.def("zfp_gpu_maxw", &adapt::zfp_gpu_maxw);
  m.def("zfp_gpu_nblocks", [](std::vector<int64_t> shape) {
    return adapt::zfp_gpu_nblocks(shape.data(), (int)shape.size());
  });
  m.def("zfp_gpu_compress", [](u64 src, std::vector<int64_t> shape, u64 scratch, u64 offs, u64 out, u64 total,
                               u64 s) {
    check(adapt::zfp_gpu_compress(P<const float>(src), shape.data(), (int)shape.size(), P<uint64_t>(scratch),
                                  P<uint64_t>(offs), P<uint64_t>(out), P<uint64_t>(total), S(s)),
          "zfp_gpu_compress");
  });
  m.def("zfp_gpu_decompress", [](u64 table, std::vector<int64_t> shape, u64 offs, u64 total, u64 dst, u64 s) {
    check(adapt::zfp_gpu_decompress(P<const uint64_t>(table), shape.data(), (int)shape.size(), P<uint64_t>(offs),
                                    P<uint64_t>(total), P<float>(dst), S(s)),
          "zfp_gpu_decompress");
  });
  m.def("bottleneck_forward", [](u64 x, u64 w1, u64 w2, u64 w3, u64 b1, u64 b2, u64 b3, u64 out, int B, int H, int W,
                                 int cin, bool proj, u64 s) {
    adapt::BottleneckParams p{P<const bf16>(x), P<const bf16>(w1), P<const bf16>(w2), P<const bf16>(w3),
                              P<const float>(b1), P<const float>(b2), P<const float>(b3), P<bf16>(out), B, H, W};
    check(adapt::bottleneck_forward(p, cin, proj, S(s)), "bottleneck_forward");
  });
  m.def("pw_pair_forward", [](u64 x, u64 w3, u64 b3, u64 res, u64 w1, u64 b1, u64 y, u64 z, int M, int cin, int co,
                              int cm, int bm, u64 s) {
    adapt::PwPairParams p{P<const bf16>(x), P<const bf16>(w3), P<const float>(b3), P<const bf16>(res),
                          P<const bf16>(w1), P<const float>(b1), P<bf16>(y), P<bf16>(z), M};
    check(adapt::pw_pair_forward(p, cin, co, cm, bm, S(s)), "pw_pair_forward");
  });
  m.def("conv3x3_rr_forward", [](u64 x, u64 wfrag, u64 bias, u64 out, int B, int H, int W, int C, int relu, int kg,
                                 u64 s) {
    adapt::Conv3x3RRParams p{P<const bf16>(x), P<const bf16>(wfrag), P<const float>(bias), P<bf16>(out), B, relu};
    check(adapt::conv3x3_rr_forward(p, C, H, W, kg, S(s)), "conv3x3_rr_forward");
  });
  m.def("conv3x3_cs_forward", [](u64 x, u64 wfrag, u64 bias, u64 out, int B, int H, int W, int C, int relu, u64 s) {
    adapt::Conv3x3RRParams p{P<const bf16>(x), P<const bf16>(wfrag), P<const float>(bias), P<bf16>(out), B, relu};
    check(adapt::conv3x3_cs_forward(p, C, H, W, S(s)), "conv3x3_cs_forward");
  });
  m.def("conv3x3_cs_supported", [](int C, int H, int W) { return adapt::conv3x3_cs_supported(C, H, W); });
  m.def("pw_pair_supported", [](int cin, int co, int cm, int bm) { return adapt::pw_pair_supported(cin, co, cm, bm); });
  m.def("ingest_u8", [](u64 x, u64 y, size_t n, int C, int reverse, std::vector<float> scale,
                        std::vector<float> shift, u64 s) {
    if ((int)scale.size() < C || (int)shift.size() < C) throw std::runtime_error("ingest_u8: scale/shift per channel");
    check(adapt::ingest_u8(P<const uint8_t>(x), P<float>(y), n, C, reverse, scale.data(), shift.data(), S(s)),
          "ingest_u8");
  });
  m.def("cast_f32_bf16", [](u64 x, u64 y, size_t n, u64 s) {
    check(adapt::cast_f32_bf16(P<const float>(x), P<bf16>(y), n, S(s)), "cast_f32_bf16");
  });
}
