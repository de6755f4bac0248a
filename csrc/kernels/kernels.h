// Host-visible declarations of the ADAPT gfx950 kernels.
#pragma once
#include "common.h"

namespace adapt {
struct ConvParams {
  const bf16* x;
  const bf16* w;
  const float* bias;
  const bf16* res;
  void* out;
  float* ws;
  int B, H, W, Cin;
  int OH, OW, N;
  int KH, KW, stride, pad_t, pad_l;
  int M, K, Kpad, ldo;
  int relu;         // fused activation: 0 none, 1 ReLU, 2 ReLU6 (common.h act_relu)
  int ksplit;       // >= 1: split-K slices (fp32 slabs in ws + reduce); < 0: stream-K over -ksplit x 256 blocks
  int* counters;    // stream-K: one arrival counter per output tile (zeroed, self-resetting)
  int sk_iters;     // stream-K: (tile, K-tile) iterations per block (conv_sk_plan)
  int th;           // halo 3x3 kernel: output rows per tile
  // dual-output GEMM (two sibling convs over one input, runtime/plan.py
  // merge_siblings): columns [0, n_split) -> out (row stride ldo, ReLU relu),
  // columns [n_split, N) -> out2 (row stride ldo2, ReLU relu2); 0 = one output
  int n_split;
  void* out2;
  int ldo2, relu2;
};

// where column n of the GEMM goes: destination base, column within it, row stride, ReLU
struct EpiDst {
  void* base;
  int col, ld, relu;
};
__device__ __forceinline__ EpiDst epi_dst(const ConvParams& p, int n) {
  if (p.n_split > 0 && n >= p.n_split) return EpiDst{p.out2, n - p.n_split, p.ldo2, p.relu2};
  return EpiDst{p.out, n, p.ldo, p.relu};
}
hipError_t conv_halo_launch(const ConvParams& p, int cfg, hipStream_t s, bool out_f32);
bool conv_halo_cfg(int cfg, int* bm, int* bn, int* patch_pix);
void conv_sk_plan(int tiles, int kt, int mult, int* grid, int* iters);
hipError_t conv_forward(const ConvParams& p, int cfg, hipStream_t s, bool out_f32);
int zvc_seg();
size_t zvc_scratch_bytes(size_t n, int esz);
size_t zvc_max_stream(size_t n, int esz);
hipError_t zvc_gpu_compress(const void* in, size_t n, int esz, uint8_t* scratch, uint32_t* sizes, uint32_t* offs,
                            uint8_t* out, uint64_t* total, hipStream_t s);
hipError_t zvc_gpu_decompress(const uint8_t* stream, const uint32_t* offs, int nseg, size_t n, int esz, void* out,
                              hipStream_t s);
int lz4_gpu_chunk();
size_t lz4_gpu_scratch_bytes(size_t n);
size_t lz4_gpu_max_frame(size_t n);
hipError_t lz4_gpu_compress(const uint8_t* in, size_t n, uint8_t* scratch, uint32_t* sizes, uint32_t* offs,
                            uint8_t* out, uint64_t* total, hipStream_t s);
hipError_t lz4_gpu_decompress(const uint8_t* frame, const uint32_t* offs, const uint32_t* sizes, int nchunks,
                              uint8_t* out, size_t n, int* err, hipStream_t s);
// device-resident frame + block-size table -> out (offsets scanned on the device)
hipError_t lz4_gpu_decompress_dev(const uint8_t* frame, const uint32_t* sizes, int nchunks, uint32_t* offs_scratch,
                                  uint8_t* out, size_t n, int* err, hipStream_t s);
hipError_t zvc_gpu_decompress_dev(const uint8_t* stream, int nseg, size_t n, int esz, void* out, uint32_t* offs_scratch,
                                  hipStream_t s);
hipError_t conv_glds_launch(const ConvParams& p, int cfg, hipStream_t s, bool pure, bool out_f32);
bool conv_glds_cfg_tile(int cfg, int* bm, int* bn);
int conv_num_cfgs();
void conv_cfg_tile(int cfg, int* bm, int* bn);
// diagnostic: occupy stream `s` until *flag != 0 (host-written) or timeout_ms; *out = 1 (flag) / 2 (timeout)
hipError_t spin_flag(const int* flag, int* out, double timeout_ms, hipStream_t s);
// test-only loopback link (loopback.hip): wait until *ctr >= target (or *abort_word != 0, or timeout_ms) /
// publish *ctr = value behind the stream's earlier work; ctr / abort_word / status in mapped host memory
hipError_t lb_wait(const unsigned long long* ctr, unsigned long long target, const int* abort_word, int* status,
                   double timeout_ms, hipStream_t s);
hipError_t lb_signal(unsigned long long* ctr, unsigned long long value, hipStream_t s);
hipError_t input_pack(const float* x, bf16* y, size_t pixels, int C, int Cp, hipStream_t s);
hipError_t bn_act(const bf16* x, bf16* y, const float* scale, const float* shift, size_t elems, int C, int relu,
                  hipStream_t s);
hipError_t add_act(const bf16* a, const bf16* b, bf16* y, size_t elems, int relu, hipStream_t s);
hipError_t relu(const bf16* x, bf16* y, size_t elems, int mode, hipStream_t s);   // mode: 1 ReLU, 2 ReLU6
// layers beyond ResNet (layers.hip): depthwise conv, average pool, channel concat
hipError_t dwconv(const bf16* x, const float* w, const float* bias, bf16* y, int B, int H, int W, int Cp, int OH,
                  int OW, int KH, int KW, int stride, int pad_t, int pad_l, int act, hipStream_t s);
hipError_t avgpool(const bf16* x, bf16* y, int B, int H, int W, int Cp, int OH, int OW, int KH, int KW, int S,
                   int pad_t, int pad_l, hipStream_t s);
hipError_t act(const bf16* x, bf16* y, size_t elems, int mode, float alpha, hipStream_t s);   // common.h ActMode
hipError_t binary(const bf16* a, const bf16* b, bf16* y, size_t elems, int Cp, int bcast_hw, int op, int act_mode,
                  hipStream_t s);
hipError_t gmp(const bf16* x, bf16* y, int B, int HW, int Cp, hipStream_t s);
int gap_large_slices(int B, int HW);
// GAP over large maps: part = [B][gap_large_slices][Cp] fp32 scratch
hipError_t gap_large(const bf16* x, bf16* y, float* y32, float* part, int B, int HW, int Cp, hipStream_t s);
hipError_t concat_into(const bf16* x, int Cx, int Cpx, bf16* y, int Cpy, int off, int zero_from, size_t pixels,
                       hipStream_t s);
hipError_t maxpool(const bf16* x, bf16* y, int B, int H, int W, int C, int OH, int OW, int K, int S, int pad_t,
                   int pad_l, int pad_zero, hipStream_t s);
hipError_t gap(const bf16* x, bf16* y, float* y32, int B, int HW, int C, hipStream_t s);
int dense_small_kslices(int K);
// M <= 32 rows: out = x[M][K] . w^T + bias -> logits and/or softmax(probs); part = [kslices][M][N] fp32 scratch
int dense_small_f32_kslices(int Kpad);
hipError_t dense_small_f32(const float* x, const float* w, const float* bias, float* part, float* logits,
                           float* probs, int M, int N, int K, int Kpad, hipStream_t s);
hipError_t dense_small(const bf16* x, const bf16* w, const float* bias, float* part, float* logits, float* probs,
                       int M, int N, int K, int Kpad, hipStream_t s);
hipError_t softmax_rows(const float* x, float* y, int rows, int N, int ldx, hipStream_t s);
hipError_t cast_bf16_f32(const bf16* x, float* y, size_t n, hipStream_t s);
hipError_t pad(const bf16* x, bf16* y, int B, int H, int W, int C, int OH, int OW, int pad_t, int pad_l,
               hipStream_t s);
hipError_t cast_f32_bf16(const float* x, bf16* y, size_t n, hipStream_t s);
// stem: fp32 NHWC image -> 7x7/s2 conv (+BN folded, ReLU) [-> 3x3/s2 max-pool], weights [64][224] bf16
// measurement only: per-wave phase stamps of the v4 pooled stem (8 words per wave), nullptr = off
void stem_set_debug(unsigned long long* buf, int exp = 0);
hipError_t stem_forward(const float* x, const bf16* w, const float* bias, bf16* out, int B, int H, int W, int C,
                        int OH, int OW, int pad_t, int pad_l, int pool, int PH, int PW, int pool_pad,
                        hipStream_t s);
// fp32 path (conv_f32.hip): MFMA f32 implicit-GEMM conv / GEMM and fp32 layers
struct ConvF32Params {
  const float* x;
  const float* w;
  const float* bias;
  const float* res;
  float* out;
  float* ws;
  int B, H, W, Cin;
  int OH, OW, N;
  int KH, KW, stride, pad_t, pad_l;
  int M, K, Kpad;
  int relu;
  int ksplit;       // >= 1: split-K slabs + reduce; < 0 (v2 configs): stream-K over -ksplit x 256 blocks
  int* counters;    // stream-K: one arrival counter per output tile (zeroed, self-resetting)
  int sk_iters;     // stream-K: (tile, K-tile) iterations per block (conv_f32g_sk_plan)
  float* out2;      // n_split > 0: two sibling 1x1 convs packed along N; columns >= n_split go to out2
  int n_split;      // (row stride N - n_split, activation relu2), columns < n_split to out (row stride n_split)
  int relu2;
};
void conv_f32g_sk_plan(int tiles, int kt, int mult, int* grid, int* iters);
struct F32Dst {
  float* base;
  int col, ld, relu;
};
// destination of output column n of an fp32 conv (dual output: merged sibling convs, n_split % 4 == 0)
__device__ __forceinline__ F32Dst f32_dst(const ConvF32Params& p, int n) {
  if (p.n_split > 0 && n >= p.n_split) return F32Dst{p.out2, n - p.n_split, p.N - p.n_split, p.relu2};
  return F32Dst{p.out, n, p.n_split > 0 ? p.n_split : p.N, p.relu};
}
bool conv_f32g_cfg_tile(int cfg, int* bm, int* bn);
// fp32 stem (stem_f32.hip): 7x7/s2 conv (+BN, ReLU) + 3x3/s2 max-pool, weights [64][160] fp32;
// variant 0 = one unit at a time, 1 = software-pipelined units, 2 = whole 112-wide rows (else 1)
hipError_t stem_f32_forward(const float* x, const float* w, const float* bias, float* out, int B, int H, int W, int C,
                            int OH, int OW, int pad_t, int pad_l, int PH, int PW, int pool_pad, hipStream_t s,
                            int variant = 2);
// v2 fp32 kernel family (conv_f32g.hip, cfg ids >= 10): LDS-DMA ring
bool conv_f32g_ok(int cfg, int Cin, int N);
hipError_t conv_f32g_launch(const ConvF32Params& p, int cfg, bool pure, hipStream_t s);
// fp32 Winograd F(2x2, 3x3) 3x3/s1/p1 conv (conv_wino_f32.hip, cfg ids 80-85): u = transformed weights
// in MFMA fragment order [C/16][N/16][16 positions][64 lanes][4] (ops/conv.py pack_wino_f32)
struct WinoF32Params {
  const float* x;
  const float* u;
  const float* bias;
  const float* res;
  float* out;
  float* ws;          // ksplit > 1: fp32 slabs [ksplit][B*H*W][N] (splitk_reduce_f32 adds bias / ReLU)
  int B, H, W, C, N;
  int TH, TW, T;      // 2x2 output tiles per column / row of an image, B * TH * TW
  int relu, ksplit;
  int* counters;      // fused split-K: one arrival counter per (tile group, channel group) block, zero
                      // before the launch, left zero after it (no splitk_reduce_f32 launch)
  int sk_iters;       // > 0: stream-K, (unit, chunk) iterations per block (conv_wino_sk_plan), ksplit 1
  int sk_mult;        // stream-K grid: about sk_mult x 256 blocks
  unsigned long long* dbg;   // measurement only (tools/wino_timeline.py): 16 words per block, else null
  int flags;          // F(4x4) (conv_wino4_f32.hip): 1 = segment bases aligned to the bank phase of their tiles
};
// tools/wino_timeline.py: v3 Winograd launches (PL != 0) stamp their phases into buf while it is set
void wino_set_debug(unsigned long long* buf);
void conv_wino_sk_plan(int units, int kc, int mult, int* grid, int* iters, int* smax);
bool conv_wino_f32_ok(int cfg, int C, int N);
bool conv_wino_f32_cfg(int cfg, int* nw, int* fn);
hipError_t conv_wino_f32_launch(const WinoF32Params& p, int cfg, hipStream_t s);

// fp32 Winograd F(4x4, 3x3) as transform + pure-MFMA GEMM (wino4s_f32.hip, cfg ids 220-235; the fused
// F(4x4) kernels of round 5, cfg 200 / 210, are retired to tools/experiments/): u = weights in
// fragment order [N/16][C/16][36 positions][64 lanes][4] (ops/conv.py wino4s_pack_np); ws holds V (then the
// split-K slabs), wino4s_ws_floats of it
struct Wino4sParams {
  const float* x;
  float* v;           // set by wino4s_forward (= ws)
  const float* u;
  const float* bias;
  float* out;
  float* ws;
  int B, H, W, C, N;
  int relu, ksplit;   // ksplit <= -2: fused split-K fixup (counters)
  int* counters;
  int TH, TW, T, TG, KC, order;   // derived by wino4s_forward
  unsigned long long* dbg;        // cfg 299 (measurement): 8 words per wave
};
void wino4s_set_debug(unsigned long long* buf);
bool wino4s_ok(int cfg, int C, int N, int ksplit);
int wino4s_blocks(int cfg, int B, int H, int W, int N);
size_t wino4s_ws_floats(int B, int H, int W, int C, int N, int ksplit);
hipError_t wino4s_forward(const Wino4sParams& p, int cfg, hipStream_t s);
// fp32 big-tile 1x1 GEMM (gemm_f32s.hip, cfg ids 300+): tile (BM, BN) per cfg; ksplit 1 (tiles) or -1 (stream-K
// over 256 blocks: gemm_f32s_ws_elems floats of workspace, one zeroed int32 counter per tile)
bool gemm_f32s_cfg(int cfg, int* bm, int* bn);
size_t gemm_f32s_ws_elems(int cfg);
// tools/gemm_f32s_timeline.py: launches stamp 8 words per wave into buf while it is set; exp selects a
// measurement variant (1 no LDS-DMA in the loop, 2 no MFMAs)
void gemm_f32s_set_debug(unsigned long long* buf, int exp);
hipError_t gemm_f32s_launch(const ConvF32Params& p, int cfg, hipStream_t s);
hipError_t conv_f32_forward(const float* x, const float* w, const float* bias, const float* res, float* out,
                            float* ws, int B, int H, int W, int Cin, int OH, int OW, int N, int KH, int KW,
                            int stride, int pad_t, int pad_l, int K, int Kpad, int relu, int ksplit, int cfg,
                            hipStream_t s, int* counters = nullptr, float* out2 = nullptr, int n_split = 0,
                            int relu2 = 0);
hipError_t maxpool_f32(const float* x, float* y, int B, int H, int W, int C, int OH, int OW, int K, int S, int pad_t,
                       int pad_l, int pad_zero, hipStream_t s);
hipError_t gap_f32(const float* x, float* y, int B, int HW, int C, hipStream_t s);
// fp32 GAP over large maps: part = [B][gap_large_slices][C] fp32 scratch
hipError_t gap_large_f32(const float* x, float* y, float* part, int B, int HW, int C, hipStream_t s);
// op 0: y = act(a + b); op 1: y = act(a * scale[c] + shift[c]); op 2: y = act(a)
hipError_t eltwise_f32(const float* a, const float* b, const float* scale, const float* shift, float* y, size_t n,
                       int C, int op, int relu, hipStream_t s);
hipError_t pad_f32(const float* x, float* y, int B, int H, int W, int C, int OH, int OW, int pad_t, int pad_l,
                   hipStream_t s);
hipError_t dwconv_f32(const float* x, const float* w, const float* bias, float* y, int B, int H, int W, int C, int OH,
                      int OW, int KH, int KW, int S, int pad_t, int pad_l, int act, float alpha, hipStream_t s);
hipError_t avgpool_f32(const float* x, float* y, int B, int H, int W, int C, int OH, int OW, int KH, int KW, int S,
                       int pad_t, int pad_l, hipStream_t s);
hipError_t concat_f32(const float* x, int Cx, float* y, int Cy, int off, size_t pixels, hipStream_t s);
hipError_t binary_f32(const float* a, const float* b, float* y, size_t n, int C, int bcast_hw, int op, int act,
                      hipStream_t s);
hipError_t affine_act_f32(const float* x, const float* scale, const float* shift, float* y, size_t n, int C, int act,
                          float alpha, hipStream_t s);
// reversible zfp-style float32 codec on the GPU (zfp_gpu.hip), bit-exact with the host v2 container
uint32_t zfp_gpu_maxw(int nd);
uint64_t zfp_gpu_nblocks(const int64_t* shape, int nd);
hipError_t zfp_gpu_compress(const float* src, const int64_t* shape, int nd, uint64_t* scratch, uint64_t* offs,
                            uint64_t* out, uint64_t* total, hipStream_t s);
hipError_t zfp_gpu_decompress(const uint64_t* table, const int64_t* shape, int nd, uint64_t* offs, uint64_t* total,
                              float* dst, hipStream_t s);
// fused ResNet bottleneck block (bottleneck.hip): 1x1 -> 3x3 -> 1x1 + shortcut, 8x8 tiles in LDS
struct BottleneckParams {
  const bf16* x;
  const bf16* w1;
  const bf16* w2;
  const bf16* w3;
  const float* b1;
  const float* b2;
  const float* b3;
  bf16* out;
  int B, H, W;
};
hipError_t bottleneck_forward(const BottleneckParams& p, int cin, bool proj, hipStream_t s);
// fused 1x1 pair across a ResNet block boundary (pw_pair.hip):
// y = relu(x . W3^T + b3 + res) [M][CO], z = relu(y . W1^T + b1) [M][CM]; W3 / W1 in MFMA fragment order
struct PwPairParams {
  const bf16* x;
  const bf16* w3;
  const float* b3;
  const bf16* res;
  const bf16* w1;
  const float* b1;
  bf16* y;
  bf16* z;
  int M;
};
bool pw_pair_supported(int cin, int co, int cm, int bm);
// fp32 fused 1x1 pair (pw_pair_f32.hip): ResNet stage 2, 64 -> 256 -> 64
struct PwPairF32Params {
  const float* x;
  const float* w3;
  const float* b3;
  const float* res;
  const float* w1;
  const float* b1;
  float* y;
  float* z;
  int M;
};
bool pw_pair_f32_supported(int cin, int co, int cm, int bm);
// fp32 persistent pointwise conv, filter slice register-resident (pw_f32.hip)
struct PwF32Params {
  const float* x;
  const float* w;      // fragment-packed [N/16][K/16][64 lanes][4]
  const float* bias;
  const float* res;
  float* out;
  int M, K, N, relu;
  int B, H, W, OH, OW, stride;   // input / output maps (stride-s 1x1: M = B x OH x OW)
  float* out2;         // n_split > 0: columns >= n_split go to out2 (row stride N - n_split, relu2)
  int n_split, relu2;
  unsigned long long* dbg = nullptr;   // streaming kernels: 16 stamps per wave (tools/pw_timeline.py)
};
void pw_set_debug(unsigned long long* buf);
int pw_f32_fpw(int K, int N, int n_split, int bm);
void pw_f32_tail_plan(int M, int K, int N, int n_split, int bm, int* tail_tiles, int* parts);
bool pw_f32_supported(int K, int N, int bm);
hipError_t pw_f32_forward(const PwF32Params& p, int bm, hipStream_t s);
hipError_t pw_pair_f32_forward(const PwPairF32Params& p, int cin, int co, int cm, int bm, int grid, hipStream_t s);
// 3x3 / s1 / p1 conv with the filter resident in VGPRs (conv3x3_rr.hip): out = act(conv(x) + bias)
struct Conv3x3RRParams {
  const bf16* x;
  const bf16* wfrag;   // [Npad][9*C] packed in MFMA fragment order
  const float* bias;
  bf16* out;
  int B;
  int relu;
};
bool conv3x3_rr_supported(int C, int H, int W);
hipError_t conv3x3_rr_forward(const Conv3x3RRParams& p, int C, int H, int W, int kg, hipStream_t s);
// channel-split register-resident 3x3 (conv3x3_cs.hip): stage 4 (256, 14x14) and stage 5 (512, 7x7)
bool conv3x3_cs_supported(int C, int H, int W);
hipError_t conv3x3_cs_forward(const Conv3x3RRParams& p, int C, int H, int W, hipStream_t s);
hipError_t pw_pair_forward(const PwPairParams& p, int cin, int co, int cm, int bm, hipStream_t s);
// persistent pointwise conv, weights register-resident per wave (pw_wide.hip):
// out[m][n] = act(x[m] . W[n] + bias[n] (+ res[m][n])), x [M][K], W in MFMA fragment order
struct PwParams {
  const bf16* x;
  const bf16* w;
  const float* bias;
  const bf16* res;
  bf16* out;
  int M;
  int relu;
};
int pw_res_supported(int K, int N);
hipError_t pw_res_forward(const PwParams& p, int K, int N, int pt, int blocks, hipStream_t s);
// channel-sliced persistent pointwise (pw_slice.hip): code -> (channel fragments per wave, waves, pixels per tile)
bool pw_slice_cfg(int code, int* cf, int* waves, int* pt);
int pw_slice_supported(int K, int N, int code);
hipError_t pw_slice_forward(const PwParams& p, int K, int N, int code, int blocks, hipStream_t s);
// serving ingest (ingest.hip): uint8 NHWC -> fp32, y = x[rev(c)] * scale[c] + shift[c] (host scale/shift, C <= 4)
hipError_t ingest_u8(const uint8_t* x, float* y, size_t n, int C, int reverse, const float* scale,
                     const float* shift, hipStream_t s);
}  // namespace adapt
