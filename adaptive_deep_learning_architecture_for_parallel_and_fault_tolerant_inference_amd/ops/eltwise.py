"""Wrappers for the memory-bound NHWC kernels (csrc/kernels/eltwise.hip).

Each wrapper validates dtype / contiguity / element counts on the host before
launching; all kernels require the channel count to be a multiple of 8
(16-byte vectors).
"""
from __future__ import annotations

from typing import Optional

import numpy as np

import torch

from ._lib import kernels, ptr, stream_handle


def _chk(t: torch.Tensor, dtype=torch.bfloat16, name="tensor"):
    if t.dtype != dtype:
        raise ValueError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")
    if not t.is_cuda:
        raise ValueError(f"{name}: must be a device tensor")


def input_pack(x: torch.Tensor, out: torch.Tensor, stream=None) -> torch.Tensor:
    """fp32 NHWC [B,H,W,C] -> bf16 NHWC [B,H,W,Cp] zero-padded channels."""
    _chk(x, torch.float32, "x")
    _chk(out, torch.bfloat16, "out")
    B, H, W, C = x.shape
    Cp = out.shape[-1]
    if out.shape[:3] != x.shape[:3] or Cp % 8 or Cp < C:
        raise ValueError(f"input_pack: bad shapes {tuple(x.shape)} -> {tuple(out.shape)}")
    kernels().input_pack(ptr(x), ptr(out), B * H * W, C, Cp, stream_handle(stream))
    return out


def bn_act(x: torch.Tensor, scale: torch.Tensor, shift: torch.Tensor, out: torch.Tensor, relu: bool = False,
           stream=None) -> torch.Tensor:
    _chk(x, name="x"); _chk(out, name="out")
    _chk(scale, torch.float32, "scale"); _chk(shift, torch.float32, "shift")
    C = x.shape[-1]
    if C % 8 or scale.numel() != C or shift.numel() != C or out.numel() != x.numel():
        raise ValueError("bn_act: bad shapes")
    kernels().bn_act(ptr(x), ptr(out), ptr(scale), ptr(shift), x.numel(), C, int(relu), stream_handle(stream))   # 2 = ReLU6
    return out


def add_act(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor, relu: bool = False, stream=None) -> torch.Tensor:
    _chk(a, name="a"); _chk(b, name="b"); _chk(out, name="out")
    if a.numel() != b.numel() or a.numel() != out.numel() or a.numel() % 8:
        raise ValueError("add_act: bad shapes")
    kernels().add_act(ptr(a), ptr(b), ptr(out), a.numel(), int(relu), stream_handle(stream))
    return out


def relu(x: torch.Tensor, out: torch.Tensor, mode: int = 1, stream=None) -> torch.Tensor:
    """mode 1: ReLU; mode 2: ReLU6 (Keras ``ReLU(max_value=6)``); any other ActMode works too."""
    _chk(x, name="x"); _chk(out, name="out")
    if x.numel() != out.numel() or x.numel() % 8 or not 0 <= mode <= 11:
        raise ValueError("relu: bad shapes or mode")
    kernels().relu(ptr(x), ptr(out), x.numel(), int(mode), stream_handle(stream))
    return out


def dwconv(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor, out: torch.Tensor, stride: int,
           pads=((0, 0), (0, 0)), act: int = 0, stream=None) -> torch.Tensor:
    """Depthwise conv (csrc/kernels/layers.hip): x [B,H,W,Cp] bf16, w fp32 [KH,KW,Cp] (BN folded),
    bias fp32 [Cp], out [B,OH,OW,Cp] bf16; `act` (ActMode: 0 none, 1 ReLU, 2 ReLU6, 3 swish, ...)."""
    _chk(x, name="x"); _chk(out, name="out")
    _chk(w, torch.float32, "w"); _chk(bias, torch.float32, "bias")
    B, H, W, Cp = x.shape
    KH, KW, Cw = w.shape
    Bo, OH, OW, Co = out.shape
    (pt, pb), (pl, pr) = pads
    if (Bo != B or Co != Cp or Cw != Cp or bias.numel() != Cp or Cp % 8
            or OH != (H + pt + pb - KH) // stride + 1 or OW != (W + pl + pr - KW) // stride + 1):
        raise ValueError(f"dwconv: bad shapes x{tuple(x.shape)} w{tuple(w.shape)} out{tuple(out.shape)}")
    kernels().dwconv(ptr(x), ptr(w), ptr(bias), ptr(out), B, H, W, Cp, OH, OW, KH, KW, stride, pt, pl, int(act),
                     stream_handle(stream))
    return out


def avgpool(x: torch.Tensor, out: torch.Tensor, k, s: int, pads=((0, 0), (0, 0)), stream=None) -> torch.Tensor:
    """Average pool (padding excluded from the count, Keras semantics)."""
    _chk(x, name="x"); _chk(out, name="out")
    kh, kw = (k, k) if isinstance(k, int) else k
    B, H, W, Cp = x.shape
    Bo, OH, OW, Co = out.shape
    (pt, pb), (pl, pr) = pads
    if (Bo != B or Co != Cp or Cp % 8 or OH != (H + pt + pb - kh) // s + 1 or OW != (W + pl + pr - kw) // s + 1):
        raise ValueError("avgpool: bad shapes")
    kernels().avgpool(ptr(x), ptr(out), B, H, W, Cp, OH, OW, kh, kw, s, pt, pl, stream_handle(stream))
    return out


def concat(xs, channels, out: torch.Tensor, out_channels: int, stream=None) -> torch.Tensor:
    """Channel concat of NHWC tensors whose channel dims are padded (xs[i] holds
    `channels[i]` real channels); the padding channels of `out` are zeroed."""
    _chk(out, name="out")
    Cpy = out.shape[-1]
    pixels = out.numel() // Cpy
    if sum(channels) != out_channels or out_channels > Cpy:
        raise ValueError("concat: channel counts do not add up")
    off = 0
    for i, (x, c) in enumerate(zip(xs, channels)):
        _chk(x, name=f"x{i}")
        if x.numel() // x.shape[-1] != pixels or c > x.shape[-1]:
            raise ValueError(f"concat: input {i} shape {tuple(x.shape)} does not match {tuple(out.shape)}")
        zero_from = out_channels if i == len(xs) - 1 else Cpy
        kernels().concat_into(ptr(x), c, x.shape[-1], ptr(out), Cpy, off, zero_from, pixels, stream_handle(stream))
        off += c
    return out


def maxpool(x: torch.Tensor, out: torch.Tensor, k: int, s: int, pad_t: int = 0, pad_l: int = 0,
            pad_zero: bool = True, stream=None) -> torch.Tensor:
    _chk(x, name="x"); _chk(out, name="out")
    B, H, W, C = x.shape
    Bo, OH, OW, Co = out.shape
    if Bo != B or Co != C or C % 8:
        raise ValueError("maxpool: bad shapes")
    # every output window must start inside the padded extent
    if (OH - 1) * s - pad_t + k > H + pad_t + 2 * k or (OW - 1) * s - pad_l + k > W + pad_l + 2 * k:
        raise ValueError("maxpool: output larger than padded input")
    kernels().maxpool(ptr(x), ptr(out), B, H, W, C, OH, OW, k, s, pad_t, pad_l, int(pad_zero), stream_handle(stream))
    return out


GAP_LARGE_HW = 1024      # from this many pixels per image the sliced two-pass GAP is used


def gap_scratch_elems(B: int, HW: int, C: int) -> int:
    """fp32 scratch the large-map GAP needs (0: the one-pass kernel serves this shape)."""
    return B * kernels().gap_large_slices(B, HW) * C if HW >= GAP_LARGE_HW else 0


def gap(x: torch.Tensor, out: Optional[torch.Tensor] = None, out32: Optional[torch.Tensor] = None,
        stream=None, scratch: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Global average pool [B,H,W,C] -> [B,C] (bf16 `out` and/or fp32 `out32`).  Maps of
    >= GAP_LARGE_HW pixels take the sliced two-pass kernel and its fp32 `scratch`."""
    _chk(x, name="x")
    B, H, W, C = x.shape
    if C % 8:
        raise ValueError("gap: C % 8 != 0")
    if out is not None:
        _chk(out, name="out")
        if out.numel() != B * C:
            raise ValueError("gap: bad out")
    if out32 is not None:
        _chk(out32, torch.float32, "out32")
        if out32.numel() != B * C:
            raise ValueError("gap: bad out32")
    need = gap_scratch_elems(B, H * W, C)
    if need:
        if scratch is None:               # the executor passes a preallocated one
            scratch = torch.empty(need, dtype=torch.float32, device=x.device)
        if scratch.numel() < need or scratch.dtype != torch.float32:
            raise ValueError(f"gap over {H}x{W}: needs an fp32 scratch of {need} elements")
        kernels().gap_large(ptr(x), ptr(out), ptr(out32), ptr(scratch), B, H * W, C, stream_handle(stream))
    else:
        kernels().gap(ptr(x), ptr(out), ptr(out32), B, H * W, C, stream_handle(stream))
    return out if out is not None else out32


def dense_small_scratch(M: int, N: int, K: int) -> int:
    """fp32 elements of the split-K scratch `dense_small` needs."""
    return kernels().dense_small_kslices(K) * M * N


def dense_small(x: torch.Tensor, pc, part: torch.Tensor, logits: Optional[torch.Tensor] = None,
                probs: Optional[torch.Tensor] = None, stream=None) -> None:
    """Classifier GEMM for M <= 32 rows (csrc/kernels/head.hip): x [M][K] bf16,
    packed weights `pc` (ops.conv.PackedConv, 1x1), fp32 logits and/or softmax probs."""
    _chk(x, name="x")
    M, K = x.shape[0], x.numel() // x.shape[0]
    N = pc.cout
    if M > 32 or K != pc.K:
        raise ValueError(f"dense_small: M={M} (<= 32) and K={K} (== {pc.K}) required")
    if part.dtype != torch.float32 or part.numel() < dense_small_scratch(M, N, K):
        raise ValueError("dense_small: scratch too small")
    for t in (logits, probs):
        if t is not None and (t.dtype != torch.float32 or t.numel() != M * N or not t.is_contiguous()):
            raise ValueError("dense_small: outputs must be contiguous fp32 [M][N]")
    kernels().dense_small(ptr(x), ptr(pc.w), ptr(pc.bias), ptr(part), ptr(logits), ptr(probs), M, N, K, pc.Kpad,
                          stream_handle(stream))


def dense_small_f32_scratch(M: int, N: int, Kpad: int) -> int:
    """fp32 elements of the split-K scratch `dense_small_f32` needs."""
    return kernels().dense_small_f32_kslices(Kpad) * M * N


def dense_small_f32(x: torch.Tensor, pc, part: torch.Tensor, logits: Optional[torch.Tensor] = None,
                    probs: Optional[torch.Tensor] = None, stream=None) -> None:
    """fp32 classifier GEMM for M <= 32 rows (csrc/kernels/head.hip dense_partial_f32_kernel + finish):
    x [M][K] fp32, weights packed by ops.conv.pack_conv_f32, fp32 logits and/or softmax probs."""
    _chk(x, torch.float32, "x")
    M, K = x.shape[0], x.numel() // x.shape[0]
    N = pc.cout
    if M > 32 or K != pc.K or pc.w.dtype != torch.float32:
        raise ValueError(f"dense_small_f32: M={M} (<= 32), K={K} (== {pc.K}) and fp32 weights required")
    if part.dtype != torch.float32 or part.numel() < dense_small_f32_scratch(M, N, pc.Kpad):
        raise ValueError("dense_small_f32: scratch too small")
    for t in (logits, probs):
        if t is not None and (t.dtype != torch.float32 or t.numel() != M * N or not t.is_contiguous()):
            raise ValueError("dense_small_f32: outputs must be contiguous fp32 [M][N]")
    kernels().dense_small_f32(ptr(x), ptr(pc.w), ptr(pc.bias), ptr(part), ptr(logits), ptr(probs), M, N, K,
                              pc.Kpad, stream_handle(stream))


def softmax_rows(x: torch.Tensor, out: torch.Tensor, stream=None) -> torch.Tensor:
    _chk(x, torch.float32, "x"); _chk(out, torch.float32, "out")
    rows, n = x.shape
    if out.shape != x.shape:
        raise ValueError("softmax: bad out")
    kernels().softmax_rows(ptr(x), ptr(out), rows, n, n, stream_handle(stream))
    return out


def cast_bf16_f32(x: torch.Tensor, out: torch.Tensor, stream=None) -> torch.Tensor:
    _chk(x, name="x"); _chk(out, torch.float32, "out")
    if x.numel() != out.numel():
        raise ValueError("cast: size mismatch")
    kernels().cast_bf16_f32(ptr(x), ptr(out), x.numel(), stream_handle(stream))
    return out


def cast_f32_bf16(x: torch.Tensor, out: torch.Tensor, stream=None) -> torch.Tensor:
    _chk(x, torch.float32, "x"); _chk(out, name="out")
    if x.numel() != out.numel():
        raise ValueError("cast: size mismatch")
    kernels().cast_f32_bf16(ptr(x), ptr(out), x.numel(), stream_handle(stream))
    return out


def pad(x: torch.Tensor, out: torch.Tensor, pad_t: int, pad_l: int, stream=None) -> torch.Tensor:
    """Materialised zero padding (NHWC)."""
    _chk(x, name="x"); _chk(out, name="out")
    B, H, W, C = x.shape
    Bo, OH, OW, Co = out.shape
    if Bo != B or Co != C or C % 8 or OH < H + pad_t or OW < W + pad_l:
        raise ValueError("pad: bad shapes")
    kernels().pad(ptr(x), ptr(out), B, H, W, C, OH, OW, pad_t, pad_l, stream_handle(stream))
    return out


from ..graph.ir import ACT_MODE as ACT_MODES  # noqa: E402  (Keras name -> csrc/kernels/common.h ActMode)

BIN_OPS = {"add": 0, "sub": 1, "mul": 2, "max": 3, "min": 4, "avg": 5}


def act(x: torch.Tensor, out: torch.Tensor, mode: int, alpha: float = 0.3, stream=None) -> torch.Tensor:
    """Standalone activation (ActMode `mode`; `alpha` = LeakyReLU slope)."""
    _chk(x, name="x"); _chk(out, name="out")
    if x.numel() != out.numel() or x.numel() % 8 or not 0 <= mode <= 12:
        raise ValueError("act: bad shapes or mode")
    kernels().act(ptr(x), ptr(out), x.numel(), int(mode), float(alpha), stream_handle(stream))
    return out


def binary(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor, op: str, act_mode: int = 0,
           stream=None) -> torch.Tensor:
    """out = act(a <op> b); b has a's shape, or one channel row per image ([B,1,1,Cp] / [B,Cp]) broadcast over
    a's pixels."""
    _chk(a, name="a"); _chk(b, name="b"); _chk(out, name="out")
    Cp = a.shape[-1]
    if out.numel() != a.numel() or Cp % 8 or b.shape[-1] != Cp:
        raise ValueError("binary: bad shapes")
    bcast = 0
    if b.numel() != a.numel():
        B = a.shape[0]
        if b.numel() != B * Cp:
            raise ValueError(f"binary: cannot broadcast {tuple(b.shape)} over {tuple(a.shape)}")
        bcast = a.numel() // (B * Cp)
    kernels().binary(ptr(a), ptr(b), ptr(out), a.numel(), Cp, bcast, BIN_OPS[op], int(act_mode),
                     stream_handle(stream))
    return out


def gmp(x: torch.Tensor, out: torch.Tensor, stream=None) -> torch.Tensor:
    """GlobalMaxPooling2D: [B,H,W,Cp] -> [B,Cp]."""
    _chk(x, name="x"); _chk(out, name="out")
    B, H, W, Cp = x.shape
    if out.numel() != B * Cp or Cp % 8:
        raise ValueError("gmp: bad shapes")
    kernels().gmp(ptr(x), ptr(out), B, H * W, Cp, stream_handle(stream))
    return out


# ------------------------------------------------------------------ fp32 path
def maxpool_f32(x: torch.Tensor, out: torch.Tensor, k: int, s: int, pad_t: int = 0, pad_l: int = 0,
                pad_zero: bool = True, stream=None) -> torch.Tensor:
    _chk(x, torch.float32, "x"); _chk(out, torch.float32, "out")
    B, H, W, C = x.shape
    _, OH, OW, C2 = out.shape
    k = k[0] if isinstance(k, (tuple, list)) else k
    s = s[0] if isinstance(s, (tuple, list)) else s
    if C2 != C or C % 4:
        raise ValueError("fp32 maxpool needs matching channels, a multiple of 4")
    kernels().maxpool_f32(ptr(x), ptr(out), B, H, W, C, OH, OW, int(k), int(s), int(pad_t), int(pad_l),
                          int(bool(pad_zero)), stream_handle(stream))
    return out


def gap_f32(x: torch.Tensor, out: torch.Tensor, stream=None, scratch: Optional[torch.Tensor] = None) -> torch.Tensor:
    """fp32 GAP; maps of >= GAP_LARGE_HW pixels take the sliced two-pass kernel and its fp32 `scratch`
    (gap_scratch_elems)."""
    _chk(x, torch.float32, "x"); _chk(out, torch.float32, "out")
    B, H, W, C = x.shape
    if out.numel() != B * C or C % 4:
        raise ValueError("fp32 GAP: out must be [B][C], C a multiple of 4")
    need = gap_scratch_elems(B, H * W, C)
    if need:
        if scratch is None:
            scratch = torch.empty(need, dtype=torch.float32, device=x.device)
        if scratch.numel() < need or scratch.dtype != torch.float32:
            raise ValueError(f"fp32 gap over {H}x{W}: needs an fp32 scratch of {need} elements")
        kernels().gap_large_f32(ptr(x), ptr(out), ptr(scratch), B, H * W, C, stream_handle(stream))
    else:
        kernels().gap_f32(ptr(x), ptr(out), B, H * W, C, stream_handle(stream))
    return out


def eltwise_f32(a: torch.Tensor, out: torch.Tensor, b: Optional[torch.Tensor] = None,
                scale: Optional[torch.Tensor] = None, shift: Optional[torch.Tensor] = None, relu: int = 0,
                stream=None) -> torch.Tensor:
    """out = act(a + b) | act(a * scale[c] + shift[c]) | act(a), all fp32."""
    _chk(a, torch.float32, "a"); _chk(out, torch.float32, "out")
    if out.numel() != a.numel():
        raise ValueError("eltwise: element counts differ")
    C = a.shape[-1]
    op = 2
    if b is not None:
        _chk(b, torch.float32, "b")
        if b.numel() != a.numel():
            raise ValueError("eltwise add: element counts differ")
        op = 0
    elif scale is not None:
        if scale.numel() != C or shift is None or shift.numel() != C:
            raise ValueError("eltwise bn: scale/shift need one value per channel")
        op = 1
    kernels().eltwise_f32(ptr(a), ptr(b), ptr(scale), ptr(shift), ptr(out), a.numel(), C, op, int(relu),
                          stream_handle(stream))
    return out


def dwconv_f32(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor, out: torch.Tensor, stride: int,
               pads=((0, 0), (0, 0)), act: int = 0, alpha: float = 0.3, stream=None) -> torch.Tensor:
    """fp32 depthwise conv: x [B,H,W,C], w [KH,KW,C] (BN folded), bias [C], out [B,OH,OW,C]; any ActMode."""
    _chk(x, torch.float32, "x"); _chk(out, torch.float32, "out")
    _chk(w, torch.float32, "w"); _chk(bias, torch.float32, "bias")
    B, H, W, C = x.shape
    KH, KW, Cw = w.shape
    _, OH, OW, C2 = out.shape
    (pt, _), (pl, _) = pads
    if Cw != C or C2 != C or bias.numel() != C:
        raise ValueError("dwconv_f32: channel counts differ")
    kernels().dwconv_f32(ptr(x), ptr(w), ptr(bias), ptr(out), B, H, W, C, OH, OW, KH, KW, int(stride), int(pt),
                         int(pl), int(act), float(alpha), stream_handle(stream))
    return out


def avgpool_f32(x: torch.Tensor, out: torch.Tensor, k, s: int, pads=((0, 0), (0, 0)), stream=None) -> torch.Tensor:
    _chk(x, torch.float32, "x"); _chk(out, torch.float32, "out")
    kh, kw = (k, k) if isinstance(k, int) else k
    B, H, W, C = x.shape
    _, OH, OW, C2 = out.shape
    (pt, _), (pl, _) = pads
    if C2 != C:
        raise ValueError("avgpool_f32: channel counts differ")
    kernels().avgpool_f32(ptr(x), ptr(out), B, H, W, C, OH, OW, kh, kw, int(s), int(pt), int(pl),
                          stream_handle(stream))
    return out


def concat_f32(xs, out: torch.Tensor, stream=None) -> torch.Tensor:
    """Channel concat of fp32 NHWC tensors (true channel counts)."""
    _chk(out, torch.float32, "out")
    Cy = out.shape[-1]
    pixels = out.numel() // Cy
    if sum(x.shape[-1] for x in xs) != Cy:
        raise ValueError("concat_f32: channel counts do not add up")
    off = 0
    for i, x in enumerate(xs):
        _chk(x, torch.float32, f"x{i}")
        if x.numel() // x.shape[-1] != pixels:
            raise ValueError(f"concat_f32: input {i} shape {tuple(x.shape)} does not match {tuple(out.shape)}")
        kernels().concat_f32(ptr(x), x.shape[-1], ptr(out), Cy, off, pixels, stream_handle(stream))
        off += x.shape[-1]
    return out


def binary_f32(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor, op: str, act_mode: int = 0,
               stream=None) -> torch.Tensor:
    """fp32 out = act(a <op> b); b has a's shape or one channel row per image (squeeze-excite broadcast)."""
    _chk(a, torch.float32, "a"); _chk(b, torch.float32, "b"); _chk(out, torch.float32, "out")
    C = a.shape[-1]
    if out.numel() != a.numel() or b.shape[-1] != C:
        raise ValueError("binary_f32: bad shapes")
    bcast = 0
    if b.numel() != a.numel():
        B = a.shape[0]
        if b.numel() != B * C:
            raise ValueError(f"binary_f32: cannot broadcast {tuple(b.shape)} over {tuple(a.shape)}")
        bcast = a.numel() // (B * C)
    kernels().binary_f32(ptr(a), ptr(b), ptr(out), a.numel(), C, bcast, BIN_OPS[op], int(act_mode),
                         stream_handle(stream))
    return out


def affine_act_f32(x: torch.Tensor, out: torch.Tensor, scale: Optional[torch.Tensor] = None,
                   shift: Optional[torch.Tensor] = None, act: int = 0, alpha: float = 0.3,
                   stream=None) -> torch.Tensor:
    """fp32 out = act(x * scale[c] + shift[c]) (or act(x)), any channel count and ActMode."""
    _chk(x, torch.float32, "x"); _chk(out, torch.float32, "out")
    if out.numel() != x.numel():
        raise ValueError("affine_act_f32: element counts differ")
    C = x.shape[-1]
    if scale is not None and (scale.numel() != C or shift is None or shift.numel() != C):
        raise ValueError("affine_act_f32: scale/shift need one value per channel")
    kernels().affine_act_f32(ptr(x), ptr(scale), ptr(shift), ptr(out), x.numel(), C, int(act), float(alpha),
                             stream_handle(stream))
    return out


def pad_f32(x: torch.Tensor, out: torch.Tensor, pad_t: int, pad_l: int, stream=None) -> torch.Tensor:
    _chk(x, torch.float32, "x"); _chk(out, torch.float32, "out")
    B, H, W, C = x.shape
    _, OH, OW, C2 = out.shape
    if C2 != C or OH < H + pad_t or OW < W + pad_l:
        raise ValueError("pad: output too small")
    kernels().pad_f32(ptr(x), ptr(out), B, H, W, C, OH, OW, int(pad_t), int(pad_l), stream_handle(stream))
    return out


# ------------------------------------------------------------------ ingest
# Keras `preprocess_input` modes (keras.applications.imagenet_utils): caffe =
# RGB -> BGR then minus the ImageNet BGR mean (ResNet / VGG; the reference's
# `test/test.py:20-23`), tf = x / 127.5 - 1 (MobileNet, Inception), torch =
# (x / 255 - mean) / std (DenseNet), none = plain cast.
PREPROCESS = {
    "none": (False, (1.0, 1.0, 1.0), (0.0, 0.0, 0.0)),
    "caffe": (True, (1.0, 1.0, 1.0), (-103.939, -116.779, -123.68)),
    "tf": (False, (1 / 127.5,) * 3, (-1.0, -1.0, -1.0)),
    "torch": (False, tuple(1 / (255.0 * s) for s in (0.229, 0.224, 0.225)),
              tuple(-m / s for m, s in zip((0.485, 0.456, 0.406), (0.229, 0.224, 0.225)))),
}


def ingest_u8(x: torch.Tensor, out: torch.Tensor, mode: str = "none", stream=None) -> torch.Tensor:
    """uint8 NHWC images (device) -> fp32 model input with `mode` preprocessing."""
    if x.dtype != torch.uint8 or not x.is_contiguous():
        raise ValueError("ingest: x must be contiguous uint8")
    _chk(out, torch.float32, "out")
    if out.numel() < x.numel() or out.shape[-1] != x.shape[-1]:
        raise ValueError(f"ingest: out {tuple(out.shape)} cannot hold x {tuple(x.shape)}")
    C = x.shape[-1]
    rev, sc, sh = PREPROCESS[mode]
    if C != 3 and mode != "none":
        raise ValueError(f"preprocess mode {mode!r} needs 3 channels, got {C}")
    scale = [sc[c] if c < 3 else 1.0 for c in range(C)]
    shift = [sh[c] if c < 3 else 0.0 for c in range(C)]
    kernels().ingest_u8(ptr(x), ptr(out), x.numel(), C, int(rev), scale, shift, stream_handle(stream))
    return out


def preprocess_ref(x: np.ndarray, mode: str) -> np.ndarray:
    """Host reference of `ingest_u8` (float64 math, fp32 result)."""
    rev, sc, sh = PREPROCESS[mode]
    y = x.astype(np.float64)
    if rev:
        y = y[..., ::-1]
    C = y.shape[-1]
    return (y * np.asarray(sc[:C]) + np.asarray(sh[:C])).astype(np.float32)
