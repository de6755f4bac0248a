"""Fused implicit-GEMM convolution (csrc/kernels/conv_igemm.hip).

Replaces what the reference gets from TF/cuDNN inside `model.predict`
(`src/node.py:177`): Conv2D + BatchNormalization [+ Add] [+ ReLU] of the
Keras ResNet graph run as ONE MFMA launch with BN folded into the weights.

Host side here: BN folding, weight packing to ``[Npad][Kpad]`` bf16 with
``k = (kh, kw, ci)``, tile-config choice, and the shape checks that keep a
launch inside its buffers (done before every launch).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from ._lib import kernels, ptr, stream_handle

BK = 64
# tile configs (must match ADAPT_CONV_CFGS in conv_igemm.hip)
CFG_TILES = {0: (128, 128), 1: (128, 64), 2: (64, 128), 3: (64, 64), 4: (256, 64), 5: (32, 64),
             # v2: LDS-DMA multi-stage ring (conv_glds.hip)
             6: (128, 128), 7: (128, 128), 8: (128, 64), 9: (64, 128), 10: (64, 64), 11: (256, 64), 12: (64, 256),
             13: (128, 128), 14: (128, 128), 15: (64, 128), 16: (64, 64), 17: (128, 64), 18: (64, 128),
             19: (256, 64), 20: (128, 128), 21: (64, 64), 22: (128, 128), 23: (64, 128), 24: (64, 64),
             25: (128, 64), 26: (256, 64), 27: (64, 256), 28: (128, 256), 29: (256, 128),
             # v2, sized for 2+ blocks per CU
             30: (128, 128), 31: (64, 128), 32: (128, 64), 33: (128, 128), 34: (64, 64),
             # v2, deep rings (5-8 stages)
             35: (64, 128), 36: (128, 64), 37: (64, 64), 38: (64, 128), 39: (64, 64),
             # v3: 3x3 halo-patch kernel (conv_halo.hip); BM = pixels of TH whole output rows
             40: (224, 64), 41: (112, 128), 42: (224, 64), 43: (64, 128), 44: (112, 64), 45: (224, 64),
             46: (224, 64), 47: (112, 128), 48: (224, 64), 49: (64, 128), 50: (224, 64), 51: (224, 64),
             52: (112, 64),
             # v2, 16 waves per block (conv_glds.hip ids 53-58)
             53: (128, 128), 54: (128, 128), 55: (256, 128), 56: (128, 256), 57: (256, 128), 58: (128, 128),
             # v2, two K-groups of waves per block (conv_glds.hip ADAPT_GLDS_KG_CFGS)
             62: (64, 128), 63: (128, 128), 64: (64, 256), 65: (128, 128), 66: (64, 128), 67: (128, 64),
             68: (64, 64), 69: (128, 256), 70: (256, 128)}
V1_CFGS = (0, 1, 2, 3, 4, 5)
# halo configs: patch capacity in pixels (must match ADAPT_HALO_CFGS)
HALO_PATCH = {40: 352, 41: 192, 42: 288, 43: 96, 44: 144, 45: 384, 46: 352, 47: 192, 48: 384, 49: 96, 50: 320,
              51: 288, 52: 144}


def halo_rows(cfg: int, pc: "PackedConv", H: int, W: int) -> int:
    """Output rows per tile for a halo config, 0 if the conv/shape does not fit it."""
    if (pc.kh, pc.kw, pc.stride, pc.pad_t, pc.pad_l, pc.pad_b, pc.pad_r) != (3, 3, 1, 1, 1, 1, 1) or pc.cin % 64:
        return 0
    bm = CFG_TILES[cfg][0]
    th = min(H, bm // W if W else 0)
    while th >= 1 and (th + 2) * (W + 2) > HALO_PATCH[cfg]:
        th -= 1
    return max(th, 0)
_CFG_EFF = {0: 1.0, 4: 0.97, 1: 0.86, 2: 0.86, 3: 0.66, 5: 0.42}


def cfg_supported(cfg: int, pc: "PackedConv", pure: bool) -> bool:
    """v2 configs walk K tap-major in 64-channel slices: they need Cin % 64 == 0;
    v3 (halo) configs take 3x3/s1/p1 convs only (the row count is checked at launch);
    pointwise configs (PW_CFGS) take 1x1 stride-1 convs of the shapes pw_wide.hip has."""
    if cfg in PW_CFGS:
        return pure and pw_supported(pc)
    if cfg in PS_CFGS:
        return pure and ps_supported(pc, cfg)
    if cfg in RR3_CFGS:
        return rr3_supported(pc)
    if cfg in CS3_CFGS:
        return cs3_supported(pc)
    if cfg in V1_CFGS:
        return True
    if cfg in HALO_PATCH:
        return (pc.kh, pc.kw, pc.stride, pc.pad_t, pc.pad_l) == (3, 3, 1, 1, 1) and pc.cin % 64 == 0
    return pc.cin % 64 == 0
NUM_CUS = 256


def fold_bn(kernel_hwio: np.ndarray, bias: Optional[np.ndarray], bn: Optional[dict], eps: float = 1.001e-5):
    """Fold inference BN into conv weights: returns (kernel_hwio, bias) fp32."""
    k = kernel_hwio.astype(np.float64)
    cout = k.shape[-1]
    b = np.zeros(cout) if bias is None else bias.astype(np.float64)
    if bn is not None:
        s = bn["gamma"].astype(np.float64) / np.sqrt(bn["moving_variance"].astype(np.float64) + eps)
        k = k * s
        b = (b - bn["moving_mean"]) * s + bn["beta"]
    return k.astype(np.float32), b.astype(np.float32)


@dataclass
class PackedConv:
    """Device-resident packed weights for one (possibly BN-folded) conv."""
    w: torch.Tensor          # [Npad][Kpad] bf16
    bias: torch.Tensor       # [N] fp32
    kh: int
    kw: int
    cin: int                 # (padded) input channels the kernel consumes
    cout: int
    stride: int
    pad_t: int
    pad_l: int
    pad_b: int
    pad_r: int
    n_split: int = 0         # > 0: two sibling convs packed along N (outputs [0, n_split) and [n_split, cout))
    wino: Optional[torch.Tensor] = None   # fp32 3x3/s1/p1: Winograd-transformed weights (pack_wino_f32)
    pwf: Optional[torch.Tensor] = None    # fp32 1x1/s1: fragment-packed weights of pw_f32.hip (pack_pw_f32)
    wino4s: Optional[torch.Tensor] = None  # fp32 3x3/s1/p1: Winograd F(4x4, 3x3) weights (wino4s_pack_np)

    @property
    def K(self) -> int:
        return self.kh * self.kw * self.cin

    @property
    def Kpad(self) -> int:
        return self.w.shape[1]

    def out_hw(self, h: int, w: int):
        oh = (h + self.pad_t + self.pad_b - self.kh) // self.stride + 1
        ow = (w + self.pad_l + self.pad_r - self.kw) // self.stride + 1
        return oh, ow


def pack_conv(kernel_hwio: np.ndarray, bias: np.ndarray, stride: int, pads, device, cin_pad: Optional[int] = None,
              row_align: int = 256) -> PackedConv:
    kh, kw, cin, cout = kernel_hwio.shape
    cp = cin_pad or cin
    if cp % 8:
        raise ValueError(f"conv input channels must be a multiple of 8 (got {cp}); pad the input")
    k = np.zeros((kh, kw, cp, cout), np.float32)
    k[:, :, :cin, :] = kernel_hwio
    K = kh * kw * cp
    Kpad = int(math.ceil(K / BK) * BK)
    Npad = int(math.ceil(cout / row_align) * row_align)
    wt = np.zeros((Npad, Kpad), np.float32)
    wt[:cout, :K] = k.transpose(3, 0, 1, 2).reshape(cout, K)       # [cout][kh][kw][ci]
    (pt, pb), (pl, pr) = pads
    return PackedConv(
        w=torch.from_numpy(wt).to(device=device, dtype=torch.bfloat16).contiguous(),
        bias=torch.from_numpy(np.ascontiguousarray(bias, np.float32)).to(device),
        kh=kh, kw=kw, cin=cp, cout=cout, stride=stride, pad_t=pt, pad_l=pl, pad_b=pb, pad_r=pr)


def choose_cfg(M: int, N: int, Kpad: int, occupancy: int = 2):
    """Heuristic (cfg, ksplit): minimise waves-of-blocks x per-block work / efficiency."""
    best = None
    ktiles = Kpad // BK
    for cfg in V1_CFGS:
        bm, bn = CFG_TILES[cfg]
        if N % 8:
            continue
        tiles = math.ceil(M / bm) * math.ceil(N / bn)
        for ks in (1, 2, 4, 8):
            if ks > 1 and (ktiles // ks < 4):
                continue
            blocks = tiles * ks
            waves = math.ceil(blocks / (NUM_CUS * occupancy))
            work = bm * bn * (Kpad / ks)
            t = waves * work / _CFG_EFF[cfg]
            if ks > 1:
                t += M * N * 4 * (ks + 1) / 2e3   # slab write + reduce traffic (arbitrary units)
                t *= 1.05
            # small-grid penalty: fewer blocks than CUs leaves the chip idle
            if blocks < NUM_CUS:
                t *= 1.0 + 0.15 * (NUM_CUS - blocks) / NUM_CUS
            cand = (t, cfg, ks)
            if best is None or cand < best:
                best = cand
    return best[1], best[2]


def sk_plan(M: int, N: int, Kpad: int, cfg: int, mult: int = 1):
    """Stream-K launch shape: (tiles, grid, iters per block, fp32 workspace elements)."""
    bm, bn = CFG_TILES[cfg]
    tiles = math.ceil(M / bm) * math.ceil(N / bn)
    g, it = kernels().conv_sk_plan(tiles, Kpad // BK, mult)
    return tiles, g, it, g * 2 * bm * bn


def workspace_elems(M: int, N: int, Kpad: int, cfg: int, ksplit: int) -> int:
    """fp32 workspace a launch needs: split-K slabs or stream-K partial slots (none for the sliced pointwise
    configs, whose `ksplit` is a grid size)."""
    if cfg in PS_CFGS:
        return 0
    if ksplit > 1:
        return ksplit * M * N
    if ksplit < 0:
        return sk_plan(M, N, Kpad, cfg, -ksplit)[3]
    return 0


def conv_forward(x: torch.Tensor, pc: PackedConv, out: torch.Tensor, residual: Optional[torch.Tensor] = None,
                 relu: bool = False, cfg: Optional[int] = None, ksplit: int = 1,
                 workspace: Optional[torch.Tensor] = None, stream=None,
                 counters: Optional[torch.Tensor] = None, out2: Optional[torch.Tensor] = None,
                 relu2: bool = False) -> torch.Tensor:
    """x: [B,H,W,Cin] bf16 NHWC; out: [B,OH,OW,Cout] bf16 (or fp32 [M][Cout] for GEMM use).

    ksplit > 1: split-K (fp32 slabs + reduce launch); ksplit < 0: stream-K over
    -ksplit x 256 blocks (v2 configs; needs `counters`, int32 zeros, one per tile).
    Dual output (``pc.n_split > 0``, two sibling convs packed along N): channels
    [0, n_split) go to `out` (ReLU `relu`), the rest to `out2` (ReLU `relu2`)."""
    if x.dim() == 2:
        B, H, W, C = x.shape[0], 1, 1, x.shape[1]
    else:
        B, H, W, C = x.shape
    if C != pc.cin:
        raise ValueError(f"conv expects {pc.cin} input channels, got {C}")
    if int(relu) not in (0, 1, 2) or int(relu2) not in (0, 1, 2):
        raise ValueError("conv epilogue activation must be 0 (none), 1 (ReLU) or 2 (ReLU6)")
    if x.dtype != torch.bfloat16 or not x.is_contiguous():
        raise ValueError("conv input must be contiguous bf16 NHWC")
    OH, OW = pc.out_hw(H, W)
    M = B * OH * OW
    N = pc.cout
    out_f32 = out.dtype == torch.float32
    ns = pc.n_split
    if ns:
        if out2 is None or residual is not None or out_f32:
            raise ValueError("dual-output conv needs a bf16 out2 and no residual")
        if out.numel() != M * ns or out2.numel() != M * (N - ns) or not out.is_contiguous() \
                or not out2.is_contiguous() or out2.dtype != torch.bfloat16:
            raise ValueError(f"dual-output conv buffers need {M * ns} + {M * (N - ns)} bf16 elements")
    elif out2 is not None:
        raise ValueError("out2 given for a single-output conv")
    elif out.numel() != M * N or not out.is_contiguous():
        raise ValueError(f"conv output buffer has {out.numel()} elements, need {M * N}")
    if residual is not None and (residual.numel() != M * N or residual.dtype != torch.bfloat16):
        raise ValueError("residual must be bf16 with the output's shape")
    if cfg is None:
        cfg, ksplit = choose_cfg(M, N, pc.Kpad)
    if cfg in RR3_CFGS:                    # register-resident-filter 3x3 (conv3x3_rr.hip)
        if ksplit != 1 or ns or out_f32 or residual is not None or (H, W) != (28, 28) or OH != H or OW != W:
            raise ValueError(f"3x3 config {cfg}: 28x28 stride-1 bf16 output, no residual / split-K")
        rr3_forward(x, pc, out.view(x.shape[0], OH, OW, N), relu=int(relu), kg=RR3_CFGS[cfg], stream=stream)
        return out
    if cfg in CS3_CFGS:                    # channel-split register-resident 3x3 (conv3x3_cs.hip)
        if ksplit != 1 or ns or out_f32 or residual is not None or OH != H or OW != W:
            raise ValueError(f"3x3 config {cfg}: stride-1 bf16 output, no residual / split-K")
        cs3_forward(x, pc, out.view(x.shape[0], OH, OW, N), relu=int(relu), stream=stream)
        return out
    if cfg in PS_CFGS:                     # channel-sliced persistent pointwise kernel (pw_slice.hip)
        # no split-K: `ksplit` 1 / 2 is the grid, one or two blocks per CU (PS_GRIDS)
        if ksplit not in PS_GRIDS or ns or out_f32 or OH != H or OW != W:
            raise ValueError(f"pointwise config {cfg}: single bf16 output, ksplit 1 / 2 = blocks per CU")
        return ps_forward(x.reshape(M, C), pc, out.view(M, N), None if residual is None else residual.view(M, N),
                          relu=int(relu), cfg=cfg, blocks=NUM_CUS * ksplit, stream=stream)
    if cfg in PW_CFGS:                     # persistent pointwise kernel (pw_wide.hip)
        if ksplit != 1 or ns or out_f32 or OH != H or OW != W:
            raise ValueError(f"pointwise config {cfg}: single bf16 output, no split-K")
        return pw_forward(x.reshape(M, C), pc, out.view(M, N), None if residual is None else residual.view(M, N),
                          relu=int(relu), cfg=cfg, blocks=NUM_CUS, stream=stream)
    bm, bn = CFG_TILES[cfg]
    if pc.w.shape[0] < math.ceil(N / bn) * bn:
        raise ValueError("packed weights not padded to the tile's N")
    if ns and ns % 8:
        raise ValueError("dual-output split must be a multiple of 8 channels")
    pure = pc.kh == 1 and pc.kw == 1 and pc.stride == 1 and pc.pad_t == 0 and pc.pad_l == 0 and OH == H and OW == W
    if not cfg_supported(cfg, pc, pure):
        raise ValueError(f"tile config {cfg} does not support this conv (Cin {pc.cin}, {pc.kh}x{pc.kw}/s{pc.stride})")
    if ksplit == 0 or (ksplit < 0 and cfg in V1_CFGS) or (ksplit != 1 and cfg in HALO_PATCH):
        raise ValueError(f"ksplit {ksplit} not supported by tile config {cfg}")
    th = 0
    if cfg in HALO_PATCH:
        th = halo_rows(cfg, pc, H, W)
        if th < 1:
            raise ValueError(f"halo config {cfg} cannot tile a {H}x{W} 3x3 conv")
    ws_ptr = ctr_ptr = 0
    sk_iters = 0
    need = workspace_elems(M, N, pc.Kpad, cfg, ksplit)
    if need:
        if workspace is None:
            workspace = torch.empty(need, dtype=torch.float32, device=x.device)
        if workspace.numel() < need or workspace.dtype != torch.float32:
            raise ValueError(f"ksplit {ksplit} needs an fp32 workspace of {need} elements")
        ws_ptr = ptr(workspace)
    if ksplit < 0:
        tiles, _, sk_iters, _ = sk_plan(M, N, pc.Kpad, cfg, -ksplit)
        if counters is None:
            counters = torch.zeros(tiles, dtype=torch.int32, device=x.device)
        if counters.numel() < tiles or counters.dtype != torch.int32:
            raise ValueError(f"stream-K needs {tiles} int32 tile counters")
        ctr_ptr = ptr(counters)
    kernels().conv_forward(ptr(x), ptr(pc.w), ptr(pc.bias), ptr(residual), ptr(out), ws_ptr, ctr_ptr, sk_iters, th,
                           B, H, W, C, OH, OW, N, pc.kh, pc.kw, pc.stride, pc.pad_t, pc.pad_l,
                           pc.K, pc.Kpad, ns or N, int(relu), int(ksplit), int(cfg), bool(out_f32),
                           stream_handle(stream), ptr(out2), int(ns), int(relu2))
    return out


# ------------------------------------------------------------------ stem
STEM_K = 224          # 7 filter rows x (8 kw x 4 channels), csrc/kernels/stem.hip ST_K


@dataclass
class PackedStem:
    """conv1 (7x7/s2, 64 filters, BN folded) packed as [64][kh*32 + kw*4 + c] bf16."""
    w: torch.Tensor
    bias: torch.Tensor
    cin: int
    pad_t: int
    pad_l: int
    pad_b: int
    pad_r: int

    def out_hw(self, h: int, w: int):
        return (h + self.pad_t + self.pad_b - 7) // 2 + 1, (w + self.pad_l + self.pad_r - 7) // 2 + 1


def pack_stem(kernel_hwio: np.ndarray, bias: np.ndarray, pads, device) -> PackedStem:
    kh, kw, cin, cout = kernel_hwio.shape
    if (kh, kw, cout) != (7, 7, 64) or cin > 4:
        raise ValueError(f"stem kernel must be 7x7x(<=4)x64, got {kernel_hwio.shape}")
    wt = np.zeros((64, 7, 8, 4), np.float32)                 # [cout][kh][kw(8)][c(4)]
    wt[:, :, :7, :cin] = kernel_hwio.transpose(3, 0, 1, 2)
    (pt, pb), (pl, pr) = pads
    return PackedStem(w=torch.from_numpy(wt.reshape(64, STEM_K)).to(device=device, dtype=torch.bfloat16).contiguous(),
                      bias=torch.from_numpy(np.ascontiguousarray(bias, np.float32)).to(device),
                      cin=cin, pad_t=pt, pad_l=pl, pad_b=pb, pad_r=pr)


def stem_forward(x: torch.Tensor, ps: PackedStem, out: torch.Tensor, pool: bool = True, pool_pad: int = 1,
                 stream=None) -> torch.Tensor:
    """x: [B,H,W,C<=4] fp32 NHWC -> relu(conv7x7/s2(x)) [-> maxpool 3x3/s2 pad pool_pad], bf16 NHWC 64 ch."""
    if x.dtype != torch.float32 or not x.is_contiguous() or x.dim() != 4:
        raise ValueError("stem input must be contiguous fp32 NHWC")
    B, H, W, C = x.shape
    if C != ps.cin:
        raise ValueError(f"stem expects {ps.cin} channels, got {C}")
    OH, OW = ps.out_hw(H, W)
    if OW > 112:
        raise ValueError(f"stem kernel handles conv rows up to 112 pixels (got {OW})")
    PH = PW = 0
    if pool:
        PH, PW = (OH + 2 * pool_pad - 3) // 2 + 1, (OW + 2 * pool_pad - 3) // 2 + 1
        need = B * PH * PW * 64
    else:
        need = B * OH * OW * 64
    if out.numel() != need or out.dtype != torch.bfloat16 or not out.is_contiguous():
        raise ValueError(f"stem output buffer must be contiguous bf16 with {need} elements")
    kernels().stem_forward(ptr(x), ptr(ps.w), ptr(ps.bias), ptr(out), B, H, W, C, OH, OW, ps.pad_t, ps.pad_l,
                           int(pool), PH, PW, pool_pad, stream_handle(stream))
    return out


STEM_F32_K = 160      # 9 halves of 16 + one MFMA's 4 slots (stem_f32.hip SF_K): 37 MFMAs for K = 147


def stem_f32_k_order() -> np.ndarray:
    """[160] flat (kh*21 + kw*3 + c) tap of each packed K position, -1 = zero.

    Slot p = 4h + fq (16h + 4fq + e in the packed row) for p < 35 holds filter
    row p // 5, taps 4 (p % 5) + e: five float4 LDS reads per filter row.  Slot
    35 holds tap 20 (kw = 6, c = 2) of rows 0..3 (a gather), and element 0 of
    the last four slots (positions 144, 148, 152) tap 20 of rows 4..6: the
    kernel's 37th MFMA.
    """
    order = np.full(STEM_F32_K, -1, np.int64)
    for p in range(35):
        for e in range(4):
            order[4 * p + e] = (p // 5) * 21 + 4 * (p % 5) + e
    for e in range(4):
        order[140 + e] = e * 21 + 20
    for fq in range(3):
        order[144 + 4 * fq] = (4 + fq) * 21 + 20
    return order


def pack_stem_f32(kernel_hwio: np.ndarray, bias: np.ndarray, pads, device) -> PackedStem:
    """conv1 (7x7/s2, 3 -> 64, BN folded) for the fp32 stem: [64][160] fp32 in
    `stem_f32_k_order` (every tap once, zeros elsewhere)."""
    kh, kw, cin, cout = kernel_hwio.shape
    if (kh, kw, cin, cout) != (7, 7, 3, 64):
        raise ValueError(f"fp32 stem kernel must be 7x7x3x64, got {kernel_hwio.shape}")
    flat = np.asarray(kernel_hwio, np.float32).transpose(3, 0, 1, 2).reshape(64, 147)
    order = stem_f32_k_order()
    wt = np.zeros((64, STEM_F32_K), np.float32)
    wt[:, order >= 0] = flat[:, order[order >= 0]]
    (pt, pb), (pl, pr) = pads
    return PackedStem(w=torch.from_numpy(wt).to(device=device).contiguous(),
                      bias=torch.from_numpy(np.ascontiguousarray(bias, np.float32)).to(device),
                      cin=3, pad_t=pt, pad_l=pl, pad_b=pb, pad_r=pr)


STEM_F32_VARIANT = 6  # stem_f32.hip: 0 = one unit at a time, 1 = software-pipelined units, 2 = whole rows (OW 112),
#                       5 = whole rows, horizontal pool in the conv epilogue, vertical pool beside the next step,
#                       6 = 5 with the next tile's operand reads issued ahead of the MFMAs (ADAPT_STEM_F32_VARIANT
#                       overrides the default at launch / capture time)


def stem_f32_forward(x: torch.Tensor, ps: PackedStem, out: torch.Tensor, pool_pad: int = 1,
                     stream=None, variant: int = None) -> torch.Tensor:
    """x: [B,H,W,3] fp32 NHWC -> maxpool3x3/s2(relu(conv7x7/s2(x))), fp32 NHWC 64 ch (csrc/kernels/stem_f32.hip)."""
    if x.dtype != torch.float32 or not x.is_contiguous() or x.dim() != 4 or x.shape[-1] != 3:
        raise ValueError("fp32 stem input must be contiguous fp32 NHWC with 3 channels")
    if ps.w.dtype != torch.float32 or ps.w.shape != (64, STEM_F32_K):
        raise ValueError("fp32 stem needs weights packed by pack_stem_f32")
    B, H, W, _ = x.shape
    OH, OW = ps.out_hw(H, W)
    PH, PW = (OH + 2 * pool_pad - 3) // 2 + 1, (OW + 2 * pool_pad - 3) // 2 + 1
    need = B * PH * PW * 64
    if out.numel() != need or out.dtype != torch.float32 or not out.is_contiguous():
        raise ValueError(f"fp32 stem output buffer must be contiguous fp32 with {need} elements")
    kernels().stem_f32_forward(ptr(x), ptr(ps.w), ptr(ps.bias), ptr(out), B, H, W, 3, OH, OW, ps.pad_t, ps.pad_l,
                               PH, PW, pool_pad, stream_handle(stream),
                               int(os.environ.get("ADAPT_STEM_F32_VARIANT", STEM_F32_VARIANT)) if variant is None
                               else int(variant))
    return out


# ------------------------------------------------------------------ fp32 path
# The reference's precision (Keras float32, `src/node.py:177`): conv / GEMM on
# the fp32 matrix cores.  Tiles (BM, BN) per cfg id: 0-5 mirror ADAPT_F32_CFGS
# (csrc/kernels/conv_f32.hip, register-staged, any Cin), 10-41 ADAPT_F32G_CFGS
# (csrc/kernels/conv_f32g.hip, LDS-DMA ring, Cin % 32 == 0); K tiles are 32 floats.
F32_BK = 32
F32_TILES = {0: (128, 128), 1: (128, 64), 2: (64, 128), 3: (64, 64), 4: (256, 64), 5: (64, 256),
             10: (128, 128), 11: (128, 128), 12: (128, 64), 13: (64, 128), 14: (64, 64), 15: (256, 128),
             16: (128, 256), 17: (128, 128), 18: (64, 64), 19: (128, 64), 20: (64, 128), 21: (256, 64)}
# 30-41: the software-pipelined twins of 10-21 (next tile's fragments read between the two
# MFMA halves of the current one); 35 / 36 would spill and do not exist
F32_TILES.update({c + 20: F32_TILES[c] for c in range(10, 22) if c not in (15, 16)})
F32G_CFGS = frozenset(list(range(10, 22)) + [c + 20 for c in range(10, 22) if c not in (15, 16)])


def f32_sk_plan(M: int, N: int, Kpad: int, cfg: int, mult: int = 1):
    """fp32 v2 stream-K launch shape: (tiles, grid, iters per block, fp32 workspace elements)."""
    bm, bn = F32_TILES[cfg]
    tiles = math.ceil(M / bm) * math.ceil(N / bn)
    g, it = kernels().conv_f32g_sk_plan(tiles, Kpad // F32_BK, mult)
    return tiles, g, it, g * 2 * bm * bn


def workspace_elems_f32(M: int, N: int, Kpad: int, cfg: int, ksplit: int) -> int:
    """fp32 workspace a launch needs: split-K slabs or stream-K partial slots
    (Winograd ksplit < 0: -ksplit slabs, the fixup fused into the kernel)."""
    if ksplit > 1:
        return ksplit * M * N
    if ksplit < 0:
        if cfg in F32S_CFGS:
            return f32s_ws_elems(cfg)
        if cfg in WINO_F32_CFGS or cfg in WINO_F32_ABLATE:
            return (4 if ksplit <= WINO_SK_BASE else -ksplit) * M * N    # stream-K: <= 4 partials per unit
        return f32_sk_plan(M, N, Kpad, cfg, -ksplit)[3]
    return 0


def wino_sk_plan(cfg: int, B: int, H: int, W: int, N: int, C: int, ksplit: int):
    """(grid, iterations per block, most partials of one unit) of a stream-K Winograd launch."""
    return tuple(kernels().conv_wino_sk_plan(wino_blocks(cfg, B, H, W, N), C // 16, WINO_SK_BASE - ksplit))


WINO_SK_V3 = frozenset((157, 158))   # stream-K over the v3 chunk body: a block meets <= 2 units


def wino_sk_feasible(cfg: int, B: int, H: int, W: int, N: int, C: int, ksplit: int) -> bool:
    """A stream-K Winograd launch the kernel accepts: <= 4 partials per unit, and for the v3 body at
    most as many chunks per block as a unit has (conv_wino_f32.hip launch_wino_v2)."""
    _, iters, smax = wino_sk_plan(cfg, B, H, W, N, C, ksplit)
    return smax <= 4 and (cfg not in WINO_SK_V3 or iters <= C // 16)


def wino_blocks(cfg: int, B: int, H: int, W: int, N: int) -> int:
    """Blocks per split of a Winograd launch (tile groups x channel groups): the fused split-K
    arrival counters it needs."""
    nwm, fn = {**WINO_F32_CFGS, **WINO_F32_ABLATE}[cfg]
    return math.ceil(B * ((H + 1) // 2) * ((W + 1) // 2) / (16 * nwm)) * (N // (16 * fn))


def f32_counter_elems(cfg: int, ksplit: int, B: int, H: int, W: int, OH: int, OW: int, N: int, Kpad: int) -> int:
    """int32 arrival counters an fp32 launch needs: stream-K tiles (v2 GEMM configs) or fused
    Winograd split-K blocks; 0 for plain launches."""
    if ksplit >= 0:
        return 0
    if cfg in F32S_CFGS:
        return f32s_tiles(cfg, B * OH * OW, N)
    if cfg in WINO4S_F32_CFGS:
        return int(kernels().wino4s_blocks(cfg, B, H, W, N))
    if cfg in WINO_F32_CFGS or cfg in WINO_F32_ABLATE:
        return wino_blocks(cfg, B, H, W, N)
    return f32_sk_plan(B * OH * OW, N, Kpad, cfg, -ksplit)[0]


# fp32 Winograd F(2x2, 3x3) configs (csrc/kernels/conv_wino_f32.hip ADAPT_WINO_CFGS): id -> (waves of 16
# tiles per block, 16-channel output fragments per wave); 3x3 / stride 1 / pad 1 convs only, split-K >= 1
WINO_F32_CFGS = {80: (4, 2), 81: (4, 1), 82: (2, 2), 83: (8, 2), 84: (4, 3), 85: (2, 1),
                 86: (4, 2), 87: (4, 3), 88: (8, 1),          # 86-88: the next chunk's patch prefetched
                 100: (8, 2), 101: (8, 1), 102: (4, 1),       # v2: input patches staged in LDS by LDS-DMA
                 103: (8, 2), 104: (8, 1), 105: (4, 1),       # v2 with the bank-swizzled wave image
                 106: (8, 2), 107: (8, 1), 108: (4, 1),       # ... and the next patch read before the barrier
                 110: (8, 2), 111: (8, 2), 112: (4, 1), 113: (4, 1), 114: (8, 1),    # stream-K twins
                 116: (8, 1), 117: (4, 1),                    # v3: pipelined chunk body (fragment prefetch,
                                                              # DMA spread over the MFMA groups)
                 130: (4, 1), 131: (8, 2), 132: (4, 1),       # 105 / 103 / 117 with the XCD-aware block order
                 118: (8, 2), 119: (8, 2),                    # FN = 2 with the next chunk's DMA spread over the
                                                              # MFMA groups (119: + XCD order)
                 150: (8, 2), 151: (8, 2), 152: (8, 2), 153: (8, 2),    # 118 / 119 with the next chunk's
                                                              # DMA front-loaded, 2 (150-151) / 3 pieces a group
                 154: (8, 2), 155: (8, 2), 156: (8, 2),       # 118 + stagger / priority / both for waves 4-7
                 157: (8, 2), 158: (8, 2),                    # stream-K twins of 118 / 155
                 160: (8, 2), 161: (8, 2),                    # 118 / 155 with the half fragment prefetch
                 162: (8, 2), 163: (8, 2),                    # front-loaded DMA + next patch rows 0-2 read early
                 164: (8, 2), 165: (8, 2),                    # 162 / 163 with the DMA hidden from the wait model
                 166: (8, 1), 167: (4, 1),                    # 116 / 117 likewise (partial waits for the prefetch)
                 170: (8, 2),                                 # 118 + in-loop phase stamps (tools/wino_timeline.py only)
                 171: (8, 2), 172: (8, 2),                    # 118 with LDS counters instead of the chunk barrier
                                                              # (172: + the in-loop stamps, measurement only)
                 140: (4, 1), 141: (8, 1)}                    # persistent: two blocks per CU walk the units as
                                                              # one chunk stream (whole K only)
WINO_V2_CFGS = frozenset((100, 101, 102, 103, 104, 105, 106, 107, 108, 110, 111, 112, 113, 114, 116, 117,
                          118, 119, 130, 131, 132, 140, 141, 150, 151, 152, 153,
                          154, 155, 156, 157, 158, 160, 161, 162, 163,
                          164, 165, 166, 167, 170, 171, 172))
WINO_MEASURE_CFGS = frozenset((170, 172))     # never tuned (stamps cost a few cycles per chunk)
WINO_PU_CFGS = frozenset((140, 141))
# stream-K Winograd configs: ksplit <= -100 means (-ksplit - 100) x 256 blocks over the (unit, chunk) space
WINO_SK_CFGS = frozenset((110, 111, 112, 113, 114, 157, 158))
WINO_SK_BASE = -100


def wino_map_ok(cfg: int, H: int, W: int) -> bool:
    """v2 configs stage a wave's 16 tiles as <= 4 tile-row segments: 2x2-tile rows of >= 4 tiles."""
    return cfg not in WINO_V2_CFGS or (W + 1) // 2 >= 4


# cfg 80 with ablation switches (conv_wino_f32.hip ABL = id - 90): tools/conv_bench_f32.py only, never tuned
WINO_F32_ABLATE = {90 + a: (4, 2) for a in (1, 2, 4, 5, 8, 9)}
# B^T (input), G (weights) and A^T (output) of F(2x2, 3x3) (Lavin & Gray 2016)
WINO_BT = np.array([[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]], np.float64)
WINO_G = np.array([[1, 0, 0], [0.5, 0.5, 0.5], [0.5, -0.5, 0.5], [0, 0, 1]], np.float64)
WINO_AT = np.array([[1, 1, 1, 0], [0, 1, -1, -1]], np.float64)


def wino_supported(pc: "PackedConv") -> bool:
    return ((pc.kh, pc.kw, pc.stride, pc.pad_t, pc.pad_l, pc.pad_b, pc.pad_r) == (3, 3, 1, 1, 1, 1, 1)
            and pc.cin % 16 == 0 and pc.cout % 16 == 0)


def wino_pack_np(kernel_hwio: np.ndarray) -> np.ndarray:
    """U_p = (G g G^T)_p of every (cin, cout) filter in fp64, rounded to fp32, in the MFMA fragment
    order conv_wino_f32.hip streams: [C/16][N/16][16 positions][64 lanes][4], lane l = 16 q + n'
    holding U_p[16 kc + 4 q + s][16 nf + n'] for s = 0..3."""
    kh, kw, C, N = kernel_hwio.shape
    if (kh, kw) != (3, 3) or C % 16 or N % 16:
        raise ValueError(f"Winograd F(2x2,3x3) packs 3x3 filters with C, N % 16 == 0 (got {kernel_hwio.shape})")
    U = np.einsum("ai,ijcn,bj->abcn", WINO_G, np.asarray(kernel_hwio, np.float64), WINO_G)   # [4][4][C][N]
    U = U.reshape(16, C // 16, 4, 4, N // 16, 16)          # p, kc, q, s, nf, n'
    return np.ascontiguousarray(U.transpose(1, 4, 0, 2, 5, 3).reshape(C // 16, N // 16, 16, 64, 4).astype(np.float32))


# B^T (input), G (weights) and A^T (output) of F(4x4, 3x3), interpolation points 0, +-1, +-2 (Lavin & Gray 2016)
WINO4_BT = np.array([[4, 0, -5, 0, 1, 0], [0, -4, -4, 1, 1, 0], [0, 4, -4, -1, 1, 0],
                     [0, -2, -1, 2, 1, 0], [0, 2, -1, -2, 1, 0], [0, 4, 0, -5, 0, 1]], np.float64)
WINO4_G = np.array([[1 / 4, 0, 0], [-1 / 6, -1 / 6, -1 / 6], [-1 / 6, 1 / 6, -1 / 6],
                    [1 / 24, 1 / 12, 1 / 6], [1 / 24, -1 / 12, 1 / 6], [0, 0, 1]], np.float64)
WINO4_AT = np.array([[1, 1, 1, 1, 1, 0], [0, 1, -1, 2, -2, 0], [0, 1, 1, 4, 4, 0], [0, 1, -1, 8, -8, 1]],
                    np.float64)


# fp32 Winograd F(4x4, 3x3) as transform + pure-MFMA GEMM (csrc/kernels/wino4s_f32.hip): id -> (WT, WN, PG, R,
# order): a block of WT x WN waves (16 tiles x 16 output channels x 36 positions each), PG positions per LDS
# ring stage, R ring slots, block order 0 = channel blocks fastest / 1 = tile blocks fastest.  ksplit >= 1
# (C / 16 divisible by it; > 1 adds the split-K reduce launch).  Workspace: V (36 x 16-tile groups x C) then
# the split-K partial outputs (wino4s_ws_elems).
WINO4S_F32_CFGS = {220: (2, 2, 6, 4, 0), 221: (2, 2, 6, 3, 0), 222: (1, 2, 6, 4, 0), 223: (2, 4, 4, 4, 0),
                   224: (2, 2, 6, 4, 1), 225: (2, 1, 6, 4, 0), 226: (1, 1, 9, 4, 0), 227: (2, 2, 4, 4, 0),
                   228: (4, 2, 4, 4, 0), 229: (4, 2, 4, 4, 1), 230: (2, 2, 12, 3, 0), 231: (2, 2, 12, 3, 1),
                   # fragments of the next stage read under the current stage's MFMAs
                   232: (2, 2, 4, 4, 0), 233: (2, 2, 6, 3, 0), 234: (2, 2, 6, 4, 0), 235: (2, 4, 4, 4, 0),
                   236: (2, 2, 4, 5, 0), 237: (2, 2, 2, 8, 0),      # deeper rings, 2 blocks per CU
                   299: (2, 2, 6, 3, 0)}     # 299: 221 with per-wave stamps (tools/wino4s_timeline.py), never tuned


def wino4s_supported(pc: "PackedConv") -> bool:
    return ((pc.kh, pc.kw, pc.stride, pc.pad_t, pc.pad_l, pc.pad_b, pc.pad_r) == (3, 3, 1, 1, 1, 1, 1)
            and pc.cin % 16 == 0 and pc.cout % 16 == 0)


def wino4s_pack_np(kernel_hwio: np.ndarray) -> np.ndarray:
    """U_p = (G g G^T)_p in fp64, rounded once to fp32, in the fragment order of wino4s_f32.hip:
    [N/16][C/16][36 positions][64 lanes][4], lane 16 g + n holding U_p[16 kc + 4 g + j][16 ng + n] at j."""
    kh, kw, C, N = kernel_hwio.shape
    if (kh, kw) != (3, 3) or C % 16 or N % 16:
        raise ValueError(f"Winograd F(4x4) split packs 3x3 filters with C, N % 16 == 0 (got {kernel_hwio.shape})")
    U = np.einsum("ai,ijcn,bj->abcn", WINO4_G, np.asarray(kernel_hwio, np.float64), WINO4_G)   # [6][6][C][N]
    U = U.reshape(36, C // 16, 4, 4, N // 16, 16)                  # p, kc, g, j, ng, n
    return np.ascontiguousarray(U.transpose(4, 1, 0, 2, 5, 3).reshape(N // 16, C // 16, 36, 64, 4)
                                .astype(np.float32))


def wino4s_ws_elems(B: int, H: int, W: int, C: int, N: int, ksplit: int) -> int:
    return int(kernels().wino4s_ws_floats(B, H, W, C, N, ksplit))


def wino4s_splits(C: int) -> list:
    kc = C // 16
    return [k for k in (1, 2, 4, 8) if kc % k == 0]


# fp32 persistent pointwise configs (csrc/kernels/pw_f32.hip): id -> pixels per tile; 1x1 / s1 / p0 convs
# with K in {64, 128, 256, 512} and N a multiple of the slice (FPW x 128 channels), ksplit 1
# 122 / 123: the streaming variant (no LDS, no block barrier; bm codes 1 / 2: two waves per SIMD / the
# widest channel slice per wave)
# 124: 123 with a 16-K-step activation ring (bm code 3; K in 256 / 512 / 1024)
# 125 / 126: 122 / 123 with the left-over tile round split by output fragment over otherwise idle waves
#            (bm codes 4 / 5; FPW >= 2 and a partial last round only, pw_f32_tail_plan)
PW_F32_CFGS = {120: 16, 121: 32, 122: 1, 123: 2, 124: 3, 125: 4, 126: 5}
PW_F32_TAIL = frozenset((125, 126))
PW_F32_FPW = {64: 2, 128: 4, 256: 2, 512: 1, 1024: 1}     # 16-channel fragments per wave
PW_F32_KG = {1024: 2}                                       # K groups of waves (partials meet in LDS)
PW_F32_BMS = {64: (1, 2, 4, 5, 16, 32), 128: (1, 2, 4, 5, 16, 32), 256: (1, 2, 3, 4, 5, 16, 32),
              512: (1, 2, 3, 4, 5, 16, 32), 1024: (1, 2, 3, 4, 5, 16)}


# fp32 big-tile 1x1 GEMM (csrc/kernels/gemm_f32s.hip, cfg ids 300+): id -> (BM, BN); 4 waves side by side
# along N, BM chosen per layer so the tiles fill the CUs; 1x1 / pad 0 / stride 1-2, Cin % 32 == 0, N % 16 == 0;
# ksplit 1 (one block per tile) or -1 (stream-K over 256 blocks, XCD-grouped, fused fixup)
F32S_CFGS = {300: (112, 256), 302: (112, 128),          # (301, 303-306 retired: never picked in-graph)
             # 112-row tiles placed 98 rows apart (the kernel's TM): 256 tiles on 6272 x 256 / 1568 x 2048; whole K
             307: (98, 64), 308: (98, 128), 309: (49, 64)}
F32S_TM = frozenset((307, 308, 309))     # owned-row tiles: ksplit 1 only
# measured behind the pointwise / ring kernels on the ResNet-50 bs=32 1x1 shapes in isolation (profiles/r5/
# gemm_f32s_attribution.md: one tile per CU writes the whole output after the K loop, 5-14 us of HBM-bound
# epilogue that nothing overlaps), so the isolated-timing tuner never picks them; cfg 307 on the stage-4 `_1`
# convs wins in the whole-model A/B (tools/ab_cfg.py: 2.2738 -> 2.2648 ms): the owned-row tiles (F32S_TM) are
# tuner candidates, which the fp32 tuner's in-graph refinement can pick
F32_UNTUNED = (frozenset(F32S_CFGS) - F32S_TM) | {299}


def f32s_supported(pc: "PackedConv") -> bool:
    return ((pc.kh, pc.kw, pc.pad_t, pc.pad_l, pc.pad_b, pc.pad_r) == (1, 1, 0, 0, 0, 0) and pc.stride in (1, 2)
            and pc.cin % 32 == 0 and pc.cout % 16 == 0 and pc.Kpad == pc.cin)


def f32s_tiles(cfg: int, M: int, N: int) -> int:
    bm, bn = F32S_CFGS[cfg]
    return math.ceil(M / bm) * math.ceil(N / bn)


def f32s_ws_elems(cfg: int) -> int:
    """Stream-K workspace floats (2 partial slots of a whole BM x BN tile per block, 256 blocks)."""
    return int(kernels().gemm_f32s_ws_elems(cfg))


def pw_f32_slice(K: int) -> int:
    """Output channels per block of the pointwise kernel (FPW x 16 x waves per K group)."""
    return PW_F32_FPW[K] * 16 * (8 // PW_F32_KG.get(K, 1))


def pw_f32_packable(pc: "PackedConv") -> bool:
    """1x1, no padding, stride 1 or 2, K one the pointwise kernel is built for."""
    return ((pc.kh, pc.kw, pc.pad_t, pc.pad_l, pc.pad_b, pc.pad_r) == (1, 1, 0, 0, 0, 0) and pc.stride in (1, 2)
            and pc.cin in PW_F32_FPW)


def pw_f32_shape_ok(pc: "PackedConv", bm: int = 16) -> bool:
    """Packable and some built instance's channel slice divides N (and the dual-output split)."""
    return pw_f32_packable(pc) and kernels().pw_f32_fpw(pc.cin, pc.cout, int(pc.n_split), bm) > 0


def pack_pw_f32(kernel_hwio: np.ndarray) -> np.ndarray:
    """[N/16][K/16][64 lanes][4] fp32: lane 16q + r of fragment gf, half h holds W[16h + 4q + s][16 gf + r]."""
    K, N = kernel_hwio.shape[2], kernel_hwio.shape[3]
    w = np.asarray(kernel_hwio[0, 0], np.float64).reshape(K // 16, 4, 4, N // 16, 16)    # h, q, s, gf, r
    return np.ascontiguousarray(w.transpose(3, 0, 1, 4, 2).reshape(N // 16, K // 16, 64, 4).astype(np.float32))


def f32_cfg_supported(cfg: int, cin: int, cout: int, pc: Optional["PackedConv"] = None) -> bool:
    """Whether fp32 tile config `cfg` runs a conv with `cin` input / `cout` output channels
    (Winograd configs also need the conv itself: 3x3 / s1 / p1 with its transformed weights;
    the pointwise configs a 1x1 / s1 conv with its fragment-packed weights)."""
    if cfg in PW_F32_CFGS:
        return (pc is not None and pc.pwf is not None and PW_F32_CFGS[cfg] in PW_F32_BMS[pc.cin]
                and pw_f32_shape_ok(pc, PW_F32_CFGS[cfg]))
    if cfg in WINO4S_F32_CFGS:
        return (pc is not None and pc.wino4s is not None and wino4s_supported(pc)
                and bool(kernels().wino4s_ok(cfg, cin, cout, 1)))
    if cfg in F32S_CFGS:
        return pc is not None and f32s_supported(pc)
    if cfg in WINO_F32_CFGS or cfg in WINO_F32_ABLATE:
        fn = {**WINO_F32_CFGS, **WINO_F32_ABLATE}[cfg][1]
        return pc is not None and pc.wino is not None and wino_supported(pc) and cout % (16 * fn) == 0
    if cfg in F32G_CFGS:
        return cin % F32_BK == 0 and cout % 4 == 0
    return cfg in F32_TILES


def pack_conv_f32(kernel_hwio: np.ndarray, bias: np.ndarray, stride: int, pads, device,
                  row_align: int = 256) -> PackedConv:
    """[Npad][Kpad] fp32 weights, k = (kh, kw, ci) with ci innermost; no channel padding."""
    kh, kw, cin, cout = kernel_hwio.shape
    K = kh * kw * cin
    Kpad = int(math.ceil(K / F32_BK) * F32_BK)
    Npad = int(math.ceil(cout / row_align) * row_align)
    wt = np.zeros((Npad, Kpad), np.float32)
    wt[:cout, :K] = np.asarray(kernel_hwio, np.float32).transpose(3, 0, 1, 2).reshape(cout, K)
    (pt, pb), (pl, pr) = pads
    pc = PackedConv(w=torch.from_numpy(wt).to(device=device).contiguous(),
                    bias=torch.from_numpy(np.ascontiguousarray(bias, np.float32)).to(device),
                    kh=kh, kw=kw, cin=cin, cout=cout, stride=stride, pad_t=pt, pad_l=pl, pad_b=pb, pad_r=pr)
    if wino_supported(pc):
        pc.wino = torch.from_numpy(wino_pack_np(kernel_hwio)).to(device=device).contiguous()
    if wino4s_supported(pc):
        pc.wino4s = torch.from_numpy(wino4s_pack_np(kernel_hwio)).to(device=device).contiguous()
    if pw_f32_packable(pc) and cout % 16 == 0:
        pc.pwf = torch.from_numpy(pack_pw_f32(kernel_hwio)).to(device=device).contiguous()
    return pc


def choose_cfg_f32(M: int, N: int, Kpad: int, occupancy: int = 2):
    """(cfg, ksplit) for the fp32 kernel: the fp32 matrix rate is 1/16 of bf16,
    so every conv is compute-bound; fill the CUs first, then prefer big tiles."""
    best = None
    ktiles = Kpad // F32_BK
    for cfg, (bm, bn) in F32_TILES.items():
        if cfg in F32G_CFGS:
            continue                                 # v2 tiles are chosen by the autotuner (tuning table)
        tiles = math.ceil(M / bm) * math.ceil(N / bn)
        for ks in (1, 2, 4, 8, 16):
            if ks > 1 and ktiles // ks < 8:
                continue
            blocks = tiles * ks
            waves = math.ceil(blocks / (NUM_CUS * occupancy))
            eff = {0: 1.0, 1: 0.93, 2: 0.93, 3: 0.8, 4: 1.0, 5: 1.0}[cfg]
            t = waves * bm * bn * (Kpad / ks) / eff
            if ks > 1:
                t += M * N * (ks + 1) * 2.0          # slab write + reduce read (fp32), arbitrary units
            if blocks < NUM_CUS:
                t *= 1.0 + 0.5 * (NUM_CUS - blocks) / NUM_CUS
            cand = (t, cfg, ks)
            if best is None or cand < best:
                best = cand
    return best[1], best[2]


def conv_forward_f32(x: torch.Tensor, pc: PackedConv, out: torch.Tensor, residual: Optional[torch.Tensor] = None,
                     relu: int = 0, cfg: Optional[int] = None, ksplit: int = 1,
                     workspace: Optional[torch.Tensor] = None, stream=None,
                     counters: Optional[torch.Tensor] = None, out2: Optional[torch.Tensor] = None,
                     relu2: int = 0) -> torch.Tensor:
    """fp32 conv / GEMM: x [B,H,W,Cin] (or [M,K]) fp32 -> out [B,OH,OW,Cout] fp32, with
    act(conv + bias (+ residual)) fused.  ksplit > 1: split-K, needs `workspace`
    (ksplit*M*N fp32); ksplit < 0 (v2 configs): stream-K over -ksplit x 256 blocks,
    needs `workspace` (workspace_elems_f32) and `counters` (int32 zeros, one per tile).
    Dual output (``pc.n_split > 0``, two sibling 1x1 convs packed along N, no residual):
    channels [0, n_split) go to `out` (activation `relu`), the rest to `out2` (`relu2`)."""
    if x.dim() == 2:
        B, H, W, C = x.shape[0], 1, 1, x.shape[1]
    else:
        B, H, W, C = x.shape
    if C != pc.cin:
        raise ValueError(f"conv expects {pc.cin} input channels, got {C}")
    for t, nm in ((x, "x"), (out, "out")):
        if t.dtype != torch.float32 or not t.is_contiguous():
            raise ValueError(f"fp32 conv: {nm} must be contiguous fp32")
    if pc.w.dtype != torch.float32:
        raise ValueError("fp32 conv needs weights packed by pack_conv_f32")
    OH, OW = pc.out_hw(H, W)
    M, N = B * OH * OW, pc.cout
    ns = pc.n_split
    if ns:
        if out2 is None or residual is not None or ns % 4:
            raise ValueError("dual-output fp32 conv needs out2 and no residual")
        if out.numel() != M * ns or out2.numel() != M * (N - ns) or out2.dtype != torch.float32 \
                or not out2.is_contiguous():
            raise ValueError("dual-output fp32 conv: out / out2 sizes")
    elif out2 is not None:
        raise ValueError("out2 given for a single-output conv")
    elif out.numel() != M * N:
        raise ValueError(f"conv output buffer has {out.numel()} elements, need {M * N}")
    if residual is not None and (residual.numel() != M * N or residual.dtype != torch.float32
                                 or not residual.is_contiguous()):
        raise ValueError("residual must be contiguous fp32 with the output's shape")
    if int(relu) not in (0, 1, 2):
        raise ValueError("conv epilogue activation must be 0 (none), 1 (ReLU) or 2 (ReLU6)")
    if cfg is None:
        cfg, ksplit = choose_cfg_f32(M, N, pc.Kpad)
    if cfg in PW_F32_CFGS:
        if not f32_cfg_supported(cfg, C, N, pc) or int(ksplit or 1) != 1 or x.dim() != 4:
            raise ValueError(f"pointwise fp32 config {cfg}: 1x1 / s1-2 conv, K in {sorted(PW_F32_FPW)}, "
                             f"N (and the dual-output split) a multiple of the slice, ksplit 1")
        if cfg in PW_F32_TAIL and not kernels().pw_f32_tail_plan(M, C, N, int(ns), PW_F32_CFGS[cfg])[0]:
            raise ValueError(f"pointwise fp32 config {cfg}: no partial last tile round to split")
        kernels().pw_f32_forward(ptr(x), ptr(pc.pwf), ptr(pc.bias), ptr(residual), ptr(out), M, C, N, int(relu),
                                 PW_F32_CFGS[cfg], stream_handle(stream), B, H, W, OH, OW, pc.stride, ptr(out2),
                                 int(ns), int(relu2))
        return out
    if cfg in F32S_CFGS:
        # big-tile 1x1 GEMM: whole K per tile (ksplit 1) or stream-K over 256 blocks (ksplit -1)
        ksplit = int(ksplit) or 1
        if not f32_cfg_supported(cfg, C, N, pc) or x.dim() != 4 or ksplit not in (1, -1):
            raise ValueError(f"fp32 1x1 GEMM config {cfg}: 1x1 / pad 0 / stride 1-2 conv, Cin % 32 == 0, "
                             f"N % 16 == 0, ksplit 1 or -1")
        ws_ptr = ctr_ptr = 0
        if ksplit < 0:
            need = f32s_ws_elems(cfg)
            if workspace is None:
                workspace = torch.empty(need, dtype=torch.float32, device=x.device)
            if workspace.numel() < need or workspace.dtype != torch.float32:
                raise ValueError(f"fp32 1x1 GEMM stream-K needs an fp32 workspace of {need} elements")
            nt = f32s_tiles(cfg, M, N)
            if counters is None or counters.numel() < nt or counters.dtype != torch.int32:
                raise ValueError(f"fp32 1x1 GEMM stream-K needs {nt} int32 tile counters (zeroed)")
            ws_ptr, ctr_ptr = ptr(workspace), ptr(counters)
        kernels().conv_f32_forward(ptr(x), ptr(pc.w), ptr(pc.bias), ptr(residual), ptr(out), ws_ptr, B, H, W,
                                   C, OH, OW, N, 1, 1, pc.stride, 0, 0, pc.K, pc.Kpad, int(relu), ksplit, int(cfg),
                                   stream_handle(stream), ctr_ptr, ptr(out2), int(ns), int(relu2))
        return out
    if cfg in WINO4S_F32_CFGS:
        # Winograd F(4x4, 3x3): input transform -> V (workspace), pure-MFMA GEMM with the output transform in
        # its epilogue, and for ksplit > 1 the split-K reduce (bias / ReLU there)
        ksplit = int(ksplit) or 1
        if (not f32_cfg_supported(cfg, C, N, pc) or (OH, OW) != (H, W) or x.dim() != 4 or residual is not None
                or not kernels().wino4s_ok(cfg, C, N, ksplit)):
            raise ValueError(f"Winograd F(4x4) split config {cfg}: 3x3/s1/p1 conv with wino4s weights, C % 16 == 0, "
                             f"N % (16 x WN) == 0, no residual, |ksplit| in {wino4s_splits(C)} (fused: <= -2)")
        need = wino4s_ws_elems(B, H, W, C, N, ksplit)
        if workspace is None:
            workspace = torch.empty(need, dtype=torch.float32, device=x.device)
        if workspace.numel() < need or workspace.dtype != torch.float32:
            raise ValueError(f"Winograd F(4x4) split needs an fp32 workspace of {need} elements")
        ctr_ptr = 0
        if ksplit < 0:                       # fused split-K fixup: one arrival counter per (tile, channel) block
            nb = int(kernels().wino4s_blocks(cfg, B, H, W, N))
            if counters is None or counters.numel() < nb or counters.dtype != torch.int32:
                raise ValueError(f"Winograd F(4x4) fused split-K needs {nb} int32 arrival counters (zeroed)")
            ctr_ptr = ptr(counters)
        kernels().wino4s_forward(ptr(x), ptr(pc.wino4s), ptr(pc.bias), ptr(out), ptr(workspace), B, H, W, C, N,
                                 int(relu), ksplit, int(cfg), stream_handle(stream), ctr_ptr)
        return out
    if cfg in WINO_F32_CFGS or cfg in WINO_F32_ABLATE:
        # ksplit > 1: slabs + splitk_reduce_f32; ksplit <= -2: -ksplit slabs, the last split of
        # each block adds them in split order inside the kernel (needs `counters`)
        # ksplit <= -100 (stream-K configs only): (-ksplit - 100) x 256 blocks over the (unit, chunk) space
        ksplit = int(ksplit) or 1
        sk = ksplit <= WINO_SK_BASE
        if not f32_cfg_supported(cfg, C, N, pc) or (OH, OW) != (H, W) or x.dim() != 4 or ksplit == -1 \
                or not wino_map_ok(cfg, H, W) or sk != (cfg in WINO_SK_CFGS):
            raise ValueError(f"Winograd config {cfg}: 3x3/s1/p1 conv with transformed weights, C % 16 == 0, "
                             f"N % 16 * fragments == 0, split-K >= 1 or fused split-K <= -2; stream-K configs "
                             f"{sorted(WINO_SK_CFGS)} take ksplit <= {WINO_SK_BASE}")
        if not sk and (abs(ksplit) > (C // 16) or ksplit < -4):
            raise ValueError(f"Winograd split-K {ksplit} exceeds the {C // 16} channel chunks (fused: <= 4 splits)")
        if cfg in WINO_PU_CFGS and ksplit != 1:
            raise ValueError(f"persistent Winograd config {cfg} runs whole K only (ksplit 1)")
        if sk and wino_sk_plan(cfg, B, H, W, N, C, ksplit)[2] > 4:
            raise ValueError("Winograd stream-K would cut a unit into more than 4 partials")
        ws_ptr = ctr_ptr = 0
        if ksplit != 1:
            need = workspace_elems_f32(M, N, pc.Kpad, cfg, ksplit)
            if need * 4 > 0x7fffffff:
                raise ValueError("Winograd split-K slabs beyond 2 GiB")
            if workspace is None:
                workspace = torch.empty(need, dtype=torch.float32, device=x.device)
            if workspace.numel() < need or workspace.dtype != torch.float32:
                raise ValueError(f"Winograd split-K {ksplit} needs an fp32 workspace of {need} elements")
            ws_ptr = ptr(workspace)
        if ksplit < 0:
            nb = wino_blocks(cfg, B, H, W, N)
            if counters is None or counters.numel() < nb or counters.dtype != torch.int32:
                raise ValueError(f"Winograd fused split-K / stream-K needs {nb} int32 arrival counters (zeroed)")
            ctr_ptr = ptr(counters)
        kernels().conv_f32_forward(ptr(x), ptr(pc.wino), ptr(pc.bias), ptr(residual), ptr(out), ws_ptr, B, H, W, C,
                                   OH, OW, N, 3, 3, 1, 1, 1, pc.K, pc.Kpad, int(relu), ksplit, int(cfg),
                                   stream_handle(stream), ctr_ptr)
        return out
    if cfg not in F32_TILES:
        raise ValueError(f"unknown fp32 tile config {cfg}")
    bm, bn = F32_TILES[cfg]
    if pc.w.shape[0] < math.ceil(N / bn) * bn or pc.Kpad % F32_BK:
        raise ValueError("packed fp32 weights not padded to the tile")
    ws_ptr = ctr_ptr = 0
    ksplit = int(ksplit) or 1
    if ksplit < 0:
        if cfg not in F32G_CFGS:
            raise ValueError("fp32 stream-K runs on the v2 configs only")
        tiles = f32_sk_plan(M, N, pc.Kpad, cfg, -ksplit)[0]
        if counters is None or counters.numel() < tiles or counters.dtype != torch.int32:
            raise ValueError(f"fp32 stream-K needs {tiles} int32 tile counters")
        ctr_ptr = ptr(counters)
    if ksplit != 1:
        need = workspace_elems_f32(M, N, pc.Kpad, cfg, ksplit)
        if workspace is None:
            workspace = torch.empty(need, dtype=torch.float32, device=x.device)
        if workspace.numel() < need or workspace.dtype != torch.float32:
            raise ValueError(f"ksplit {ksplit} needs an fp32 workspace of {need} elements")
        ws_ptr = ptr(workspace)
    kernels().conv_f32_forward(ptr(x), ptr(pc.w), ptr(pc.bias), ptr(residual), ptr(out), ws_ptr, B, H, W, C, OH, OW,
                               N, pc.kh, pc.kw, pc.stride, pc.pad_t, pc.pad_l, pc.K, pc.Kpad, int(relu),
                               ksplit, int(cfg), stream_handle(stream), ctr_ptr, ptr(out2), int(ns), int(relu2))
    return out


# ------------------------------------------------- persistent pointwise conv
# csrc/kernels/pw_wide.hip: 1x1 / stride 1, K <= 128, N = 4 x 64 x waves, weights held in
# registers by each wave for the whole launch (ResNet stage 3's 128 -> 512 "_out" convs)
PW_CFGS = {60: 16, 61: 32}                   # config id -> pixels per tile


def pw_supported(pc: "PackedConv") -> bool:
    return ((pc.kh, pc.kw, pc.stride, pc.pad_t, pc.pad_l, pc.pad_b, pc.pad_r) == (1, 1, 1, 0, 0, 0, 0)
            and pc.cin == pc.Kpad and pc.cout == pc.w.shape[0] and not pc.n_split
            and bool(kernels().pw_res_supported(int(pc.cin), int(pc.cout))))


def pw_fragments(pc: "PackedConv") -> torch.Tensor:
    """pc.w ([N][K] bf16) in MFMA fragment order (pack_fragments), cached on pc."""
    wf = getattr(pc, "_pw_frag", None)
    if wf is None:
        N, K = pc.w.shape
        wf = pc.w.reshape(N // 16, 16, K // 32, 4, 8).permute(0, 2, 3, 1, 4).contiguous().reshape(-1)
        pc._pw_frag = wf
    return wf


def pw_forward(x: torch.Tensor, pc: "PackedConv", out: torch.Tensor, residual: Optional[torch.Tensor] = None,
               relu: int = 0, cfg: int = 61, blocks: int = 256, stream=None) -> torch.Tensor:
    if not pw_supported(pc):
        raise ValueError("pw conv: needs a 1x1 stride-1 conv with (K, N) in (128, 512) / (64, 256)")
    M = x.numel() // pc.cin
    for t, n in ((x, "x"), (out, "out"), (residual, "residual")):
        if t is not None and (t.dtype != torch.bfloat16 or not t.is_contiguous()):
            raise ValueError(f"pw conv: {n} must be contiguous bf16")
    if x.shape[-1] != pc.cin or out.numel() != M * pc.cout or (residual is not None and residual.numel() != M * pc.cout):
        raise ValueError(f"pw conv: x {tuple(x.shape)} / out {tuple(out.shape)} do not match {pc.cin} -> {pc.cout}")
    kernels().pw_res_forward(ptr(x), ptr(pw_fragments(pc)), ptr(pc.bias), ptr(residual), ptr(out), M, pc.cin,
                             pc.cout, int(relu), PW_CFGS[cfg], int(blocks), stream_handle(stream))
    return out


# channel-sliced persistent pointwise (csrc/kernels/pw_slice.hip): config id -> kernel code; a block keeps a
# slice of NS = CF x WAVES x 16 output channels' weights in VGPRs and walks pixel tiles (code: (CF, WAVES, PT)
# = 0: (4, 8, 16), 1: (2, 8, 16), 2: (1, 8, 16), 3: (2, 4, 32), 4: (1, 4, 32), 5: (4, 4, 16)); K in 128 / 256 /
# 512 / 1024 with CF x K <= 1024, N a multiple of NS
PS_CFGS = {74: 0, 75: 1, 76: 2, 77: 3, 78: 4, 79: 5}
PS_GRIDS = (1, 2)          # the tuner's `ksplit` for these configs: blocks per CU (1 or 2 x NUM_CUS blocks)


def ps_supported(pc: "PackedConv", cfg: int) -> bool:
    return ((pc.kh, pc.kw, pc.stride, pc.pad_t, pc.pad_l, pc.pad_b, pc.pad_r) == (1, 1, 1, 0, 0, 0, 0)
            and pc.cin == pc.Kpad and pc.cout <= pc.w.shape[0] and not pc.n_split     # padded rows never read
            and bool(kernels().pw_slice_supported(int(pc.cin), int(pc.cout), PS_CFGS[cfg])))


def ps_forward(x: torch.Tensor, pc: "PackedConv", out: torch.Tensor, residual: Optional[torch.Tensor] = None,
               relu: int = 0, cfg: int = 74, blocks: int = 256, stream=None) -> torch.Tensor:
    if not ps_supported(pc, cfg):
        raise ValueError(f"pw_slice conv: config {cfg} does not take {pc.cin} -> {pc.cout} (1x1 / stride 1)")
    M = x.numel() // pc.cin
    for t, n in ((x, "x"), (out, "out"), (residual, "residual")):
        if t is not None and (t.dtype != torch.bfloat16 or not t.is_contiguous()):
            raise ValueError(f"pw_slice conv: {n} must be contiguous bf16")
    if x.shape[-1] != pc.cin or out.numel() != M * pc.cout or (residual is not None and residual.numel() != M * pc.cout):
        raise ValueError(f"pw_slice conv: x {tuple(x.shape)} / out {tuple(out.shape)} do not match {pc.cin} -> {pc.cout}")
    kernels().pw_slice_forward(ptr(x), ptr(pw_fragments(pc)), ptr(pc.bias), ptr(residual), ptr(out), M, pc.cin,
                               pc.cout, int(relu), PS_CFGS[cfg], int(blocks), stream_handle(stream))
    return out


RR3_CFGS = {71: 1, 72: 2}                     # 3x3 with the filter resident in VGPRs (conv3x3_rr.hip) -> K groups


def rr3_supported(pc: "PackedConv") -> bool:
    return ((pc.kh, pc.kw, pc.stride, pc.pad_t, pc.pad_l, pc.pad_b, pc.pad_r) == (3, 3, 1, 1, 1, 1, 1)
            and pc.cin == 128 and pc.cout == 128 and pc.Kpad == 9 * 128 and not pc.n_split)


def rr3_forward(x: torch.Tensor, pc: "PackedConv", out: torch.Tensor, relu: int = 1, kg: int = 1,
                stream=None) -> torch.Tensor:
    if not rr3_supported(pc):
        raise ValueError("rr3 conv: needs a 3x3 / s1 / p1 conv 128 -> 128")
    if x.dim() != 4 or tuple(x.shape[1:]) != (28, 28, 128) or tuple(out.shape) != tuple(x.shape):
        raise ValueError(f"rr3 conv: x {tuple(x.shape)} out {tuple(out.shape)} (needs B x 28 x 28 x 128)")
    for t in (x, out):
        if t.dtype != torch.bfloat16 or not t.is_contiguous():
            raise ValueError("rr3 conv: contiguous bf16 NHWC tensors")
    kernels().conv3x3_rr_forward(ptr(x), ptr(pw_fragments(pc)), ptr(pc.bias), ptr(out), int(x.shape[0]), 28, 28,
                                 128, int(relu), int(kg), stream_handle(stream))
    return out


# channel-split register-resident 3x3 (conv3x3_cs.hip): a block holds a 64- (stage 4) or
# 32-channel (stage 5) slice of the filter in VGPRs and walks pixel tiles staged in LDS
CS3_CFGS = {73: 0}
CS3_SHAPES = {(256, 14, 14), (512, 7, 7)}       # (C, H, W): ResNet stages 4 and 5


def cs3_supported(pc: "PackedConv") -> bool:
    return ((pc.kh, pc.kw, pc.stride, pc.pad_t, pc.pad_l, pc.pad_b, pc.pad_r) == (3, 3, 1, 1, 1, 1, 1)
            and pc.cin == pc.cout and pc.cin in (256, 512) and pc.Kpad == 9 * pc.cin and not pc.n_split)


def cs3_forward(x: torch.Tensor, pc: "PackedConv", out: torch.Tensor, relu: int = 1, stream=None) -> torch.Tensor:
    if not cs3_supported(pc):
        raise ValueError("cs3 conv: needs a 3x3 / s1 / p1 conv 256 -> 256 or 512 -> 512")
    if x.dim() != 4 or (x.shape[3], x.shape[1], x.shape[2]) not in CS3_SHAPES or x.shape[3] != pc.cin \
            or tuple(out.shape) != tuple(x.shape):
        raise ValueError(f"cs3 conv: x {tuple(x.shape)} out {tuple(out.shape)} (needs B x 14 x 14 x 256 or B x 7 x 7 x 512)")
    for t in (x, out):
        if t.dtype != torch.bfloat16 or not t.is_contiguous():
            raise ValueError("cs3 conv: contiguous bf16 NHWC tensors")
    B, H, W, C = (int(v) for v in x.shape)
    kernels().conv3x3_cs_forward(ptr(x), ptr(pw_fragments(pc)), ptr(pc.bias), ptr(out), B, H, W, C, int(relu),
                                 stream_handle(stream))
    return out


# ------------------------------------------------------- fused bottleneck
# One launch per ResNet bottleneck block of stage 2 (csrc/kernels/bottleneck.hip):
# 1x1 (CIN -> 64) -> 3x3 (64 -> 64) -> 1x1 (64 -> 256) + identity / projection
# shortcut, BN folded, over 8x8 output tiles held in LDS.
def pack_fragments(bm: np.ndarray) -> np.ndarray:
    """[N][K] fp32 -> bf16-ready fp32 array in MFMA 16x16x32 B-fragment order:
    (n-frag, k-step, lane = (k-chunk << 4) | row, 8 k values), so each wave
    loads one fragment as a single coalesced 1 KiB read."""
    N, K = bm.shape
    if N % 16 or K % 32:
        raise ValueError(f"fragment packing needs N % 16 == 0 and K % 32 == 0, got {bm.shape}")
    return np.ascontiguousarray(bm.reshape(N // 16, 16, K // 32, 4, 8).transpose(0, 2, 3, 1, 4)).reshape(-1)


@dataclass
class PackedBottleneck:
    w1: torch.Tensor
    w2: torch.Tensor
    w3: torch.Tensor
    b1: torch.Tensor
    b2: torch.Tensor
    b3: torch.Tensor
    cin: int
    proj: bool


def pack_bottleneck(k1, b1, k2, b2, k3, b3, kp=None, bp=None, device="cuda") -> PackedBottleneck:
    """HWIO kernels (BN folded) of the three convs [+ the projection shortcut]."""
    cin = k1.shape[2]
    if k1.shape[:2] != (1, 1) or k1.shape[3] != 64 or k2.shape != (3, 3, 64, 64) or k3.shape != (1, 1, 64, 256):
        raise ValueError("fused bottleneck: expects 1x1 CIN->64, 3x3 64->64, 1x1 64->256")
    if (kp is None) != (cin == 256) or (kp is not None and kp.shape != (1, 1, 64, 256)):
        raise ValueError("fused bottleneck: identity needs CIN 256, projection needs CIN 64 and a 64->256 1x1")
    w3 = k3[0, 0].T                                       # [256][64]
    bias3 = np.asarray(b3, np.float64)
    if kp is not None:
        w3 = np.concatenate([w3, kp[0, 0].T], axis=1)     # K = [y2 | x]: the projection rides the last GEMM
        bias3 = bias3 + np.asarray(bp, np.float64)

    def dev(a, dt=torch.bfloat16):
        return torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(device=device, dtype=dt).contiguous()
    return PackedBottleneck(
        w1=dev(pack_fragments(k1[0, 0].T)), w2=dev(pack_fragments(k2.transpose(3, 0, 1, 2).reshape(64, 576))),
        w3=dev(pack_fragments(w3)), b1=dev(b1, torch.float32), b2=dev(b2, torch.float32),
        b3=dev(bias3, torch.float32), cin=cin, proj=kp is not None)


def bottleneck_forward(x: torch.Tensor, pb: PackedBottleneck, out: torch.Tensor, stream=None) -> torch.Tensor:
    if x.dtype != torch.bfloat16 or out.dtype != torch.bfloat16 or not x.is_contiguous() or not out.is_contiguous():
        raise ValueError("fused bottleneck: contiguous bf16 NHWC in and out")
    B, H, W, C = x.shape
    if C != pb.cin or H % 8 or W % 8:
        raise ValueError(f"fused bottleneck: input {tuple(x.shape)} (needs {pb.cin} channels, H, W multiples of 8)")
    if tuple(out.shape) != (B, H, W, 256):
        raise ValueError(f"fused bottleneck: output {tuple(out.shape)} != {(B, H, W, 256)}")
    kernels().bottleneck_forward(ptr(x), ptr(pb.w1), ptr(pb.w2), ptr(pb.w3), ptr(pb.b1), ptr(pb.b2), ptr(pb.b3),
                                 ptr(out), B, H, W, pb.cin, bool(pb.proj), stream_handle(stream))
    return out


# ------------------------------------------------------- fused 1x1 pair
# `_out` of block k (1x1 CIN -> CO + BN + residual + ReLU) and `_1` of block k+1
# (1x1 CO -> CM + BN + ReLU) in one launch (csrc/kernels/pw_pair.hip): y stays
# in LDS for the second GEMM and is written once, as the next residual.
PAIR_BM = {128: 16}                   # pixels per tile of the persistent kernel, by CIN (ResNet stage 3)
# (CIN, CO, CM, BM) instances (must match ADAPT_PAIR_CFGS in pw_pair.hip)
PAIR_CFGS = {(128, 512, 128, 16)}


@dataclass
class PackedPair:
    w3: torch.Tensor
    b3: torch.Tensor
    w1: torch.Tensor
    b1: torch.Tensor
    cin: int
    co: int
    cm: int
    bm: int = 0               # pixels per workgroup, fixed when packed (ADAPT_PAIR_BM overrides the table)


def pair_bm(cin: int) -> int:
    """Pixels per workgroup for a pair with CIN input channels; ADAPT_PAIR_BM="128:32,256:16"
    overrides the table per CIN (0 disables the fusion for that CIN)."""
    table = dict(PAIR_BM)
    for kv in os.environ.get("ADAPT_PAIR_BM", "").split(","):
        if ":" in kv:
            c, b = kv.split(":")
            table[int(c)] = int(b)
    return table.get(cin, 0)


def pair_supported(cin: int, co: int, cm: int, bm: Optional[int] = None) -> bool:
    bm = pair_bm(cin) if bm is None else bm
    return (cin, co, cm, bm) in PAIR_CFGS


def pack_pair(k3, b3, k1, b1, device="cuda") -> PackedPair:
    """HWIO kernels (BN folded) of the two 1x1 convs."""
    if k3.shape[:2] != (1, 1) or k1.shape[:2] != (1, 1) or k1.shape[2] != k3.shape[3]:
        raise ValueError(f"fused 1x1 pair: shapes {k3.shape} -> {k1.shape}")

    def dev(a, dt=torch.bfloat16):
        return torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(device=device, dtype=dt).contiguous()
    return PackedPair(w3=dev(pack_fragments(k3[0, 0].T)), b3=dev(b3, torch.float32),
                      w1=dev(pack_fragments(k1[0, 0].T)), b1=dev(b1, torch.float32),
                      cin=k3.shape[2], co=k3.shape[3], cm=k1.shape[3], bm=pair_bm(k3.shape[2]))


# fp32 fused 1x1 pair (csrc/kernels/pw_pair_f32.hip): ResNet stage 2 only (64 -> 256 -> 64); the
# weights of wider pairs do not fit one block's registers at fp32
PAIR_F32_SHAPES = frozenset({(64, 256, 64)})
PAIR_F32_BM = (16, 32)


def pair_f32_supported(cin: int, co: int, cm: int) -> bool:
    return (cin, co, cm) in PAIR_F32_SHAPES


def pair_f32_bm() -> int:
    bm = int(os.environ.get("ADAPT_PAIR_F32_BM", "16"))   # A/B: 16 beats 32 by ~4 us per forward (profiles/r3/r3v)
    if bm not in PAIR_F32_BM:
        raise ValueError(f"ADAPT_PAIR_F32_BM must be one of {PAIR_F32_BM}")
    return bm


def pack_pair_f32(k3, b3, k1, b1, device="cuda") -> PackedPair:
    """HWIO kernels (BN folded, fp64 / fp32) of the two 1x1 convs, packed in the fragment order
    pw_pair_f32.hip keeps in registers: W3 [16 channel frags][4 k halves][64 lanes][4] with lane
    16q + r holding W3[16h + 4q + s][16 cf + r]; W1 [2 K halves x 4 channel frags][8 halves][64][4]
    holding W1[128 kh + 16h + 4q + s][16 c2 + r] (wave = 4 kh + c2)."""
    if k3.shape[:2] != (1, 1) or k1.shape[:2] != (1, 1) or k1.shape[2] != k3.shape[3]:
        raise ValueError(f"fused 1x1 pair: shapes {k3.shape} -> {k1.shape}")
    cin, co, cm = k3.shape[2], k3.shape[3], k1.shape[3]
    if not pair_f32_supported(cin, co, cm):
        raise ValueError(f"fp32 fused 1x1 pair: no kernel for {cin}->{co}->{cm}")
    w3 = np.asarray(k3[0, 0], np.float64).reshape(4, 4, 4, 16, 16)          # h, q, s, cf, r
    w3 = w3.transpose(3, 0, 1, 4, 2).reshape(16, 4, 64, 4)
    w1 = np.asarray(k1[0, 0], np.float64).reshape(2, 8, 4, 4, 4, 16)        # kh, h, q, s, c2, r
    w1 = w1.transpose(0, 4, 1, 2, 5, 3).reshape(8, 8, 64, 4)

    def dev(a):
        return torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(device=device).contiguous()
    return PackedPair(w3=dev(w3), b3=dev(b3), w1=dev(w1), b1=dev(b1), cin=cin, co=co, cm=cm, bm=pair_f32_bm())


def pair_f32_forward(x: torch.Tensor, res: torch.Tensor, pp: PackedPair, y: torch.Tensor, z: torch.Tensor,
                     bm: Optional[int] = None, grid: int = 0, stream=None):
    """y = relu(x . W3 + b3 + res), z = relu(y . W1 + b1) in one fp32 launch (pw_pair_f32.hip)."""
    bm = (pp.bm or pair_f32_bm()) if bm is None else bm
    for t in (x, res, y, z):
        if t.dtype != torch.float32 or not t.is_contiguous() or t.device != x.device:
            raise ValueError("fp32 fused 1x1 pair: contiguous fp32 tensors on one device")
    M = x.numel() // pp.cin
    if x.shape[-1] != pp.cin or res.numel() != M * pp.co or y.numel() != M * pp.co or z.numel() != M * pp.cm:
        raise ValueError(f"fp32 fused 1x1 pair: x {tuple(x.shape)} res {tuple(res.shape)} y {tuple(y.shape)} "
                         f"z {tuple(z.shape)} for {pp.cin}->{pp.co}->{pp.cm}")
    if not kernels().pw_pair_f32_supported(pp.cin, pp.co, pp.cm, bm):
        raise ValueError(f"fp32 fused 1x1 pair: no kernel for {pp.cin}->{pp.co}->{pp.cm} at {bm} pixels per tile")
    kernels().pw_pair_f32_forward(ptr(x), ptr(pp.w3), ptr(pp.b3), ptr(res), ptr(pp.w1), ptr(pp.b1), ptr(y), ptr(z),
                                  M, pp.cin, pp.co, pp.cm, bm, int(grid), stream_handle(stream))
    return y, z


def pair_forward(x: torch.Tensor, res: torch.Tensor, pp: PackedPair, y: torch.Tensor, z: torch.Tensor,
                 bm: Optional[int] = None, stream=None):
    bm = (pp.bm or pair_bm(pp.cin)) if bm is None else bm
    for t in (x, res, y, z):
        if t.dtype != torch.bfloat16 or not t.is_contiguous() or t.device != x.device:
            raise ValueError("fused 1x1 pair: contiguous bf16 tensors on one device")
    M = x.numel() // pp.cin
    if x.shape[-1] != pp.cin or res.numel() != M * pp.co or y.numel() != M * pp.co or z.numel() != M * pp.cm:
        raise ValueError(f"fused 1x1 pair: x {tuple(x.shape)} res {tuple(res.shape)} y {tuple(y.shape)} "
                         f"z {tuple(z.shape)} for {pp.cin}->{pp.co}->{pp.cm}")
    if not pair_supported(pp.cin, pp.co, pp.cm, bm):
        raise ValueError(f"fused 1x1 pair: no kernel for {pp.cin}->{pp.co}->{pp.cm} at {bm} pixels per block")
    kernels().pw_pair_forward(ptr(x), ptr(pp.w3), ptr(pp.b3), ptr(res), ptr(pp.w1), ptr(pp.b1), ptr(y), ptr(z),
                              M, pp.cin, pp.co, pp.cm, bm, stream_handle(stream))
    return y, z
