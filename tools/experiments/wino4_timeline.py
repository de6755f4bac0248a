#!/usr/bin/env python3
"""Per-wave phase timelines of the Winograd F(4x4, 3x3) kernel (csrc/kernels/conv_wino4_f32.hip, cfg 200)
on the ResNet-50 bs=32 3x3 shapes: each wave stamps the shader clock at start, after its DMA table,
after the first patch is transformed (prologue), after the K loop, after its partial outputs are staged,
and after the stores, plus the 100 MHz wall clock at start / end (one launch, whole K).

    python tools/wino4_timeline.py [--json out.json] [--exp 0,1,2,4,8]

--exp runs the kernel's measurement variants (conv_wino4_f32.hip EXP: 1 no weight DMA in the K loop, 2 no
image DMA, 4 no input transform, 8 the spread schedule, sums combine) on the shapes whose image fits 15-16
pieces; their outputs are wrong by design, only their clocks are read.
"""
import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops import conv as C  # noqa: E402

SHAPES = [(32, 56, 56, 64, 64, 1), (32, 28, 28, 128, 128, 1), (32, 14, 14, 256, 256, 2), (32, 7, 7, 512, 512, 4)]
PHASES = ["table", "prologue", "loop", "out_transform", "stores"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default="")
    ap.add_argument("--exp", default="0")
    ap.add_argument("--cfg", type=int, default=200)
    a = ap.parse_args()
    if a.cfg == 210:
        return main_pc(a)
    K = C.kernels()
    rows = []
    exps = [int(e) for e in a.exp.split(",")]
    for (B, H, W, Cin, Cout, ks), exp in [(s, e) for s in SHAPES for e in exps]:
        if exp and K.conv_wino4_pieces(B, H, W)[0] not in (15, 16):
            continue
        x = torch.randn(B, H, W, Cin, device="cuda")
        kern = (np.random.default_rng(0).standard_normal((3, 3, Cin, Cout)) / math.sqrt(9 * Cin)).astype(np.float32)
        pc = C.pack_conv_f32(kern, np.zeros(Cout, np.float32), 1, ((1, 1), (1, 1)), "cuda")
        out = torch.empty(B * H * W * Cout, device="cuda")
        blocks = C.wino4_blocks(B, H, W, Cout) * ks
        dbg = torch.zeros(blocks * 4 * 8, dtype=torch.int64, device="cuda")
        for _ in range(3):                                   # warm the weights / caches
            C.conv_forward_f32(x, pc, out, relu=1, cfg=200, ksplit=ks)
        torch.cuda.synchronize()
        K.wino4_set_debug(int(dbg.data_ptr()), exp)
        C.conv_forward_f32(x, pc, out, relu=1, cfg=200, ksplit=ks)
        torch.cuda.synchronize()
        K.wino4_set_debug(0, 0)
        d = dbg.view(-1, 8).cpu().numpy().astype(np.float64)
        ok = d[:, 7] > 0 if ks == 1 else d[:, 3] > 0
        d = d[ok]
        # shader-clock rate from the stamps of the longest-lived waves (cycles per 100 MHz tick)
        ghz = np.median((d[:, 5] - d[:, 0]) / np.maximum(d[:, 7] - d[:, 6], 1)) * 0.1 if ks == 1 else 2.1
        ph = {}
        for i, name in enumerate(PHASES):
            if ks != 1 and i == 4:
                continue
            v = (d[:, i + 1] - d[:, i]) / (ghz * 1e3)
            ph[name] = {"median_us": round(float(np.median(v)), 2), "p90_us": round(float(np.percentile(v, 90)), 2)}
        span = (d[:, 7].max() - d[:, 6].min()) / 100.0 if ks == 1 else None
        chunks = (Cin // 8) // ks
        rec = {"shape": [B, H, W, Cin, Cout], "exp": exp, "ksplit": ks, "blocks": blocks, "chunks_per_block": chunks,
               "clock_GHz": round(float(ghz), 3), "phases": ph,
               "loop_us_per_chunk": round(ph["loop"]["median_us"] / chunks, 3),
               "mfma_us_per_chunk": round(72 * 32 / (ghz * 1e3), 3), "kernel_span_us": span}
        rows.append(rec)
        print(json.dumps(rec), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


def main_pc(a):
    """cfg 210 (conv_wino4pc_f32.hip): per wave stamps start / prologue done / K loop done / epilogue done
    (+ wall clock at start and end), consumers (waves 0-3) and producers (4-7) reported apart."""
    K = C.kernels()
    rows = []
    exps = [int(e) for e in a.exp.split(",")]
    for (B, H, W, Cin, Cout, ks), exp in [(s, e) for s in SHAPES for e in exps]:
        x = torch.randn(B, H, W, Cin, device="cuda")
        kern = (np.random.default_rng(0).standard_normal((3, 3, Cin, Cout)) / math.sqrt(9 * Cin)).astype(np.float32)
        pc = C.pack_conv_f32(kern, np.zeros(Cout, np.float32), 1, ((1, 1), (1, 1)), "cuda")
        out = torch.empty(B * H * W * Cout, device="cuda")
        M = B * H * W
        nws = C.workspace_elems_f32(M, Cout, pc.Kpad, 210, ks)
        ws = torch.empty(nws, device="cuda") if nws else None
        blocks = C.wino4_blocks(B, H, W, Cout) * ks
        dbg = torch.zeros(blocks * 8 * 8, dtype=torch.int64, device="cuda")
        for _ in range(3):
            C.conv_forward_f32(x, pc, out, relu=1, cfg=210, ksplit=ks, workspace=ws)
        torch.cuda.synchronize()
        K.wino4_set_debug(int(dbg.data_ptr()), exp)
        C.conv_forward_f32(x, pc, out, relu=1, cfg=210, ksplit=ks, workspace=ws)
        torch.cuda.synchronize()
        K.wino4_set_debug(0, 0)
        d = dbg.view(blocks, 8, 8).cpu().numpy().astype(np.float64)
        d = d[:, :, [0, 1, 2, 4, 5, 3, 6, 7]]               # start, prologue, loop, E0, half 0, end
        ghz = float(np.median((d[:, :, 5] - d[:, :, 0]) / np.maximum(d[:, :, 7] - d[:, :, 6], 1)) * 0.1)
        chunks = (Cin // 8) // ks
        rec = {"shape": [B, H, W, Cin, Cout], "cfg": 210, "exp": exp, "ksplit": ks, "blocks": blocks, "chunks_per_block": chunks,
               "clock_GHz": round(ghz, 3)}
        for role, sl in (("consumer", slice(0, 4)), ("producer", slice(4, 8))):
            ph = {}
            for i, name in enumerate(("prologue", "loop", "e0_wait", "half0", "half1")):
                v = (d[:, sl, i + 1] - d[:, sl, i]).ravel() / (ghz * 1e3)
                ph[name] = {"median_us": round(float(np.median(v)), 2), "p90_us": round(float(np.percentile(v, 90)), 2)}
            rec[role] = ph
        rec["loop_us_per_chunk"] = round(rec["consumer"]["loop"]["median_us"] / chunks, 3)
        rec["mfma_us_per_chunk"] = round(72 * 32 / (ghz * 1e3), 3)
        rec["kernel_span_us"] = round(float((d[:, :, 7].max() - d[:, :, 6].min()) / 100.0), 2)
        rows.append(rec)
        print(json.dumps(rec), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
