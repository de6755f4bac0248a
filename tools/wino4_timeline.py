#!/usr/bin/env python3
"""Per-wave phase timelines of the Winograd F(4x4, 3x3) kernel (csrc/kernels/conv_wino4_f32.hip, cfg 200)
on the ResNet-50 bs=32 3x3 shapes: each wave stamps the shader clock at start, after its DMA table,
after the first patch is transformed (prologue), after the K loop, after its partial outputs are staged,
and after the stores, plus the 100 MHz wall clock at start / end (one launch, whole K).

    python tools/wino4_timeline.py [--ks 1] [--json out.json]
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
    a = ap.parse_args()
    K = C.kernels()
    rows = []
    for B, H, W, Cin, Cout, ks in SHAPES:
        x = torch.randn(B, H, W, Cin, device="cuda")
        kern = (np.random.default_rng(0).standard_normal((3, 3, Cin, Cout)) / math.sqrt(9 * Cin)).astype(np.float32)
        pc = C.pack_conv_f32(kern, np.zeros(Cout, np.float32), 1, ((1, 1), (1, 1)), "cuda")
        out = torch.empty(B * H * W * Cout, device="cuda")
        blocks = C.wino4_blocks(B, H, W, Cout) * ks
        dbg = torch.zeros(blocks * 4 * 8, dtype=torch.int64, device="cuda")
        for _ in range(3):                                   # warm the weights / caches
            C.conv_forward_f32(x, pc, out, relu=1, cfg=200, ksplit=ks)
        torch.cuda.synchronize()
        K.wino4_set_debug(int(dbg.data_ptr()))
        C.conv_forward_f32(x, pc, out, relu=1, cfg=200, ksplit=ks)
        torch.cuda.synchronize()
        K.wino4_set_debug(0)
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
        rec = {"shape": [B, H, W, Cin, Cout], "ksplit": ks, "blocks": blocks, "chunks_per_block": chunks,
               "clock_GHz": round(float(ghz), 3), "phases": ph,
               "loop_us_per_chunk": round(ph["loop"]["median_us"] / chunks, 3),
               "mfma_us_per_chunk": round(72 * 32 / (ghz * 1e3), 3), "kernel_span_us": span}
        rows.append(rec)
        print(json.dumps(rec), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
