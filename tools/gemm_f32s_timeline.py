#!/usr/bin/env python3
"""Per-wave timelines of the fp32 big-tile 1x1 GEMM (csrc/kernels/gemm_f32s.hip, whole-K tiles): shader clock at
start, first chunk landed, K loop done, epilogue stores acknowledged; per-chunk loop time against the MFMA floor;
measurement variants (--exp 1: no LDS-DMA in the loop, 2: no MFMAs).

    python tools/gemm_f32s_timeline.py [--exp 0,1,2] [--json out.json]
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

CASES = [(32, 28, 28, 512, 128, 302), (32, 7, 7, 512, 2048, 302), (32, 14, 14, 256, 1024, 300),
         (32, 28, 28, 128, 512, 300)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--exp", default="0,1,2")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    K = C.kernels()
    rows = []
    for (B, H, W, Cin, Cout, cfg), exp in [(c, int(e)) for c in CASES for e in a.exp.split(",")]:
        x = torch.randn(B, H, W, Cin, device="cuda")
        kern = (np.random.default_rng(0).standard_normal((1, 1, Cin, Cout)) / math.sqrt(Cin)).astype(np.float32)
        pc = C.pack_conv_f32(kern, np.zeros(Cout, np.float32), 1, ((0, 0), (0, 0)), "cuda")
        out = torch.empty(B * H * W * Cout, device="cuda")
        M = B * H * W
        tiles = C.f32s_tiles(cfg, M, Cout)
        dbg = torch.zeros(tiles * 4 * 8, dtype=torch.int64, device="cuda")
        for _ in range(3):
            C.conv_forward_f32(x, pc, out, relu=1, cfg=cfg, ksplit=1)
        torch.cuda.synchronize()
        K.gemm_f32s_set_debug(int(dbg.data_ptr()), exp)
        C.conv_forward_f32(x, pc, out, relu=1, cfg=cfg, ksplit=1)
        torch.cuda.synchronize()
        K.gemm_f32s_set_debug(0, 0)
        d = dbg.view(tiles * 4, 8).cpu().numpy().astype(np.float64)
        ghz = float(np.median((d[:, 3] - d[:, 0]) / np.maximum(d[:, 7] - d[:, 6], 1)) * 0.1)
        chunks = Cin // 32
        bm, bn = C.F32S_CFGS[cfg]
        mfma_chunk = (bm // 16) * (bn // 64) * 8 * 32          # cycles of MFMA per chunk per wave
        ph = {}
        for i, name in enumerate(("first_chunk", "loop", "epilogue")):
            v = (d[:, i + 1] - d[:, i]) / (ghz * 1e3)
            ph[name] = {"median_us": round(float(np.median(v)), 2), "p90_us": round(float(np.percentile(v, 90)), 2)}
        rec = {"shape": [B, H, W, Cin, Cout], "cfg": cfg, "exp": exp, "tiles": tiles, "chunks": chunks,
               "clock_GHz": round(ghz, 3), "phases": ph,
               "loop_us_per_chunk": round(ph["loop"]["median_us"] / max(chunks - 1, 1), 3),
               "mfma_us_per_chunk": round(mfma_chunk / (ghz * 1e3), 3),
               "span_us": round(float((d[:, 7].max() - d[:, 6].min()) / 100.0), 2)}
        rows.append(rec)
        print(json.dumps(rec), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
