#!/usr/bin/env python3
"""Isolated timing of the fp32 3x3 paths on the ResNet-50 bs=32 shapes: the tuned config of the plan
(tuning table) against every Winograd F(4x4) split config (csrc/kernels/wino4s_f32.hip) and split-K.
Each candidate runs 20 launches captured in one hipGraph (device time per launch).

    python tools/wino4s_bench.py [--json out.json]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

import torch  # noqa: E402

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops import conv as C_  # noqa: E402
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.runtime.executor import (  # noqa: E402
    SliceExecutor, conv_key, load_tuning)

SHAPES = [(32, 56, 64), (32, 28, 128), (32, 14, 256), (32, 7, 512)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default="")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--cfgs", default="")
    ap.add_argument("--ks", default="", help="comma list of split-K factors (default: all valid)")
    ap.add_argument("--shapes", default="", help="comma list of H (56, 28, 14, 7)")
    ap.add_argument("--no-tuned", action="store_true")
    a = ap.parse_args()
    table = load_tuning()
    cfgs = [int(c) for c in a.cfgs.split(",") if c] or sorted(C_.WINO4S_F32_CFGS)
    res = []
    shapes = [sh for sh in SHAPES if not a.shapes or str(sh[1]) in a.shapes.split(",")]
    kss = [int(k) for k in a.ks.split(",") if k]
    for (B, H, C) in shapes:
        x = torch.randn((B, H, H, C), device="cuda")
        k = torch.randn((3, 3, C, C)) / (3.0 * C ** 0.5)
        pc = C_.pack_conv_f32(k.numpy(), torch.zeros(C).numpy(), 1, ((1, 1), (1, 1)), "cuda")
        out = torch.empty((B, H, H, C), device="cuda")
        key = "f32|" + conv_key(B, H, H, C, pc)
        tuned = tuple(table[key][:2]) if key in table else None
        ws = torch.empty(1 << 26, dtype=torch.float32, device="cuda")
        ctr = torch.zeros(1 << 16, dtype=torch.int32, device="cuda")
        row = {"shape": f"{B}x{H}x{H}x{C}", "tuned": tuned}
        if tuned and not a.no_tuned:
            cfg, ks = tuned
            row["tuned_us"] = 1e3 * SliceExecutor._time_graph(
                lambda: C_.conv_forward_f32(x, pc, out, relu=1, cfg=cfg, ksplit=ks, workspace=ws, counters=ctr),
                a.reps)
        best = None
        for cfg in cfgs:
            for ks in C_.wino4s_splits(C) + [-k for k in C_.wino4s_splits(C) if k > 1]:
                if (kss and ks not in kss) or not C_.kernels().wino4s_ok(cfg, C, C, ks):
                    continue
                need = C_.wino4s_ws_elems(B, H, H, C, C, ks)
                w2 = ws if ws.numel() >= need else torch.empty(need, dtype=torch.float32, device="cuda")
                us = 1e3 * SliceExecutor._time_graph(
                    lambda: C_.conv_forward_f32(x, pc, out, relu=1, cfg=cfg, ksplit=ks, workspace=w2, counters=ctr),
                    a.reps)
                row[f"{cfg}/{ks}"] = round(us, 2)
                if best is None or us < best[0]:
                    best = (us, cfg, ks)
        row["best"] = best
        print(json.dumps(row), flush=True)
        res.append(row)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
