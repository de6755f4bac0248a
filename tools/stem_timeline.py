#!/usr/bin/env python3
"""Per-wave timelines of the v4 pooled bf16 stem (csrc/kernels/stem.hip stem_pool_v4_kernel) at ResNet-50
bs=32: shader clock at start, patch rows 0-10 in LDS, step 0 (3 conv rows) done, the pipelined steps done,
the last pool row's stores acknowledged; wall-clock span of the launch.

    python tools/stem_timeline.py [--batch 32] [--json out.json]
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

WAVES = 8
SP = 7                                                     # pool rows per block (S4_SP)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--json", default="")
    ap.add_argument("--version", default="6", choices=["4", "6"],
                    help="ADAPT_STEM_V1 (v6: v4 + block-staged weights; the v5 / v7 channel-half variants and the "
                    "ablation builds are retired, profiles/r5/stem_bf16_v4.md holds their timelines)")
    ap.add_argument("--exp", default="0", help="0 only (the ablation builds are no longer compiled)")
    a = ap.parse_args()
    K = C.kernels()
    B = a.batch
    rng = np.random.default_rng(0)
    kern = (rng.standard_normal((7, 7, 3, 64)) / math.sqrt(147)).astype(np.float32)
    ps = C.pack_stem(kern, np.zeros(64, np.float32), ((3, 3), (3, 3)), "cuda")
    x = torch.randn(B, 224, 224, 3, device="cuda")
    out = torch.empty(B, 56, 56, 64, device="cuda", dtype=torch.bfloat16)
    os.environ["ADAPT_STEM_V1"] = a.version
    if a.version != "4" and a.exp != "0":
        ap.error("the --exp variants are built for v4 only")
    blocks = B * math.ceil(56 / SP)
    recs = []
    for exp in [int(e) for e in a.exp.split(",")]:
        dbg = torch.zeros(blocks * WAVES * 8, dtype=torch.int64, device="cuda")
        for _ in range(3):
            C.stem_forward(x, ps, out, pool=True)
        torch.cuda.synchronize()
        K.stem_set_debug(int(dbg.data_ptr()), exp)
        C.stem_forward(x, ps, out, pool=True)
        torch.cuda.synchronize()
        K.stem_set_debug(0, 0)
        d = dbg.view(blocks * WAVES, 8).cpu().numpy().astype(np.float64)
        ghz = float(np.median((d[:, 4] - d[:, 0]) / np.maximum(d[:, 7] - d[:, 6], 1)) * 0.1)
        ph = {}
        for i, name in enumerate(("patch_rows_0_10", "step0", "steps", "last_pool_stores")):
            v = (d[:, i + 1] - d[:, i]) / (ghz * 1e3)
            ph[name] = {"median_us": round(float(np.median(v)), 2), "p90_us": round(float(np.percentile(v, 90)), 2),
                        "max_us": round(float(v.max()), 2)}
        start = (d[:, 6] - d[:, 6].min()) / 100.0
        rec = {"kernel": f"stem_pool v{a.version}", "exp": exp, "batch": B, "blocks": blocks, "clock_GHz": round(ghz, 3),
               "phases": ph,
               "block_start_us": {"median": round(float(np.median(start)), 2), "max": round(float(start.max()), 2)},
               "wave_total_us_median": round(float(np.median((d[:, 4] - d[:, 0]) / (ghz * 1e3))), 2),
               "span_us": round(float((d[:, 7].max() - d[:, 6].min()) / 100.0), 2)}
        print(json.dumps(rec), flush=True)
        recs.append(rec)
    rec = recs if len(recs) > 1 else recs[0]
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rec, f, indent=1)


if __name__ == "__main__":
    main()
