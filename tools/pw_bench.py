"""Persistent pointwise conv (pw_wide.hip) vs the implicit-GEMM configs on the
ResNet stage-3 "_out" shape (M = 25088, 128 -> 512, + residual, ReLU): device
time per launch from hipGraphs of 20 launches, all variants interleaved.

    python tools/pw_bench.py [--M 25088] [--json out.json]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops import conv as C  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=25088)
    ap.add_argument("--K", type=int, default=128)
    ap.add_argument("--N", type=int, default=512)
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    rng = np.random.default_rng(0)
    kern = (rng.standard_normal((1, 1, a.K, a.N)) / np.sqrt(a.K)).astype(np.float32)
    pc = C.pack_conv(kern, rng.standard_normal(a.N).astype(np.float32), 1, ((0, 0), (0, 0)), "cuda")
    x = torch.randn((1, 1, a.M, a.K), device="cuda").to(torch.bfloat16)
    r = torch.randn((1, 1, a.M, a.N), device="cuda").to(torch.bfloat16)
    out = torch.empty_like(r)
    variants = {}
    for cfg in (3, 8, 10, 12, 27, 32, 34):
        if C.cfg_supported(cfg, pc, True):
            variants[f"igemm cfg {cfg}"] = (lambda c=cfg: C.conv_forward(x, pc, out, r, relu=1, cfg=c))
    for cfg, pt in C.PW_CFGS.items():
        tiles = (a.M + pt - 1) // pt
        for blocks in sorted({196, 224, 256, 392, 512}):
            if blocks <= tiles:
                variants[f"pw PT={pt} blocks={blocks}"] = (
                    lambda c=cfg, b=blocks: C.pw_forward(x.view(a.M, a.K), pc, out.view(a.M, a.N), r.view(a.M, a.N),
                                                         relu=1, cfg=c, blocks=b))
    graphs = {}
    s = torch.cuda.Stream()
    for name, fn in variants.items():
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(20):
                fn()
        graphs[name] = g
    res = {n: [] for n in graphs}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(a.rounds):
        for n, g in graphs.items():
            g.replay()
            e0.record()
            g.replay()
            e1.record()
            e1.synchronize()
            res[n].append(e0.elapsed_time(e1) * 1e3 / 20)
    gb = (a.M * a.K + 2 * a.M * a.N) * 2 / 1e9
    out_rows = []
    for n, v in sorted(res.items(), key=lambda kv: statistics.median(kv[1])):
        us = statistics.median(v)
        out_rows.append({"variant": n, "us": round(us, 2), "TB_s": round(gb / us * 1e3, 2)})
        print(f"{n:28s} {us:7.2f} us  {gb / us * 1e3:5.2f} TB/s")
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"M": a.M, "K": a.K, "N": a.N, "rows": out_rows}, f, indent=1)


if __name__ == "__main__":
    main()
