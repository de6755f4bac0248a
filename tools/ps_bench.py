#!/usr/bin/env python3
"""Channel-sliced persistent pointwise conv (pw_slice.hip, cfgs 74-79) vs the implicit-GEMM configs on the
ResNet-50 bs=32 1x1 shapes it takes: device time per launch from hipGraphs of 20 launches, all variants
interleaved, best first.

    python tools/ps_bench.py [--shape M,K,N,res ...] [--json out.json]
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

SHAPES = ["25088,128,512,1", "6272,256,1024,1", "6272,1024,256,0", "1568,512,2048,1", "25088,512,128,0", "1568,2048,512,0"]
IGEMM = (3, 20, 22, 23, 24, 54, 55, 56, 62, 63)


def bench_shape(M, K, N, has_res, rounds):
    rng = np.random.default_rng(0)
    kern = (rng.standard_normal((1, 1, K, N)) / np.sqrt(K)).astype(np.float32)
    pc = C.pack_conv(kern, rng.standard_normal(N).astype(np.float32), 1, ((0, 0), (0, 0)), "cuda")
    x = torch.randn((1, 1, M, K), device="cuda").to(torch.bfloat16)
    r = torch.randn((1, 1, M, N), device="cuda").to(torch.bfloat16) if has_res else None
    out = torch.empty((1, 1, M, N), device="cuda", dtype=torch.bfloat16)
    variants = {}
    for cfg in IGEMM:
        if C.cfg_supported(cfg, pc, True):
            for ks in (1, 2):
                need = C.workspace_elems(M, N, pc.Kpad, cfg, ks)
                ws = torch.empty(need, dtype=torch.float32, device="cuda") if need else None
                variants[f"igemm cfg {cfg} ks {ks}"] = (
                    lambda c=cfg, k=ks, w=ws: C.conv_forward(x, pc, out, r, relu=1, cfg=c, ksplit=k, workspace=w))
    for cfg in C.PS_CFGS:
        if C.ps_supported(pc, cfg):
            for blocks in (256, 512):
                variants[f"pw_slice cfg {cfg} blocks {blocks}"] = (
                    lambda c=cfg, b=blocks: C.ps_forward(x.view(M, K), pc, out.view(M, N),
                                                         None if r is None else r.view(M, N), relu=1, cfg=c, blocks=b))
    graphs = {}
    s = torch.cuda.Stream()
    for name, fn in list(variants.items()):
        try:
            fn()
            torch.cuda.synchronize()
        except (RuntimeError, ValueError):
            continue
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(20):
                fn()
        graphs[name] = g
    res = {n: [] for n in graphs}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(rounds):
        for n, g in graphs.items():
            g.replay()
            e0.record()
            g.replay()
            e1.record()
            e1.synchronize()
            res[n].append(e0.elapsed_time(e1) * 1e3 / 20)
    gb = (M * K + (2 if has_res else 1) * M * N + K * N) * 2 / 1e9
    rows = []
    print(f"== M={M} K={K} N={N} res={int(has_res)}  {gb * 1e3:.1f} MB compulsory", flush=True)
    for n, v in sorted(res.items(), key=lambda kv: statistics.median(kv[1])):
        us = statistics.median(v)
        rows.append({"variant": n, "us": round(us, 2), "TB_s": round(gb / us * 1e3, 2)})
        print(f"  {n:32s} {us:7.2f} us  {gb / us * 1e3:5.2f} TB/s", flush=True)
    return {"M": M, "K": K, "N": N, "res": has_res, "rows": rows}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", action="append")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    out = []
    for sh in a.shape or SHAPES:
        M, K, N, rr = (int(v) for v in sh.split(","))
        out.append(bench_shape(M, K, N, bool(rr), a.rounds))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
