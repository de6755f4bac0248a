#!/usr/bin/env python3
"""Time the fused 1x1 pair kernel (csrc/kernels/pw_pair.hip) on ResNet-50 stage 3
(M = 32*28*28, 128 -> 512 -> 128) against the two tuned unfused convs, each as
20 launches in one hipGraph.  --only-pair: just the fused kernel (for PMC runs)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops import conv as C  # noqa: E402


def gtime(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / (5 * reps) * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bm", default="16")
    ap.add_argument("--only-pair", action="store_true")
    a = ap.parse_args()
    M, cin, co, cm = 32 * 28 * 28, 128, 512, 128
    rng = np.random.default_rng(0)
    k3 = (rng.standard_normal((1, 1, cin, co)) / cin ** 0.5).astype(np.float32)
    k1 = (rng.standard_normal((1, 1, co, cm)) / co ** 0.5).astype(np.float32)
    b3, b1 = np.zeros(co, np.float32), np.zeros(cm, np.float32)
    x = torch.randn(M, cin, device="cuda").to(torch.bfloat16)
    res = torch.randn(M, co, device="cuda").to(torch.bfloat16)
    y = torch.empty(M, co, device="cuda", dtype=torch.bfloat16)
    z = torch.empty(M, cm, device="cuda", dtype=torch.bfloat16)
    for bm in (int(b) for b in a.bm.split(",")):
        os.environ["ADAPT_PAIR_BM"] = f"128:{bm}"
        pp = C.pack_pair(k3, b3, k1, b1, device="cuda")
        t = gtime(lambda: C.pair_forward(x, res, pp, y, z))
        print(f"pair BM {bm:3d}: {t:7.2f} us  ({(x.numel() + res.numel() + y.numel() + z.numel()) * 2 / t / 1e6:.2f} TB/s)")
    if a.only_pair:
        return
    p3 = C.pack_conv(k3, b3, 1, ((0, 0), (0, 0)), "cuda")
    p1 = C.pack_conv(k1, b1, 1, ((0, 0), (0, 0)), "cuda")
    x4, r4 = x.view(32, 28, 28, cin), res.view(32, 28, 28, co)
    y4, z4 = y.view(32, 28, 28, co), z.view(32, 28, 28, cm)
    for cfg3 in (3, 30):
        t3 = gtime(lambda: C.conv_forward(x4, p3, y4, residual=r4, relu=True, cfg=cfg3))
        print(f"unfused _out cfg {cfg3}: {t3:7.2f} us")
    for cfg1 in (22, 54):
        t1 = gtime(lambda: C.conv_forward(y4, p1, z4, relu=True, cfg=cfg1))
        print(f"unfused _1 cfg {cfg1}: {t1:7.2f} us")


if __name__ == "__main__":
    main()
