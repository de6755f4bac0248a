#!/usr/bin/env python3
"""Fused stem kernel (csrc/kernels/stem.hip) vs the unfused pack -> conv -> maxpool
chain on the ResNet-50 bs=32 stem, hipGraph-timed (device time only).

    python tools/stem_bench.py [--batch 32] [--only fused|unfused]
"""
import argparse
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops import conv as C  # noqa: E402
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops import eltwise as E  # noqa: E402


def graph_time(fn, reps=20, rounds=5):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(rounds):
        g.replay()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1000 / (reps * rounds)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    B, dev = a.batch, "cuda"
    x = torch.randn(B, 224, 224, 3, device=dev)
    k = (torch.randn(7, 7, 3, 64) / math.sqrt(147)).numpy()
    b = (torch.randn(64) * 0.1).numpy()
    ps = C.pack_stem(k, b, ((3, 3), (3, 3)), dev)
    pooled = torch.empty(B, 56, 56, 64, device=dev, dtype=torch.bfloat16)
    res = {}
    if a.only in ("", "fused"):
        res["fused stem auto"] = graph_time(lambda: C.stem_forward(x, ps, pooled, pool=True))
        os.environ["ADAPT_STEM_V1"] = "0"
        res["fused stem v2 (conv+pool, row groups)"] = graph_time(lambda: C.stem_forward(x, ps, pooled, pool=True))
        ref = pooled.clone()
        os.environ["ADAPT_STEM_V1"] = "1"
        res["fused stem v1 (conv+pool)"] = graph_time(lambda: C.stem_forward(x, ps, pooled, pool=True))
        del os.environ["ADAPT_STEM_V1"]
        print("v1 == v2:", bool(torch.equal(ref, pooled)))
        full = torch.empty(B, 112, 112, 64, device=dev, dtype=torch.bfloat16)
        res["fused stem (conv only)"] = graph_time(lambda: C.stem_forward(x, ps, full, pool=False))
    if a.only in ("", "unfused"):
        k8 = torch.zeros(7, 7, 8, 64)
        k8[:, :, :3] = torch.from_numpy(k)
        pc = C.pack_conv(k8.numpy(), b, 2, ((3, 3), (3, 3)), dev)
        xp = torch.empty(B, 224, 224, 8, device=dev, dtype=torch.bfloat16)
        y = torch.empty(B, 112, 112, 64, device=dev, dtype=torch.bfloat16)
        cfg, ks = C.choose_cfg(B * 112 * 112, 64, pc.Kpad)

        def chain():
            E.input_pack(x, xp)
            C.conv_forward(xp, pc, y, relu=True, cfg=1, ksplit=1)
            E.maxpool(y, pooled, 3, 2, 1, 1, True)
        res["unfused pack+conv+maxpool"] = graph_time(chain)
    for n, t in res.items():
        print(f"{n:30s} {t:8.2f} us")


if __name__ == "__main__":
    main()
