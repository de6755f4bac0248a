#!/usr/bin/env python3
"""How far the vendor fp32 GEMM (torch.mm -> hipBLASLt / rocBLAS on ROCm, full fp32: TF32 off) is from the
tuned 1x1 kernels on the ResNet-50 bs=32 pointwise shapes: plain GEMM time and GEMM + bias/residual/ReLU
(torch.addmm + add_ + relu_) per shape, graph-replayed."""
import json
import sys

import torch

SHAPES = [  # (M, K, N, residual)
    (25088, 128, 512, True), (25088, 512, 128, False), (6272, 256, 1024, True), (6272, 1024, 256, False),
    (1568, 512, 2048, True), (1568, 2048, 512, False), (100352, 64, 256, True), (100352, 256, 64, False)]


def gtime(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    g.replay()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (5 * reps)


def main():
    torch.backends.cuda.matmul.allow_tf32 = False
    for M, K, N, res in SHAPES:
        a = torch.randn(M, K, device="cuda")
        w = torch.randn(K, N, device="cuda") / K ** 0.5
        b = torch.randn(N, device="cuda")
        r = torch.randn(M, N, device="cuda")
        out = torch.empty(M, N, device="cuda")
        t_mm = gtime(lambda: torch.mm(a, w, out=out))
        if res:
            t_full = gtime(lambda: torch.addmm(r, a, w, out=out).add_(b).relu_())
        else:
            t_full = gtime(lambda: torch.addmm(b, a, w, out=out).relu_())
        tf = 2.0 * M * K * N / t_mm / 1e6
        print(json.dumps({"M": M, "K": K, "N": N, "res": res, "mm_us": round(t_mm, 2), "mm_TFs": round(tf, 1),
                          "fused_like_us": round(t_full, 2)}), flush=True)


if __name__ == "__main__":
    sys.exit(main())
