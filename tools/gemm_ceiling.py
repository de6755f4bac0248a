#!/usr/bin/env python3
"""Library ceiling for the ResNet-50 bs=32 conv GEMM shapes: plain
torch.matmul (hipBLASLt on ROCm) on the implicit-GEMM dims M x N x K, timed by
hipGraph replay.  A reference point for our fused implicit-GEMM kernels only.
    python tools/gemm_ceiling.py [--dtype bf16|fp32]
(fp32 runs with TF32 off: true fp32 matrix math, as the fp32 conv kernels do)."""
import argparse

import torch

SHAPES = [  # name, M, N, K
    ("s2 3x3", 100352, 64, 576), ("s3 3x3", 25088, 128, 1152), ("s4 3x3", 6272, 256, 2304),
    ("s5 3x3", 1568, 512, 4608), ("s2 1x1 64->256", 100352, 256, 64), ("s2 1x1 256->64", 100352, 64, 256),
    ("s3 1x1 512->128", 25088, 128, 512), ("s3 1x1 128->512", 25088, 512, 128),
    ("s4 1x1 256->1024", 6272, 1024, 256), ("s4 1x1 1024->256", 6272, 256, 1024),
    ("s5 1x1 2048->512", 1568, 512, 2048), ("s5 1x1 512->2048", 1568, 2048, 512),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    dt = torch.bfloat16 if ap.parse_args().dtype == "bf16" else torch.float32
    torch.backends.cuda.matmul.allow_tf32 = False
    dev = "cuda"
    shapes = SHAPES + ([("square 8192", 8192, 8192, 8192)] if dt == torch.float32 else [])
    for name, M, N, K in shapes:
        a = torch.randn(M, K, device=dev).to(dt)
        b = torch.randn(K, N, device=dev).to(dt)
        out = torch.empty(M, N, device=dev, dtype=dt)
        torch.matmul(a, b, out=out)
        torch.cuda.synchronize()
        reps = 20
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(reps):
                torch.matmul(a, b, out=out)
        g.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            g.replay()
        e1.record()
        e1.synchronize()
        us = e0.elapsed_time(e1) / (5 * reps) * 1e3
        print(f"{name:18s} M={M:6d} N={N:5d} K={K:5d}  {us:7.2f} us  {2 * M * N * K / us / 1e6:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
