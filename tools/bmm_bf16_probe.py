#!/usr/bin/env python3
"""Batched bf16 GEMM speed for a Winograd F(2x2, 3x3) formulation of the bf16 stage-4 / stage-5 3x3s:
16 positions x (tiles x Cin) @ (Cin x Cout), graph-replayed (torch.bmm -> hipBLASLt)."""
import json

import torch


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


for P, T, C, N in [(16, 512, 512, 512), (16, 1568, 256, 256), (16, 6272, 128, 128), (36, 128, 512, 512),
                   (36, 512, 256, 256)]:
    a = torch.randn(P, T, C, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(P, C, N, device="cuda", dtype=torch.bfloat16)
    o = torch.empty(P, T, N, device="cuda", dtype=torch.bfloat16)
    o32 = torch.empty(P, T, N, device="cuda", dtype=torch.float32)
    t = gtime(lambda: torch.bmm(a, b, out=o))
    fl = 2.0 * P * T * C * N
    rec = {"P": P, "T": T, "C": C, "N": N, "bmm_bf16_out_us": round(t, 2), "TFs": round(fl / t / 1e6, 1)}
    try:
        t2 = gtime(lambda: torch.matmul(a, b, out=o32) if False else torch.bmm(a.float(), b.float(), out=o32))
        rec["bmm_fp32_us"] = round(t2, 2)
    except Exception as e:  # noqa: BLE001
        rec["fp32_err"] = str(e)[:80]
    print(json.dumps(rec), flush=True)
