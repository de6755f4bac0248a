#!/usr/bin/env python3
"""Time every (tile config, split-K) of the conv kernels on given conv
problems with hipGraph replay (device time only).

    python tools/conv_bench.py                 # the distinct ResNet-50 bs=32 problems
    python tools/conv_bench.py --shape 32,14,14,256,256,3,1,1 --only 6,10
"""
import argparse
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops import conv as C  # noqa: E402

R50 = [  # B, H, W, Cin, Cout, k, stride, pad, residual
    (32, 56, 56, 64, 64, 3, 1, 1, 0),
    (32, 28, 28, 128, 128, 3, 1, 1, 0),
    (32, 14, 14, 256, 256, 3, 1, 1, 0),
    (32, 7, 7, 512, 512, 3, 1, 1, 0),
    (32, 56, 56, 64, 256, 1, 1, 0, 1),
    (32, 56, 56, 256, 64, 1, 1, 0, 0),
    (32, 28, 28, 512, 128, 1, 1, 0, 0),
    (32, 14, 14, 256, 1024, 1, 1, 0, 1),
    (32, 7, 7, 2048, 512, 1, 1, 0, 0),
]


def bench(shape, only=None, reps=20, ks_list=(1, 2, 3, 4, 6, 8, -1, -2)):
    B, H, W, Cin, Cout, k, s, p, has_res = shape
    dev = "cuda"
    x = torch.randn(B, H, W, Cin, device=dev).to(torch.bfloat16)
    kern = (torch.randn(k, k, Cin, Cout) / math.sqrt(k * k * Cin)).numpy()
    pc = C.pack_conv(kern, torch.zeros(Cout).numpy(), s, ((p, p), (p, p)), dev)
    OH, OW = pc.out_hw(H, W)
    M, N = B * OH * OW, Cout
    out = torch.empty(M * N, device=dev, dtype=torch.bfloat16)
    res = torch.randn(M * N, device=dev).to(torch.bfloat16) if has_res else None
    flop = 2.0 * M * N * pc.K
    byts = (x.numel() + M * N * (2 if has_res else 1)) * 2 + pc.w.numel() * 2
    rows = []
    pure = k == 1 and s == 1 and p == 0
    for cfg in (only or C.CFG_TILES):
        if not C.cfg_supported(cfg, pc, pure):
            continue
        for ks in ks_list:
            if ks > 1 and pc.Kpad // 64 // ks < 2:
                continue
            if ks < 0 and cfg in C.V1_CFGS:
                continue
            if ks != 1 and cfg not in C.CFG_TILES:      # register-resident / persistent kernels: whole K only
                continue
            need = C.workspace_elems(M, N, pc.Kpad, cfg, ks) if cfg in C.CFG_TILES else 0
            ws = torch.empty(need, device=dev, dtype=torch.float32) if need else None
            ctr = torch.zeros(C.sk_plan(M, N, pc.Kpad, cfg, -ks)[0], device=dev, dtype=torch.int32) if ks < 0 else None
            try:
                C.conv_forward(x, pc, out, residual=res, relu=True, cfg=cfg, ksplit=ks, workspace=ws, counters=ctr)
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for _ in range(reps):
                        C.conv_forward(x, pc, out, residual=res, relu=True, cfg=cfg, ksplit=ks, workspace=ws,
                                       counters=ctr)
                g.replay()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    g.replay()
                e1.record()
                e1.synchronize()
                t = e0.elapsed_time(e1) / (5 * reps) * 1e3
            except (RuntimeError, ValueError) as e:
                print("skip", cfg, ks, e)
                continue
            bm, bn = C.CFG_TILES.get(cfg, (0, 0))
            blocks = (C.sk_plan(M, N, pc.Kpad, cfg, -ks)[1] if ks < 0 else
                      math.ceil(M / bm) * math.ceil(N / bn) * ks if bm else 0)
            rows.append((t, cfg, ks, blocks))
    rows.sort()
    print(f"\n== B{B} {H}x{W}x{Cin} -> {Cout} k{k} s{s}  M={M} N={N} K={pc.K}  "
          f"{flop / 1e9:.2f} GFLOP {byts / 1e6:.1f} MB")
    for t, cfg, ks, blocks in rows[:30]:
        print(f"  cfg {cfg:2d} {str(C.CFG_TILES.get(cfg, '-')):10s} ks {ks}  blocks {blocks:5d}  {t:7.2f} us  "
              f"{flop / t / 1e6:7.1f} TF/s  {byts / t / 1e3:6.2f} TB/s")
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", action="append", default=[])
    ap.add_argument("--only", default="")
    ap.add_argument("--ks", default="1,2,3,4,6,8,-1,-2")
    a = ap.parse_args()
    only = [int(c) for c in a.only.split(",") if c] or None
    shapes = [tuple(int(v) for v in s.split(",")) + ((0,) if len(s.split(",")) == 8 else ()) for s in a.shape] or R50
    for sh in shapes:
        bench(sh, only, ks_list=[int(k) for k in a.ks.split(",")])


if __name__ == "__main__":
    main()
