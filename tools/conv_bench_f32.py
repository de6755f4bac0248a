#!/usr/bin/env python3
"""Isolated fp32 conv timings: every fp32 tile config (conv_f32.hip v1, conv_f32g.hip v2)
x split-K / stream-K for the given conv shapes, in a replayed hipGraph, with the
achieved TFLOP/s against the fp32 matrix peak (~150 TF/s measured, profiles/r3/mfma_f32_peak.txt).

    python tools/conv_bench_f32.py --shape 32,14,14,256,256,3,1,1,0 [--only 10,30] [--ks 1,-1,-2]
shape = B,H,W,Cin,Cout,k,stride,pad,has_residual
"""
import argparse
import math
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: E402

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops import conv as C  # noqa: E402


def bench(shape, only=None, ks_list=(1, 2, 4, -1, -2), reps=10, top=20):
    B, H, W, Cin, Cout, k, s, p, has_res = shape
    dev = "cuda"
    x = torch.randn(B, H, W, Cin, device=dev)
    kern = (torch.randn(k, k, Cin, Cout) / math.sqrt(k * k * Cin)).numpy()
    pc = C.pack_conv_f32(kern, torch.zeros(Cout).numpy(), s, ((p, p), (p, p)), dev)
    OH, OW = pc.out_hw(H, W)
    M, N = B * OH * OW, Cout
    out = torch.empty(M * N, device=dev)
    res = torch.randn(M * N, device=dev) if has_res else None
    flop = 2.0 * M * N * pc.K
    rows = []
    for cfg in (only or list(C.F32_TILES) + list(C.WINO_F32_CFGS)):
        if not C.f32_cfg_supported(cfg, Cin, Cout, pc):
            continue
        wino = cfg in C.WINO_F32_CFGS or cfg in C.WINO_F32_ABLATE
        for ks in ks_list:
            if wino and (ks <= C.WINO_SK_BASE) != (cfg in C.WINO_SK_CFGS):
                continue                              # stream-K twins take ksplit <= -100 only
            if cfg in C.WINO_PU_CFGS and ks != 1:
                continue                              # persistent Winograd: whole K
            if -100 < ks and abs(ks) > 1 and (wino or ks > 0) and (Cin // 16 if wino else pc.Kpad // C.F32_BK) // abs(ks) < 2:
                continue
            if ks < 0 and cfg not in C.F32G_CFGS and not (wino and ks <= -2) and not (cfg in C.F32S_CFGS and ks == -1):
                continue
            nws = C.workspace_elems_f32(M, N, pc.Kpad, cfg, ks)
            ws = torch.empty(nws, device=dev) if nws else None
            nctr = C.f32_counter_elems(cfg, ks, B, H, W, OH, OW, N, pc.Kpad)
            ctr = torch.zeros(nctr, device=dev, dtype=torch.int32) if nctr else None
            try:
                def run():
                    C.conv_forward_f32(x, pc, out, residual=res, relu=1, cfg=cfg, ksplit=ks, workspace=ws,
                                       counters=ctr)
                run()
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for _ in range(reps):
                        run()
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
            rows.append((t, cfg, ks))
    rows.sort()
    print(f"\n== fp32 B{B} {H}x{W}x{Cin} -> {Cout} k{k} s{s} res{has_res}  M={M} N={N} K={pc.K}  "
          f"{flop / 1e9:.2f} GFLOP  (floor {flop / 150e12 * 1e6:.1f} us at 150 TF/s)", flush=True)
    for t, cfg, ks in rows[:top]:
        if cfg in C.F32S_CFGS:
            kind = ("gemm_s",) + C.F32S_CFGS[cfg]
        elif cfg in C.PW_F32_CFGS:
            kind = ("pw", C.PW_F32_CFGS[cfg])
        else:
            kind = C.F32_TILES.get(cfg, ("wino",) + {**C.WINO_F32_CFGS, **C.WINO_F32_ABLATE}.get(cfg, ()))
        print(f"  cfg {cfg:2d} {str(kind):10s} ks {ks:2d}  {t:7.2f} us  {flop / t / 1e6:6.1f} TF/s", flush=True)
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", action="append", required=True)
    ap.add_argument("--only", default="")
    ap.add_argument("--ks", default="1,2,4,-1,-2")
    ap.add_argument("--top", type=int, default=20)
    a = ap.parse_args()
    only = [int(c) for c in a.only.split(",")] if a.only else None
    for sh in a.shape:
        v = [int(t) for t in sh.split(",")]
        if len(v) == 8:
            v.append(0)
        bench(v, only, ks_list=[int(k) for k in a.ks.split(",")], top=a.top)


if __name__ == "__main__":
    main()
