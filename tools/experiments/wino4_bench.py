#!/usr/bin/env python3
"""F(4x4, 3x3) (cfg 200) against the tuned F(2x2, 3x3) configs on the ResNet-50 bs=32 3x3 shapes:
isolated hipGraph-replayed timings per split, plus the F(4x4) error against an fp64 oracle.

    python tools/wino4_bench.py [--reps 20]
"""
import argparse
import math
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops import conv as C  # noqa: E402

SHAPES = [(32, 56, 56, 64, 64), (32, 28, 28, 128, 128), (32, 14, 14, 256, 256), (32, 7, 7, 512, 512)]
F2 = {64: [(156, 1), (118, 1)], 128: [(156, 1), (118, 1)], 256: [(166, 1), (118, -2)], 512: [(167, -2), (118, -4)]}


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(5):
        g.replay()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / (5 * reps) * 1000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    for B, H, W, Cin, Cout in SHAPES:
        x = torch.randn(B, H, W, Cin, device="cuda")
        kern = (np.random.default_rng(0).standard_normal((3, 3, Cin, Cout)) / math.sqrt(9 * Cin)).astype(np.float32)
        pc = C.pack_conv_f32(kern, np.zeros(Cout, np.float32), 1, ((1, 1), (1, 1)), "cuda")
        out = torch.empty(B * H * W * Cout, device="cuda")
        M = B * H * W
        flop = 2.0 * M * Cout * 9 * Cin
        tiles4 = B * ((H + 3) // 4) * ((W + 3) // 4)
        f4_floor = 2.0 * tiles4 * 36 * Cin * Cout / 150e12 * 1e6
        print(f"shape {B}x{H}x{W}x{Cin}->{Cout}: pieces/align {tuple(C.kernels().conv_wino4_pieces(B, H, W))}, "
              f"F(4x4) MFMA floor {f4_floor:.1f} us at 150 TF", flush=True)
        cands = [(cfg, ks) for cfg in (200, 210) for ks in C.wino4_splits(Cin) for ks in ((ks,) if ks == 1 else (ks, -ks))]
        cands += F2[Cin]
        for cfg, ks in cands:
            nws = C.workspace_elems_f32(M, Cout, pc.Kpad, cfg, ks)
            ws = torch.empty(nws, device="cuda") if nws else None
            nctr = C.f32_counter_elems(cfg, ks, B, H, W, H, W, Cout, pc.Kpad)
            ctr = torch.zeros(nctr, device="cuda", dtype=torch.int32) if nctr else None
            try:
                us = timed(lambda: C.conv_forward_f32(x, pc, out, relu=1, cfg=cfg, ksplit=ks, workspace=ws,
                                                      counters=ctr), a.reps)
            except (RuntimeError, ValueError) as e:
                print(f"  cfg {cfg} ks {ks}: {e}")
                continue
            print(f"  cfg {cfg:3d} ks {ks:3d}: {us:7.2f} us  {flop / us / 1e6:6.1f} TF(direct-equiv)", flush=True)


if __name__ == "__main__":
    main()
