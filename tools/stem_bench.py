"""Isolated timing of the fp32 fused stem (csrc/kernels/stem_f32.hip) at the
ResNet-50 shape: conv1 7x7/s2 3->64 + BN/ReLU + 3x3/s2 max-pool, bs=32.
Floor columns: MFMA work at the kernel's K (37 MFMAs per 16x16 tile for K=147)
and at the true K, both at the measured fp32 matrix ceiling."""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops import conv as C

PEAK_TF = 150.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--iters", type=int, default=200)
    a = ap.parse_args()
    B, H = a.batch, 224
    rng = np.random.default_rng(0)
    kern = (rng.standard_normal((7, 7, 3, 64)) / np.sqrt(147)).astype(np.float32)
    ps = C.pack_stem_f32(kern, np.zeros(64, np.float32), ((3, 3), (3, 3)), "cuda")
    x = torch.randn(B, H, H, 3, device="cuda")
    out = torch.empty(B, 56, 56, 64, device="cuda")
    res = {}
    for variant in (0, 1, 2, 5, 6):
        for _ in range(10):
            C.stem_f32_forward(x, ps, out, variant=variant)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            C.stem_f32_forward(x, ps, out, variant=variant)
        e.record()
        torch.cuda.synchronize()
        res[variant] = (s.elapsed_time(e) * 1e3 / a.iters, out.clone())
    us = res[C.STEM_F32_VARIANT][0]
    same = bool(torch.equal(res[0][1], res[1][1])) and bool(torch.allclose(res[0][1], res[2][1], rtol=1e-5, atol=1e-5))
    px = B * 112 * 112
    true_flop = 2.0 * px * 64 * 147
    kernel_flop = 2.0 * px * 64 * 148 * 15 / 14          # 37 MFMAs x K=4, one extra conv row per 7 pool rows
    rec = {"kernel": "stem_f32", "batch": B, "us": round(us, 2),
           "us_by_variant": {v: round(t, 2) for v, (t, _) in res.items()}, "variants_bitwise_equal": same,
           "floor_true_us": round(true_flop / PEAK_TF / 1e6, 1),
           "floor_kernel_us": round(kernel_flop / PEAK_TF / 1e6, 1)}
    print(json.dumps(rec))
    # bf16 stem (csrc/kernels/stem.hip): v1 one pool row per block, v2 row groups with the patch loaded a
    # step ahead, v3 row groups with the whole patch requested up front, v4 v3 with 8 waves and the pool of
    # step k-1 beside the conv of step k (ADAPT_STEM_V1 selects)
    ps16 = C.pack_stem(kern, np.zeros(64, np.float32), ((3, 3), (3, 3)), "cuda")
    o16 = torch.empty(B, 56, 56, 64, device="cuda", dtype=torch.bfloat16)
    r16 = {}
    for ver in ("1", "0", "3", "4", "6"):
        os.environ["ADAPT_STEM_V1"] = ver
        for _ in range(10):
            C.stem_forward(x, ps16, o16, pool=True)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            C.stem_forward(x, ps16, o16, pool=True)
        e.record()
        torch.cuda.synchronize()
        r16[{"1": "v1", "0": "v2", "3": "v3", "4": "v4", "6": "v6"}[ver]] = (s.elapsed_time(e) * 1e3 / a.iters, o16.clone())
    os.environ.pop("ADAPT_STEM_V1")
    print(json.dumps({"kernel": "stem_bf16", "batch": B, "us_by_version": {k: round(t, 2) for k, (t, _) in r16.items()},
                      "versions_bitwise_equal": all(torch.equal(r16["v1"][1], o[1]) for o in r16.values())}))


if __name__ == "__main__":
    main()
