#!/usr/bin/env python3
"""Stage-2 fused bottleneck (csrc/kernels/bottleneck.hip) time vs batch size:
8x8 tiles, 49 per image, 2 workgroups per CU (512 slots).  bs=32 is 1568 tiles =
3 full rounds + 32 workgroups, so a jump between bs=31 (1519 tiles, 3 rounds)
and bs=32 measures the cost of the partial last round."""
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


rng = np.random.default_rng(0)
k1 = (rng.standard_normal((1, 1, 256, 64)) / 16).astype(np.float32)
k2 = (rng.standard_normal((3, 3, 64, 64)) / 24).astype(np.float32)
k3 = (rng.standard_normal((1, 1, 64, 256)) / 8).astype(np.float32)
z64, z256 = np.zeros(64, np.float32), np.zeros(256, np.float32)
pb = C.pack_bottleneck(k1, z64, k2, z64, k3, z256, device="cuda")
for bs in (20, 21, 26, 28, 30, 31, 32, 33, 34, 36, 42, 48):
    x = torch.randn(bs, 56, 56, 256, device="cuda").to(torch.bfloat16)
    out = torch.empty_like(x)
    t = gtime(lambda: C.bottleneck_forward(x, pb, out))
    tiles = bs * 49
    print(f"bs {bs:2d}: {tiles:5d} tiles ({tiles / 512:5.2f} rounds of 512)  {t:7.2f} us  {t / bs:6.3f} us/img", flush=True)
