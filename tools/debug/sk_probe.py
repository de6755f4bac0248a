"""Probe the stream-K Winograd launch of one cfg on one shape (prints the launch error, if any)."""
import math
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops import conv as C  # noqa: E402

B, H, W, Cin, Cout = [int(v) for v in sys.argv[1].split(",")]
kern = (np.random.default_rng(0).standard_normal((3, 3, Cin, Cout)) / math.sqrt(9 * Cin)).astype(np.float32)
pc = C.pack_conv_f32(kern, np.zeros(Cout, np.float32), 1, ((1, 1), (1, 1)), "cuda")
x = torch.randn(B, H, W, Cin, device="cuda")
out = torch.empty(B * H * W * Cout, device="cuda")
for cfg in [int(c) for c in sys.argv[2].split(",")]:
    for ks in (-101, -102):
        ctr = torch.zeros(C.wino_blocks(cfg, B, H, W, Cout), dtype=torch.int32, device="cuda")
        try:
            C.conv_forward_f32(x, pc, out, relu=1, cfg=cfg, ksplit=ks, counters=ctr)
            torch.cuda.synchronize()
            print(cfg, ks, "ok", C.wino_sk_plan(cfg, B, H, W, Cout, Cin, ks), flush=True)
        except Exception as e:  # noqa: BLE001
            print(cfg, ks, "FAIL", repr(e)[:200], C.wino_sk_plan(cfg, B, H, W, Cout, Cin, ks), flush=True)
