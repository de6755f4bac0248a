#!/usr/bin/env python3
"""ResNet-50 with and without the fused stage-3 1x1 pairs on the same weights and
input: max |prob diff|, max logits rel diff, top-1 agreement, per batch size."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

import torch  # noqa: E402

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.resnet import build_resnet, init_weights  # noqa: E402
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.runtime.executor import SliceExecutor  # noqa: E402

g = build_resnet("resnet50")
w = init_weights(g, seed=0)
for bs in (4, 32):
    x = torch.randn(bs, 224, 224, 3, generator=torch.Generator().manual_seed(7)).cuda()
    res = {}
    for flag in ("0", "1"):
        os.environ["ADAPT_FUSED_PAIR"] = flag
        ex = SliceExecutor(g, w, bs, device="cuda:0", precision="bf16")
        p = ex(x).float().clone()
        res[flag] = (p, ex.logits().double().clone(), [ex.cfg.get(i) for i in sorted(ex.cfg)][:12])
    torch.cuda.synchronize()
    (p0, l0, c0), (p1, l1, c1) = res["0"], res["1"]
    print(f"bs {bs}: max|prob diff| {(p1 - p0).abs().max().item():.3e}  logits rel "
          f"{((l1 - l0).abs().max() / l0.abs().max()).item():.3e}  top1 {(p1.argmax(-1) == p0.argmax(-1)).float().mean().item():.3f}"
          f"  cfgs unpaired {c0}", flush=True)
