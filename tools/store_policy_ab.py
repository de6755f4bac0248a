"""A/B the per-site output store policy (plain vs write-through `sc1`, common.h
StoreSite bits) on whole-model hipGraph replay, every policy interleaved in one
process so box-to-box variance cancels.

    python tools/store_policy_ab.py --model resnet50 --batch 32 --policies 0,5,1,4,127

Prints ms/batch per policy (median of rounds) and writes --json.
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

import torch  # noqa: E402

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.resnet import init_weights  # noqa: E402
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.zoo import build_model  # noqa: E402
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops._lib import kernels  # noqa: E402
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.runtime.executor import SliceExecutor  # noqa: E402

SITES = {1: "conv", 2: "splitk", 4: "bottleneck", 8: "stem", 16: "eltwise", 32: "layers", 64: "head"}


def name(p):
    return "+".join(v for k, v in SITES.items() if p & k) or "plain"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--policies", default="0,1,4,5,13,127")
    ap.add_argument("--rounds", type=int, default=15)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    pols = [int(p, 0) for p in a.policies.split(",")]
    g = build_model(a.model)
    ex = SliceExecutor(g, init_weights(g, 0), a.batch, precision=a.dtype)
    ex.input_buf(g.input).copy_(torch.randn((a.batch,) + tuple(g.layers[g.input].out_shape), device="cuda"))
    ex.capture()
    K = kernels()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = {p: [] for p in pols}
    for r in range(a.rounds):
        for p in (pols if r % 2 == 0 else pols[::-1]):
            K.set_store_policy(p)
            torch.cuda.synchronize()
            for _ in range(5):
                ex.forward(0)
            s.record()
            for _ in range(a.reps):
                ex.forward(0)
            e.record()
            e.synchronize()
            res[p].append(s.elapsed_time(e) / a.reps)
        print(f"round {r}: " + "  ".join(f"{p}:{res[p][-1]:.4f}" for p in pols), flush=True)
    K.set_store_policy(5)
    out = {"model": a.model, "batch": a.batch, "dtype": a.dtype,
           "policies": {str(p): {"sites": name(p), "ms_median": statistics.median(v), "ms_min": min(v)}
                        for p, v in res.items()}}
    base = statistics.median(res[pols[0]])
    for p in pols:
        m = statistics.median(res[p])
        print(f"policy {p:4d} {name(p):40s} {m:.4f} ms  ({a.batch / m * 1e3:7.0f} img/s, {100 * (m / base - 1):+.1f}%)")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
