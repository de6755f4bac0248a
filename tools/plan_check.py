#!/usr/bin/env python3
"""Check the pipeline planner against measurement on one MI355X.

For each stage count k: plan cuts (calibrated per-layer costs when the
calibration table has this model/batch, else the analytic model), build every
slice's executor exactly as a stage worker would, time each slice's captured
hipGraph, and report measured max-stage / ideal (ideal = sum / k).  The
planner's job is to keep that ratio near 1.

    python tools/plan_check.py --model resnet50 --batch 32 --stages 2,4,8 [--analytic] --json out.json
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.graph.planner import (  # noqa: E402
    load_calibration, plan_cuts)
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.graph.slicer import (  # noqa: E402
    partition, subgraph)
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.resnet import init_weights  # noqa: E402
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.zoo import build_model  # noqa: E402
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.runtime.executor import SliceExecutor  # noqa: E402


def time_slice(sg, w, batch, precision, reps=50):
    ex = SliceExecutor(sg, w, batch, device="cuda", num_sets=2, precision=precision)
    for n in sg.input_names:
        for j in range(2):
            b = ex.input_buf(n, j)
            b.copy_(torch.randn(b.shape, device="cuda").to(b.dtype))
    ex.capture()
    for _ in range(5):
        ex.forward(0)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(reps):
        ex.forward(i % 2)
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--stages", default="2,4,8")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--analytic", action="store_true", help="ignore the calibration table")
    ap.add_argument("--objective", default="compute", choices=["compute", "throughput"],
                    help="planner objective (compute: balance the per-stage compute this tool measures)")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    g = build_model(a.model)
    w = init_weights(g, 0)
    calibrated = (not a.analytic) and load_calibration(g, a.batch, a.dtype) is not None
    out = {"model": a.model, "batch": a.batch, "dtype": a.dtype, "calibrated": calibrated,
           "objective": a.objective, "plans": []}
    full_ms = time_slice(g, w, a.batch, a.dtype)
    out["unsliced_ms"] = full_ms
    for k in [int(v) for v in a.stages.split(",") if v]:
        cuts, est = plan_cuts(g, k, batch=a.batch, precision=a.dtype, calibrated=not a.analytic,
                              objective=a.objective)
        meas = [time_slice(subgraph(g, s), w, a.batch, a.dtype) for s in partition(g, cuts)]
        ideal = sum(meas) / k
        rec = {"stages": k, "part_at": cuts, "est_ms": [round(t * 1e3, 4) for t in est],
               "measured_ms": [round(t, 4) for t in meas], "max_over_ideal": round(max(meas) / ideal, 4),
               "max_over_unsliced_ideal": round(max(meas) / (full_ms / k), 4)}
        out["plans"].append(rec)
        print(json.dumps(rec), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
