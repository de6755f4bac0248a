#!/usr/bin/env python3
"""fp32 (or --precision bf16) conv autotune on the GPU box: every (tile config, split-K) of the v1
(conv_f32.hip) and v2 LDS-DMA (conv_f32g.hip) kernels per conv problem of the
given models, isolated timings (SliceExecutor.autotune_f32).  Writes the chosen
entries ("f32|" keys of tuning/gfx950_conv.json) to --out so they can be merged
into the tree, and prints per-problem old -> new times.

    python tools/tune_f32.py --models resnet50 --batch 32 --out gpurun_out/x/tune_f32.json
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: E402

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.resnet import init_weights  # noqa: E402
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.zoo import build_model  # noqa: E402
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.runtime import executor as E  # noqa: E402


def graph_ms(ex, reps=20):
    ex.capture()
    ex.forward(0)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        ex.forward(0)
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="resnet50")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--out", required=True)
    ap.add_argument("--precision", default="fp32", choices=["fp32", "bf16"],
                    help="bf16: SliceExecutor.autotune (isolated timing + in-graph refinement of the best 3)")
    a = ap.parse_args()
    before = dict(E.load_tuning())
    allres = {}
    for name in a.models.split(","):
        g = build_model(name)
        w = init_weights(g, 0)
        ex = E.SliceExecutor(g, w, a.batch, device="cuda:0", precision=a.precision)
        t_old = graph_ms(ex)
        t0 = time.time()
        res = (ex.autotune_f32(persist=True, verbose=True) if a.precision == "fp32"
               else ex.autotune(persist=True, verbose=True))
        for k, v in res.items():
            old = before.get(k)
            print(f"{name} {k}: {old} -> {v}", flush=True)
        allres.update(res)
        ex2 = E.SliceExecutor(g, w, a.batch, device="cuda:0", precision=a.precision)
        t_new = graph_ms(ex2)
        print(json.dumps({"model": name, "batch": a.batch, "graph_ms_before": round(t_old, 4),
                          "graph_ms_after": round(t_new, 4), "img_s_after": round(a.batch / t_new * 1e3, 1),
                          "tune_s": round(time.time() - t0, 1)}), flush=True)
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(allres, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
