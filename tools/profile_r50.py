#!/usr/bin/env python3
"""Per-step timing of the fused ResNet plan on one GPU, optional autotune,
and a PyTorch/MIOpen bf16 baseline on the same graph for comparison.

    python tools/profile_r50.py --batch 32 [--tune] [--baseline] [--model resnet50]
"""
import argparse
import contextlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.resnet import init_weights  # noqa: E402
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.zoo import build_model  # noqa: E402
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops.reference import ReferenceExecutor  # noqa: E402
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.runtime.executor import SliceExecutor  # noqa: E402


def time_fn(fn, reps=50, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


@contextlib.contextmanager
def single_step(ex, i):
    """Temporarily make step `i` the executor's whole plan (same buffers, same
    packed weights and tuned config), so `ex._launch(0)` runs just that step."""
    st = ex.steps[i]
    saved = (ex.steps, ex.packed, ex.cfg, ex._logits, ex._dense_part, ex._gap_part, ex._side, ex.relay)
    ex.steps = [st]
    ex.packed = {0: saved[1][i]} if i in saved[1] else {}
    ex.cfg = {0: saved[2][i]} if i in saved[2] else {}
    ex._logits = {0: saved[3][i]} if i in saved[3] else {}
    ex._dense_part = {0: saved[4][i]} if i in saved[4] else {}
    ex._gap_part = {0: saved[5][i]} if i in saved[5] else {}
    ex._side = {}
    ex.relay = []
    try:
        yield st
    finally:
        ex.steps, ex.packed, ex.cfg, ex._logits, ex._dense_part, ex._gap_part, ex._side, ex.relay = saved


def step_flop(g, st, batch):
    """FLOPs of a plan step: 2 x MACs of every conv / dense layer it covers
    (a fused bottleneck step covers three or four convs)."""
    return 2 * batch * sum(g.layer_macs(c) for c in st.covers if g.layers[c].op in ("conv", "dwconv", "dense"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--tune", action="store_true")
    ap.add_argument("--baseline", action="store_true")
    ap.add_argument("--json", default="")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--calib", action="store_true",
                    help="write the measured per-layer costs into the planner's calibration table")
    a = ap.parse_args()
    g = build_model(a.model)
    w = init_weights(g, 0)
    ex = SliceExecutor(g, w, a.batch, tune=a.tune, precision=a.dtype)
    x = torch.randn((a.batch,) + tuple(g.layers[g.input].out_shape), device="cuda")
    ex.input_buf(g.input).copy_(x)
    # per-step eager timing
    total_flop = 0
    # time each step alone by swapping in a one-step plan (same buffers)
    per = []
    for i, st in enumerate(ex.steps):
        with single_step(ex, i):
            # capture 20 back-to-back launches of this one step in a hipGraph so the
            # number is device time, not Python launch overhead
            ex._launch(0)
            torch.cuda.synchronize()
            gg = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gg):
                for _ in range(20):
                    ex._launch(0)
            t = time_fn(lambda: gg.replay(), reps=5, warm=2) / 20
        flop = step_flop(g, st, a.batch)
        total_flop += flop
        per.append({"i": i, "kind": st.kind, "out": st.out, "ms": round(t, 4),
                    "tflops": round(flop / t / 1e9, 1) if flop else None, "cfg": ex.cfg.get(i),
                    "flop": flop, "covers": list(st.covers)})
    ex.capture()
    t_graph = time_fn(lambda: ex.forward(0), reps=100, warm=10)
    print(f"{'i':>3} {'kind':8} {'out':28} {'ms':>8} {'TF/s':>7} cfg")
    for r in per:
        print(f"{r['i']:3d} {r['kind']:8} {r['out']:28} {r['ms']:8.4f} {str(r['tflops']):>7} {r['cfg']}")
    s_eager = sum(r["ms"] for r in per)
    print(f"sum of steps {s_eager:.3f} ms; graph replay {t_graph:.3f} ms/batch -> "
          f"{a.batch / t_graph * 1e3:.0f} img/s; {total_flop / t_graph / 1e9:.1f} TFLOP/s effective")
    out = {"model": a.model, "batch": a.batch, "graph_ms": t_graph, "img_s": a.batch / t_graph * 1e3, "steps": per}
    if a.baseline:
        ref = ReferenceExecutor(g, w, device="cuda", dtype=torch.bfloat16)
        xb = x.to(torch.bfloat16).contiguous(memory_format=torch.contiguous_format)
        with torch.no_grad():
            t_eager = time_fn(lambda: ref.run({g.input: xb}), reps=20, warm=3)
            gr = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                ref.run({g.input: xb})
            torch.cuda.current_stream().wait_stream(s)
            with torch.cuda.graph(gr):
                ref.run({g.input: xb})
            t_tg = time_fn(lambda: gr.replay(), reps=50, warm=5)
        print(f"torch/MIOpen bf16 baseline: eager {t_eager:.3f} ms ({a.batch / t_eager * 1e3:.0f} img/s), "
              f"graph {t_tg:.3f} ms ({a.batch / t_tg * 1e3:.0f} img/s)")
        out["torch_eager_ms"] = t_eager
        out["torch_graph_ms"] = t_tg
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)
    if a.calib:
        from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.graph.planner import \
            save_calibration
        save_calibration(g, a.batch, a.dtype, per, graph_ms=t_graph)
        print(f"calibration written for {g.name} b{a.batch} {a.dtype}")


if __name__ == "__main__":
    main()
