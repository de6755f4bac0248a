"""Whole-model A/B of one conv config change: the executor as tuned vs the same
executor with every conv whose tuning key contains --key switched to --cfg,
both hipGraph-captured and replayed alternately in one process.

    python tools/ab_cfg.py --model resnet50 --key 32x28x28x128,1x1s1p0000,512 --cfg 60
(--key: comma-separated parts that must all occur in the conv's tuning key)
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
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.runtime.executor import SliceExecutor, conv_key  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--key", default="")
    ap.add_argument("--cfg", type=int, default=-1)
    ap.add_argument("--set", action="append", default=[],
                    help="KEYPARTS@CFG@KSPLIT, repeatable: switch several conv groups in the B variant")
    ap.add_argument("--ksplit", type=int, default=1, help="split-K (> 1) or stream-K (< 0) of the switched convs")
    ap.add_argument("--env-a", default="", help="K=V;... set while building the A (tuned) executor")
    ap.add_argument("--env-b", default="", help="K=V;... set while building the B executor (plan switches)")
    ap.add_argument("--rounds", type=int, default=15)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    g = build_model(a.model)
    w = init_weights(g, 0)
    x = torch.randn((a.batch,) + tuple(g.layers[g.input].out_shape), device="cuda")
    exs = {}
    sets = [(k, int(c), int(ks)) for k, c, ks in (x.split("@") for x in a.set)]
    if a.key:
        sets.append((a.key, a.cfg, a.ksplit))
    if not sets and not a.env_b:
        ap.error("--key/--cfg, --set or --env-b required")
    bname = f"cfg {a.cfg}" if len(sets) == 1 and a.key else "switched"
    for variant in ("tuned", bname):
        env = dict(kv.split("=", 1) for kv in (a.env_a if variant == "tuned" else a.env_b).split(";") if kv)
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        ex = SliceExecutor(g, w, a.batch, precision=a.precision)
        if env:
            print(f"{variant}: built with {env}, {len(ex.steps)} steps")
        if variant != "tuned":
            hit = []
            for i in list(ex.cfg):
                B, H, W, C, OH, OW, pc = ex._conv_geom(i)
                ck = conv_key(B, H, W, C, pc)
                for key, cfg, ks in sets:
                    if all(part in ck for part in key.split(",")):
                        ex.cfg[i] = (cfg, ks)
                        hit.append(f"{ex.steps[i].out}->{cfg}/{ks}")
            print(f"{variant}: switched {hit}")
            ex._ensure_ws()
        ex.input_buf(g.input).copy_(x.to(ex.input_buf(g.input).dtype)[..., :ex.input_buf(g.input).shape[-1]]
                                    if ex.input_buf(g.input).shape[-1] == x.shape[-1] else
                                    torch.nn.functional.pad(x, (0, ex.input_buf(g.input).shape[-1] - x.shape[-1]))
                                    .to(ex.input_buf(g.input).dtype))
        ex.capture()                     # launch-time switches (env read by the host launchers) land in the graph
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        exs[variant] = ex
    outs = {}
    for v, ex in exs.items():
        ex.forward(0)
        torch.cuda.synchronize()
        outs[v] = ex.output_buf(ex.outputs[0]).float().clone()
    diff = (outs["tuned"] - outs[bname]).abs().max().item()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = {v: [] for v in exs}
    for r in range(a.rounds):
        for v, ex in (exs.items() if r % 2 == 0 else reversed(list(exs.items()))):
            for _ in range(5):
                ex.forward(0)
            e0.record()
            for _ in range(50):
                ex.forward(0)
            e1.record()
            e1.synchronize()
            res[v].append(e0.elapsed_time(e1) / 50)
    rec = {"model": a.model, "batch": a.batch, "precision": a.precision, "sets": sets, "max_abs_diff": diff,
           "ms_median": {v: statistics.median(t) for v, t in res.items()}}
    for v, t in res.items():
        m = statistics.median(t)
        print(f"{v:10s} {m:.4f} ms/batch  {a.batch / m * 1e3:8.0f} img/s")
    print(f"max |output difference| {diff:.3e}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rec, f, indent=1)


if __name__ == "__main__":
    main()
