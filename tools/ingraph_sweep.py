#!/usr/bin/env python3
"""In-graph sweep: for each conv problem (tuning key substring), time the whole
captured ResNet slice with each candidate (cfg, ksplit) against the tuned table,
alternating candidate and baseline captures in one process (isolated kernel
timings mis-rank candidates: tools/ab_cfg.py records).  --adopt writes winners
(>= 0.4 % faster) into the tuning table.

    python tools/ingraph_sweep.py --key 32x7x7x512,3x3s1p1111 --cands 68@-1,62@-1,20@-1
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

import torch  # noqa: E402

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.resnet import init_weights  # noqa: E402
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.zoo import build_model  # noqa: E402
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.runtime.executor import (  # noqa: E402
    SliceExecutor, conv_key, save_tuning)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--key", action="append", required=True, help="comma-separated parts of one tuning key")
    ap.add_argument("--cands", action="append", required=True, help="cfg@ks,... for the matching --key")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--adopt", action="store_true")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    g = build_model(a.model)
    w = init_weights(g, 0)
    ex = SliceExecutor(g, w, a.batch, precision="bf16")
    x = torch.randn((a.batch,) + tuple(g.layers[g.input].out_shape), device="cuda")
    ex.input_buf(g.input).copy_(x)
    rec = {}
    for key, cands in zip(a.key, a.cands):
        idx, fullkey = [], None
        for i in list(ex.cfg):
            B, H, W, C, OH, OW, pc = ex._conv_geom(i)
            ck = conv_key(B, H, W, C, pc)
            if all(p in ck for p in key.split(",")):
                idx.append(i)
                fullkey = ck
        if not idx:
            print(f"{key}: no conv matches")
            continue
        base_cfg = ex.cfg[idx[0]]
        rows = []
        for cand in cands.split(","):
            cfg, ks = (int(v) for v in cand.split("@"))
            tb, tc = [], []
            for _ in range(a.rounds):
                for i in idx:
                    ex.cfg[i] = base_cfg
                ex._ensure_ws()
                tb.append(ex._graph_time(rounds=3, reps=20))
                try:
                    for i in idx:
                        ex.cfg[i] = (cfg, ks)
                    ex._ensure_ws()
                    tc.append(ex._graph_time(rounds=3, reps=20))
                except (RuntimeError, ValueError) as e:
                    print(f"{fullkey} cfg {cfg} ks {ks}: {e}")
                    break
            for i in idx:
                ex.cfg[i] = base_cfg
            if len(tc) < a.rounds:
                continue
            b, c = sorted(tb)[len(tb) // 2], sorted(tc)[len(tc) // 2]
            rows.append((c / b - 1.0, cfg, ks, b, c))
            print(f"{fullkey} x{len(idx)}: tuned {base_cfg} {b:.4f} ms | cfg {cfg} ks {ks} {c:.4f} ms "
                  f"({(c / b - 1) * 100:+.2f} %)", flush=True)
        rows.sort()
        rec[fullkey] = {"tuned": list(base_cfg), "rows": rows}
        if a.adopt and rows and rows[0][0] < -0.004:
            _, cfg, ks, _, _ = rows[0]
            for i in idx:
                ex.cfg[i] = (cfg, ks)
            ex._ensure_ws()
            save_tuning({fullkey: [cfg, ks, 0.0]})
            print(f"adopted {fullkey}: cfg {cfg} ks {ks}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rec, f, indent=1)


if __name__ == "__main__":
    main()
