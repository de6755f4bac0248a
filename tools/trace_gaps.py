#!/usr/bin/env python3
"""Inter-kernel gaps of a replayed hipGraph from a rocprofv3 kernel trace.

For every pair of consecutive dispatches on the same queue: gap = start(k+1) - end(k).  Gaps longer than
`--step-gap` µs are taken as the host's turn between replays and split the trace into steps; per step it
reports the kernels, the summed kernel time, the summed gaps inside the step and the step's span.
Measured on the ResNet-50 graphs (profiles/r4/r4s): inside a replayed graph the gap is 0 -- the command
processor stamps a kernel's start when it dispatches it, right after the previous one completes, so the
~2 µs dependent-launch latency shows up inside every kernel's duration, not between kernels; between
two replays of the bench loop the host leaves ~8 µs.

    python tools/trace_gaps.py gpurun_out/r4s/prof_fp32 [--step-gap 4]
"""
import argparse
import glob
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from rocprof_summary import rows_from_csv, rows_from_db  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path", help="rocprofv3 output dir, *_results.db or *kernel_trace.csv")
    ap.add_argument("--step-gap", type=float, default=4.0, help="a gap above this (µs) ends a step")
    ap.add_argument("--min-kernels", type=int, default=20, help="steps with fewer kernels are dropped")
    a = ap.parse_args()
    p = a.path
    if os.path.isdir(p):
        c = glob.glob(os.path.join(p, "**", "*kernel_trace.csv"), recursive=True) or \
            glob.glob(os.path.join(p, "**", "*results.db"), recursive=True)
        if not c:
            raise SystemExit(f"no kernel trace under {p}")
        p = c[0]
    rows = rows_from_db(p) if p.endswith(".db") else rows_from_csv(p)
    rows.sort(key=lambda r: r[5])
    steps, cur = [], [rows[0]]
    for prev, r in zip(rows, rows[1:]):
        if r[5] - prev[6] > a.step_gap:
            steps.append(cur)
            cur = []
        cur.append(r)
    steps.append(cur)
    steps = [s for s in steps if len(s) >= a.min_kernels]
    if not steps:
        raise SystemExit("no step with enough kernels")
    # the modal kernel count is the replayed graph; other groups (warm-up, setup) are dropped
    n = statistics.mode(len(s) for s in steps)
    steps = [s for s in steps if len(s) == n]
    busy = [sum(r[1] for r in s) for s in steps]
    span = [s[-1][6] - s[0][5] for s in steps]
    gaps = [[b[5] - a_[6] for a_, b in zip(s, s[1:])] for s in steps]
    gsum = [sum(g) for g in gaps]
    allg = sorted(x for g in gaps for x in g)
    rec = {"trace": p, "steps": len(steps), "kernels_per_step": n,
           "span_us": round(statistics.median(span), 2), "kernel_us": round(statistics.median(busy), 2),
           "gap_us": round(statistics.median(gsum), 2),
           "gap_per_launch_us": {"p10": round(allg[len(allg) // 10], 2), "p50": round(allg[len(allg) // 2], 2),
                                 "p90": round(allg[9 * len(allg) // 10], 2)},
           "gap_share": round(statistics.median(gsum) / statistics.median(span), 3)}
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
