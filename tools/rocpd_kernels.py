#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 rocpd database (the .db that `rocprofv3 --kernel-trace` writes on
ROCm 7.2): name, calls, total / mean / min µs, sorted by total; optionally the dispatch sequence.

    python tools/rocpd_kernels.py gpurun_out/x/prof/name_results.db [--seq N] [--grid]
"""
import argparse
import sqlite3
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--seq", type=int, default=0, help="print the first N dispatches in order")
    ap.add_argument("--match", default="")
    ap.add_argument("--grid", action="store_true", help="group by (kernel, grid size) instead of kernel")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name_col}, start, end, grid_x, workgroup_x from kernels order by start").fetchall()
    rows = [r for r in rows if a.match in r[0]]
    per = {}
    for n, s, e, gx, wx in rows:
        key = f"{n} grid={gx // max(1, wx)}x{wx}" if a.grid else n
        per.setdefault(key, []).append((e - s) / 1e3)
    tot = sum(sum(v) for v in per.values())
    print(f"{'total_us':>11} {'pct':>6} {'calls':>6} {'mean_us':>9} {'min_us':>9}  kernel")
    for n, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        print(f"{sum(v):11.1f} {100 * sum(v) / tot:6.2f} {len(v):6d} {statistics.mean(v):9.2f} {min(v):9.2f}  {n[:150]}")
    for n, s, e, _, _ in rows[:a.seq]:
        print(f"{(e - s) / 1e3:9.2f}  {n[:120]}")


if __name__ == "__main__":
    main()
