#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace (rocpd SQLite `*_results.db` or
`kernel_trace.csv`) into a per-kernel table: calls, total/avg µs, share,
VGPR/LDS, grid.  Usage: tools/rocprof_summary.py <db-or-csv> [--top 40] [--skip-first N]
"""
import argparse
import csv
import os
import re
import sqlite3
from collections import defaultdict


def short(name: str) -> str:
    name = re.sub(r"\(.*\)$", "", name)
    name = name.replace("adapt::", "")
    return name[:110]


def rows_from_db(path):
    c = sqlite3.connect(path)
    sym = {}
    for r in c.execute("select id, kernel_name, arch_vgpr_count, accum_vgpr_count, group_segment_size from rocpd_info_kernel_symbol"):
        sym[r[0]] = (r[1], r[2], r[3], r[4])
    out = []
    for kid, start, end, gx, gy, wx in c.execute(
            "select kernel_id, start, end, grid_size_x, grid_size_y, workgroup_size_x from rocpd_kernel_dispatch order by start"):
        name, vg, ag, lds = sym.get(kid, (str(kid), 0, 0, 0))
        out.append((name, (end - start) / 1e3, vg + ag, lds, (gx // max(wx, 1)) * gy, start / 1e3, end / 1e3))
    return out


def rows_from_csv(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            out.append((r["Kernel_Name"], (e - s) / 1e3, int(r.get("VGPR_Count", 0) or 0), int(r.get("LDS_Block_Size", 0) or 0),
                        int(r.get("Grid_Size", 0) or 0) // max(int(r.get("Workgroup_Size", 1) or 1), 1), s / 1e3, e / 1e3))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--skip-first", type=int, default=0, help="drop the first N dispatches (warm-up / tuning)")
    a = ap.parse_args()
    rows = rows_from_db(a.path) if a.path.endswith(".db") else rows_from_csv(a.path)
    rows = rows[a.skip_first:]
    agg = defaultdict(lambda: [0, 0.0, 0, 0, 0])
    for name, us, vg, lds, grid, _, _ in rows:
        k = agg[short(name)]
        k[0] += 1
        k[1] += us
        k[2], k[3], k[4] = vg, lds, grid
    total = sum(v[1] for v in agg.values())
    span = (max(r[6] for r in rows) - min(r[5] for r in rows)) if rows else 0
    print(f"{len(rows)} dispatches, busy {total / 1e3:.3f} ms over a {span / 1e3:.3f} ms span "
          f"({100 * total / span if span else 0:.1f}% busy)")
    print(f"{'kernel':110s} {'calls':>6s} {'total_us':>10s} {'avg_us':>8s} {'pct':>6s} {'vgpr':>5s} {'lds':>6s} {'wgs':>6s}")
    for name, (n, t, vg, lds, grid) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: a.top]:
        print(f"{name:110s} {n:6d} {t:10.1f} {t / n:8.2f} {100 * t / total:6.2f} {vg:5d} {lds:6d} {grid:6d}")


if __name__ == "__main__":
    main()
