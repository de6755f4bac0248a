#!/usr/bin/env python3
"""Average rocprofv3 --pmc csv counters per kernel (name filter optional).
    python tools/pmc_summary.py gpurun_out/pmc_stem [substring]"""
import collections
import csv
import glob
import sys


def main():
    root = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0][:70]
            if filt in k:
                agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in agg.items():
        print(k)
        for c, v in sorted(d.items()):
            print(f"    {c:28s} {sum(v) / len(v):16.0f}")


if __name__ == "__main__":
    main()
