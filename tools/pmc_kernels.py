#!/usr/bin/env python3
"""Mean rocprofv3 --pmc counters per kernel over every run_counter_collection.csv under a directory,
plus derived rates (MFMA busy share of SIMD cycles, wait share of wave cycles, L2 hit rate).
    python tools/pmc_kernels.py gpurun_out/r6f/pmc/h56_221_1 [substring]"""
import collections
import csv
import glob
import sys


def main():
    root, filt = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("adapt::(anonymous namespace)::", "").replace("(adapt::", "[")
            k = k.split("(")[0][:70]
            if filt in k:
                agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in agg.items():
        m = {c: sum(v) / len(v) for c, v in d.items()}
        print(k)
        for c, v in sorted(m.items()):
            print(f"    {c:28s} {v:16.0f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
            # MFMA busy is summed over SIMDs (1024 on MI355X)
            print(f"    mfma_busy_share {m['SQ_VALU_MFMA_BUSY_CYCLES'] / (m['GRBM_GUI_ACTIVE'] * 1024):.3f}")
        if "SQ_WAIT_INST_ANY" in m and "SQ_WAVE_CYCLES" in m:
            print(f"    wait_inst_share {m['SQ_WAIT_INST_ANY'] / max(1, m['SQ_WAVE_CYCLES']):.3f}")
        if "TCC_HIT_sum" in m and "TCC_MISS_sum" in m:
            print(f"    l2_hit_rate     {m['TCC_HIT_sum'] / max(1, m['TCC_HIT_sum'] + m['TCC_MISS_sum']):.3f}")


if __name__ == "__main__":
    main()
