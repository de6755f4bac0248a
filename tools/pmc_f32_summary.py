#!/usr/bin/env python3
"""Summarise tools/pmc_f32.sh output: one line per (shape, cfg, split) tag with the chip-wide MFMA busy
share (SQ_VALU_MFMA_BUSY_CYCLES over 1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs), the waves' wait shares,
LDS bank-conflict share, instruction mix and L2 hit rate of the adapt:: kernels in each pass.
    python tools/pmc_f32_summary.py gpurun_out/<run>/pmcw"""
import collections
import csv
import glob
import os
import sys


def main():
    root = sys.argv[1]
    for d in sorted(glob.glob(os.path.join(root, "*/"))):
        agg = collections.defaultdict(list)
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if "adapt" in r["Kernel_Name"] and "splitk" not in r["Kernel_Name"]:
                    agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
        a = {k: sum(v) / len(v) for k, v in agg.items()}
        if "GRBM_GUI_ACTIVE" not in a:
            continue
        gui = a["GRBM_GUI_ACTIVE"] / 8
        print(f"{os.path.basename(d.rstrip('/')):40s} mfma_busy {a['SQ_VALU_MFMA_BUSY_CYCLES'] / (gui * 1024):.3f}  "
              f"wait_any {a['SQ_WAIT_ANY'] / a['SQ_WAVE_CYCLES']:.3f}  "
              f"wait_inst_any {a['SQ_WAIT_INST_ANY'] / a['SQ_WAVE_CYCLES']:.3f}  "
              f"lds_conflict/active {a['SQ_LDS_BANK_CONFLICT'] / max(1, a.get('SQ_LDS_IDX_ACTIVE', 1)):.3f}  "
              f"mfma {a['SQ_INSTS_MFMA']:.0f} valu {a.get('SQ_INSTS_VALU', 0):.0f} lds {a.get('SQ_INSTS_LDS', 0):.0f}  "
              f"L2 hit {a['TCC_HIT_sum'] / max(1, a['TCC_HIT_sum'] + a['TCC_MISS_sum']):.2f}")


if __name__ == "__main__":
    main()
