"""tools/trace_gaps.py on a synthetic rocprofv3 kernel trace: steps are split at the host's long gaps,
the modal step (the replayed graph) is kept, and gaps / spans come out in µs."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _write_trace(path, steps=5, kernels=30, dur_ns=10_000, gap_ns=2_000, step_gap_ns=500_000):
    t = 1_000_000
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Start_Timestamp", "End_Timestamp", "VGPR_Count",
                                          "LDS_Block_Size", "Grid_Size", "Workgroup_Size"])
        w.writeheader()
        # a short warm-up group that must be dropped
        for _ in range(3):
            w.writerow({"Kernel_Name": "warm", "Start_Timestamp": t, "End_Timestamp": t + dur_ns, "VGPR_Count": 8,
                        "LDS_Block_Size": 0, "Grid_Size": 256, "Workgroup_Size": 256})
            t += dur_ns + gap_ns
        t += step_gap_ns
        for _ in range(steps):
            for k in range(kernels):
                w.writerow({"Kernel_Name": f"k{k}", "Start_Timestamp": t, "End_Timestamp": t + dur_ns,
                            "VGPR_Count": 64, "LDS_Block_Size": 0, "Grid_Size": 65536, "Workgroup_Size": 256})
                t += dur_ns + gap_ns
            t += step_gap_ns


def test_trace_gaps_steps_and_gap_share(tmp_path):
    p = tmp_path / "run_kernel_trace.csv"
    _write_trace(p)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "trace_gaps.py"), str(p), "--step-gap", "50"],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    assert rec["steps"] == 5 and rec["kernels_per_step"] == 30
    assert rec["kernel_us"] == 300.0                      # 30 x 10 us
    assert rec["gap_us"] == 58.0                          # 29 gaps of 2 us inside a step
    assert rec["span_us"] == 358.0
    assert rec["gap_per_launch_us"]["p50"] == 2.0
    assert abs(rec["gap_share"] - 58.0 / 358.0) < 1e-3
