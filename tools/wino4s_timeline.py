#!/usr/bin/env python3
"""Per-wave phase timeline of the split Winograd GEMM (csrc/kernels/wino4s_f32.hip, cfg 299 = cfg 221 with
stamps): for each ResNet-50 bs=32 3x3 shape, one launch with the debug buffer set, then per wave the
prologue (start -> first stage landed), the K loop, the epilogue, and inside the loop the clocks spent in the
land wait (vmcnt + barrier) against the MFMA work (stages x 24 MFMAs x 32 cycles at 1 wave/SIMD), in µs at
the shader clock (s_memtime counts shader clocks, taken as 2.1 GHz under load).

    python tools/wino4s_timeline.py [--json out.json] [--ks 4]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

import torch  # noqa: E402

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops import conv as C_  # noqa: E402

SHAPES = [(32, 56, 64, 1), (32, 28, 128, 2), (32, 14, 256, 4), (32, 7, 512, 8)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    K = C_.kernels()
    out = []
    for (B, H, C, ks) in SHAPES:
        x = torch.randn((B, H, H, C), device="cuda")
        k = torch.randn((3, 3, C, C)) / (3.0 * C ** 0.5)
        pc = C_.pack_conv_f32(k.numpy(), torch.zeros(C).numpy(), 1, ((1, 1), (1, 1)), "cuda")
        y = torch.empty((B, H, H, C), device="cuda")
        ws = torch.empty(C_.wino4s_ws_elems(B, H, H, C, C, ks), dtype=torch.float32, device="cuda")
        nblk = int(K.wino4s_blocks(299, B, H, H, C)) * ks
        dbg = torch.zeros(nblk * 4 * 8, dtype=torch.int64, device="cuda")
        for _ in range(3):                       # warm caches and clocks
            C_.conv_forward_f32(x, pc, y, relu=1, cfg=299, ksplit=ks, workspace=ws)
        torch.cuda.synchronize()
        K.wino4s_set_debug(int(dbg.data_ptr()))
        C_.conv_forward_f32(x, pc, y, relu=1, cfg=299, ksplit=ks, workspace=ws)
        torch.cuda.synchronize()
        K.wino4s_set_debug(0)
        d = dbg.view(-1, 8).cpu().tolist()
        t0 = min(r[0] for r in d)
        us = lambda c: c / 2.1e3                   # noqa: E731 - s_memtime counts shader clocks (~2.1 GHz)
        stages = d[0][6]
        mfma_us = stages * 24 * 32 / 2.1e3       # at ~2.1 GHz, one wave per SIMD's MFMA issue
        rec = {"shape": f"{B}x{H}x{H}x{C}", "ksplit": ks, "waves": len(d), "stages": stages,
               "span_us": round(us(max(r[3] for r in d) - t0), 2),
               "start_skew_us": round(us(max(r[0] for r in d) - t0), 2),
               "prologue_us": round(statistics.mean(us(r[1] - r[0]) for r in d), 2),
               "loop_us": round(statistics.mean(us(r[2] - r[1]) for r in d), 2),
               "epilogue_us": round(statistics.mean(us(r[3] - r[2]) for r in d), 2),
               "land_wait_us": round(statistics.mean(us(r[4]) for r in d), 2),
               "stage_work_us": round(statistics.mean(us(r[5]) for r in d), 2),
               "mfma_issue_floor_us": round(mfma_us, 2)}
        print(json.dumps(rec), flush=True)
        out.append(rec)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
