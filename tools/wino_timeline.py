#!/usr/bin/env python3
"""Per-block phase timeline of one fp32 Winograd launch (v3 chunk body, cfgs with PL != 0).

The kernel stamps, per block (thread 0, `conv_wino_f32.hip` `p.dbg`): the shader clock at unit
start, when the first chunk has landed, at the end of the chunk loop and after the epilogue, the
100 MHz wall clock at start and end, HW_ID and XCC_ID.  From one launch (after warm-up ones) this
prints how long the prologue, the chunk loop and the epilogue take per block, how the blocks are
spread over CUs and in time (rounds), and how much of the launch the CUs spend idle.

    python tools/wino_timeline.py --shape 32,56,56,64,64 --cfg 155 --ks 1
"""
import argparse
import json
import math
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops import conv as C  # noqa: E402
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops._lib import kernels  # noqa: E402


def pct(a, q):
    return float(np.percentile(a, q))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", required=True, help="B,H,W,Cin,Cout (3x3, stride 1, pad 1)")
    ap.add_argument("--cfg", type=int, required=True)
    ap.add_argument("--ks", type=int, default=1)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    B, H, W, Cin, Cout = [int(v) for v in a.shape.split(",")]
    dev = "cuda"
    x = torch.randn(B, H, W, Cin, device=dev)
    kern = (torch.randn(3, 3, Cin, Cout) / math.sqrt(9 * Cin)).numpy()
    pc = C.pack_conv_f32(kern, np.zeros(Cout, np.float32), 1, ((1, 1), (1, 1)), dev)
    M, N = B * H * W, Cout
    out = torch.empty(M * N, device=dev)
    nws = C.workspace_elems_f32(M, N, pc.Kpad, a.cfg, a.ks)
    ws = torch.empty(nws, device=dev) if nws else None
    nctr = C.f32_counter_elems(a.cfg, a.ks, B, H, W, H, W, N, pc.Kpad)
    ctr = torch.zeros(nctr, device=dev, dtype=torch.int32) if nctr else None
    nw, fn = C.WINO_F32_CFGS[a.cfg]
    T = B * ((H + 1) // 2) * ((W + 1) // 2)
    nblocks = math.ceil(T / (16 * nw)) * (N // (16 * fn)) * max(1, abs(a.ks))
    if a.ks <= C.WINO_SK_BASE:                    # stream-K: a 1-D grid; a block's second unit overwrites its stamps
        nblocks = C.wino_sk_plan(a.cfg, B, H, W, N, Cin, a.ks)[0]
    dbg = torch.zeros(nblocks * 16, dtype=torch.int64, device=dev)

    def run():
        C.conv_forward_f32(x, pc, out, relu=1, cfg=a.cfg, ksplit=a.ks, workspace=ws, counters=ctr)

    for _ in range(20):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    kernels().wino_set_debug(dbg.data_ptr())
    try:
        e0.record()
        run()
        e1.record()
        torch.cuda.synchronize()
    finally:
        kernels().wino_set_debug(0)
    launch_us = e0.elapsed_time(e1) * 1e3
    d = dbg.cpu().numpy().astype(np.int64).reshape(nblocks, 16)
    if (d[:, 0] == 0).any():
        raise SystemExit(f"{int((d[:, 0] == 0).sum())} of {nblocks} blocks left no stamp (cfg without PL?)")
    wall0, wall1 = d[:, 4], d[:, 5]
    cyc = d[:, 3] - d[:, 0]
    ghz = float(np.median(cyc / np.maximum(1, wall1 - wall0) / 10.0))     # shader cycles per ns
    us = lambda c: c / ghz / 1e3                                          # noqa: E731
    pro, loop, epi = us(d[:, 1] - d[:, 0]), us(d[:, 2] - d[:, 1]), us(d[:, 3] - d[:, 2])
    start = (wall0 - wall0.min()) / 100.0                                 # us
    end = (wall1 - wall0.min()) / 100.0
    hw = d[:, 6]
    cu_key = d[:, 7] * 4096 + ((hw >> 13) & 7) * 256 + ((hw >> 12) & 1) * 16 + ((hw >> 8) & 15)  # xcc, se, sh, cu
    cus, per_cu = np.unique(cu_key, return_counts=True)
    busy = float((end - start).sum())
    span = float(end.max())
    rec = {
        "shape": [B, H, W, Cin, Cout], "cfg": a.cfg, "ks": a.ks, "blocks": nblocks, "launch_us": round(launch_us, 2),
        "shader_ghz": round(ghz, 3), "span_us": round(span, 2), "cus_used": int(len(cus)),
        "blocks_per_cu": {int(k): int(v) for k, v in zip(*np.unique(per_cu, return_counts=True))},
        "prologue_us": [round(pct(pro, q), 2) for q in (10, 50, 90)],
        "loop_us": [round(pct(loop, q), 2) for q in (10, 50, 90)],
        "epilogue_us": [round(pct(epi, q), 2) for q in (10, 50, 90)],
        **({"epi_stage_us": round(float(np.median(us(d[:, 8] - d[:, 2]))), 2),
            "epi_readback_us": round(float(np.median(us(d[:, 9] - d[:, 8]))), 2),
            "epi_stores_us": round(float(np.median(us(d[:, 10] - d[:, 9]))), 2),
            "epi_tail_us": round(float(np.median(us(d[:, 3] - d[:, 10]))), 2)} if (d[:, 10] != 0).all() else {}),
        **({"chunk_barrier_wait_us": round(float(np.median(us(d[:, 12] - d[:, 11]))), 3),
            "chunk_groups_0_7_us": round(float(np.median(us(d[:, 13] - d[:, 12]))), 3),
            "chunk_groups_8_15_us": round(float(np.median(us(d[:, 14] - d[:, 13]))), 3),
            "chunk_patch_read_us": round(float(np.median(us(d[:, 15] - d[:, 14]))), 3)}
           if (d[:, 15] != 0).all() else {}),
        "start_us": [round(pct(start, q), 2) for q in (0, 50, 90, 100)],
        "end_us": [round(pct(end, q), 2) for q in (0, 10, 50, 90, 100)],
        "cu_busy_fraction": round(busy / (256 * span), 3),
    }
    print(json.dumps(rec))
    if a.json:
        with open(a.json, "w") as f:
            json.dump({**rec, "raw": d.tolist()}, f)


if __name__ == "__main__":
    main()
