#!/usr/bin/env python3
"""Per-wave timeline of one streaming fp32 pointwise launch (csrc/kernels/pw_f32.hip cfgs 122-126).

Every wave of the streaming kernel stamps (`p.dbg`, lane 0): the shader clock and the 100 MHz wall clock
at start, HW_ID / XCC_ID, when its weights and first activation ring have landed (the kernel waits for
them only in this measurement mode), the end of each of its pixel tiles, and the clocks after its last
stores.  From one launch (after warm-up ones) this prints the prologue, the steady per-tile time, the
last tile, the store drain, how the waves start and end in wall time, and the launch span -- where a
launch's time goes beyond its MFMA work.

    python tools/pw_timeline.py --shape 32,28,28,512,128 --cfg 123
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

MFMA_CYCLES = 32          # v_mfma_f32_16x16x4_f32 issue cycles on gfx950


def pct(a, q):
    return round(float(np.percentile(a, q)), 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", required=True, help="B,H,W,K,N (1x1, stride 1)")
    ap.add_argument("--cfg", type=int, default=123)
    ap.add_argument("--res", action="store_true", help="with a residual input")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    B, H, W, K, N = [int(v) for v in a.shape.split(",")]
    dev = "cuda"
    x = torch.randn(B, H, W, K, device=dev)
    kern = (torch.randn(1, 1, K, N) / math.sqrt(K)).numpy()
    pc = C.pack_conv_f32(kern, np.zeros(N, np.float32), 1, ((0, 0), (0, 0)), dev)
    out = torch.empty(B, H, W, N, device=dev)
    res = torch.randn(B, H, W, N, device=dev) if a.res else None
    bm = C.PW_F32_CFGS[a.cfg]
    fpw = kernels().pw_f32_fpw(K, N, 0, bm)
    if fpw <= 0 or bm not in (1, 2, 3, 4, 5):
        raise SystemExit(f"cfg {a.cfg} is not a streaming pointwise config for K={K} N={N}")
    cap = 4096                                     # >= ncg x nslots for every built instance (<= 2048)
    dbg = torch.zeros(cap * 16, dtype=torch.int64, device=dev)

    def run():
        C.conv_forward_f32(x, pc, out, res, relu=1, cfg=a.cfg)

    for _ in range(20):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    kernels().pw_set_debug(dbg.data_ptr())
    try:
        e0.record()
        run()
        e1.record()
        torch.cuda.synchronize()
    finally:
        kernels().pw_set_debug(0)
    launch_us = e0.elapsed_time(e1) * 1e3
    d = dbg.cpu().numpy().astype(np.int64).reshape(cap, 16)
    d = d[d[:, 0] != 0]
    if not len(d):
        raise SystemExit("no wave left a stamp")
    tailw = d[:, 15] >= 100                    # cfgs 125 / 126: the wave also ran a tail fragment
    nt = d[:, 15] % 100
    cyc = d[:, 13] - d[:, 0]
    ghz = float(np.median(cyc / np.maximum(1, d[:, 14] - d[:, 1]) / 10.0))
    us = lambda c: c / ghz / 1e3                                           # noqa: E731
    pro = us(d[:, 4] - d[:, 0])
    tiles = []                                                           # steady tiles: 1 .. nt-2 (<= 7)
    first, last = [], []
    for row, n in zip(d, nt):
        st = [row[4]] + [row[5 + i] for i in range(min(n, 8))]
        dur = np.diff(st)
        first.append(us(dur[0]))
        if n <= 8:
            last.append(us(dur[-1]))
        tiles.extend(us(dur[1:-1]).tolist())
    after = us(d[:, 13] - np.array([r[5 + min(n, 8) - 1] for r, n in zip(d, nt)]))
    drain = after[~tailw] if (~tailw).any() else after
    start = (d[:, 1] - d[:, 1].min()) / 100.0
    end = (d[:, 14] - d[:, 1].min()) / 100.0
    KH = K // 16
    tile_mfma_us = us(KH * 4 * fpw * MFMA_CYCLES)
    hw = d[:, 2]
    cu_key = d[:, 3] * 4096 + ((hw >> 13) & 7) * 256 + ((hw >> 12) & 1) * 16 + ((hw >> 8) & 15)
    simd_key = cu_key * 4 + ((hw >> 4) & 3)
    _, per_simd = np.unique(simd_key, return_counts=True)
    rec = {
        "shape": [B, H, W, K, N], "cfg": a.cfg, "fpw": fpw, "waves": int(len(d)), "launch_us": round(launch_us, 2),
        "shader_ghz": round(ghz, 3), "span_us": round(float(end.max()), 2),
        "tiles_per_wave": {int(k): int(v) for k, v in zip(*np.unique(nt, return_counts=True))},
        "waves_per_simd": {int(k): int(v) for k, v in zip(*np.unique(per_simd, return_counts=True))},
        "tile_mfma_us": round(tile_mfma_us, 3),
        "prologue_us": [pct(pro, q) for q in (10, 50, 90)],
        "first_tile_us": [pct(first, q) for q in (10, 50, 90)],
        "steady_tile_us": [pct(tiles, q) for q in (10, 50, 90)] if tiles else None,
        "last_tile_us": [pct(last, q) for q in (10, 50, 90)] if last else None,
        "store_drain_us": [pct(drain, q) for q in (10, 50, 90)],
        "start_us": [pct(start, q) for q in (0, 50, 90, 100)],
        "end_us": [pct(end, q) for q in (0, 10, 50, 90, 100)],
        "end_us_by_tiles": {int(n): pct(end[(nt == n) & ~tailw], 50) for n in np.unique(nt[~tailw])},
    }
    if tailw.any():
        rec["tail_waves"] = int(tailw.sum())
        rec["tail_fragment_us"] = [pct(after[tailw], q) for q in (10, 50, 90)]
        rec["end_us_tail_waves"] = [pct(end[tailw], q) for q in (50, 100)]
    print(json.dumps(rec))
    if a.json:
        with open(a.json, "w") as f:
            json.dump({**rec, "raw": d.tolist()}, f)


if __name__ == "__main__":
    main()
