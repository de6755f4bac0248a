#!/usr/bin/env python3
"""Per-layer roofline table of the fused ResNet plan from rocprofv3 counters.

Two halves:

* ``--run`` (under ``rocprofv3 --pmc ...``): warm the executor, then for every
  plan step launch a separator kernel (``torch.cuda._sleep``, a name no plan
  step uses) followed by REPS eager launches of that step alone; a closing
  separator follows the REPS launches.  ``--meta`` writes the step list (flops,
  compulsory bytes, measured ms from a graph-timed pass): run it once WITHOUT
  the profiler (counter collection serialises dispatches and inflates times),
  and the PMC passes without ``--meta``.
* ``--table``: read the rocprofv3 counter CSVs, split the dispatch stream at
  the separators, average each step's counters over its REPS and print /
  write the table: achieved TFLOP/s, L2<->fabric bytes (TCC_EA0_RDREQ x 128 B
  -- gfx950 tallies a 128-B request at 64 B, MI355X_MICROARCH.md "HBM" --
  plus TCC_EA0_WRREQ x 64 B), compulsory bytes, MFMA busy share and the
  roofline floor max(flop / peak, compulsory bytes / 6.3 TB/s) next to the
  measured time (peak: 2.5 PF bf16, or the measured 150 TF fp32 matrix ceiling
  with ``--dtype fp32``).

The fabric counters include Infinity-Cache hits (the whole bs=32 ResNet-50
working set fits in the 256 MiB MALL), so "fabric bytes" is an upper bound on
HBM traffic.

    rocprofv3 --pmc ... -d out/g1 -o run -- python3 tools/roofline_r50.py --run --meta out/meta.json
    python tools/roofline_r50.py --table out --meta out/meta.json --json profiles/.../roofline.json
"""
import argparse
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

PEAK_BF16 = 2.5e15         # dense bf16 MFMA (no sparsity)
PEAK_FP32 = 1.50e14        # v_mfma_f32_16x16x4_f32 under full load, measured (profiles/r3/mfma_f32_peak.txt)
HBM_BW = 6.3e12            # achievable HBM3E stream (MI355X_MICROARCH.md "HBM")
SEP_NAME = "spin_kernel"   # torch.cuda._sleep: a kernel no plan step launches (fill_ is also used by steps)
REPS = 10


def _bytes_of(ex, g, name, batch):
    b = ex.bufs(0).get(name) if hasattr(ex.bufs(0), "get") else None
    if b is not None:
        return b.numel() * b.element_size()
    return g.tensor_bytes(name, 2) * batch


def _weight_bytes(g, st, esize=2):
    tot = 0
    for c in st.covers:
        L = g.layers[c]
        if L.op not in ("conv", "dwconv", "dense"):
            continue
        shp = L.out_shape
        pix = shp[0] * shp[1] if len(shp) == 3 else 1
        tot += g.layer_macs(c) // pix * esize
    return tot


def _wino_flop(ex, i):
    """Matrix work of a step that runs as Winograd F(2x2, 3x3): 16 positions x (2x2 output tiles, the
    partial edge tiles included) x Cin x Cout MACs -- the floor a Winograd kernel is measured against
    (the direct-conv flop over-states it 2.25x).  None for every other step."""
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops import conv as C
    cfg = ex.cfg.get(i)
    c = cfg[0] if isinstance(cfg, (tuple, list)) else cfg
    if ex.steps[i].kind != "conv" or c not in C.WINO_F32_CFGS:
        return None
    B, H, W, Cin, OH, OW, pc = ex._conv_geom(i)
    tiles = B * ((OH + 1) // 2) * ((OW + 1) // 2)
    return 2 * 16 * tiles * Cin * pc.cout


def _wino4_flop(ex, i):
    """F(4x4, 3x3) matrix work of any 3x3 / stride-1 conv step: 36 positions x (4x4 output tiles, edge tiles
    included) x Cin x Cout MACs -- the floor an F(4,3) Winograd kernel would be measured against (round-4
    verdict item 1), whatever kernel the step runs now.  None for every other step."""
    if ex.steps[i].kind != "conv":
        return None
    B, H, W, Cin, OH, OW, pc = ex._conv_geom(i)
    if (pc.kh, pc.kw, pc.stride) != (3, 3, 1):
        return None
    tiles = B * ((OH + 3) // 4) * ((OW + 3) // 4)
    return 2 * 36 * tiles * Cin * pc.cout


def run(a):
    import torch
    from profile_r50 import single_step, step_flop, time_fn

    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.resnet import \
        init_weights
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.zoo import \
        build_model
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.runtime.executor import \
        SliceExecutor
    g = build_model(a.model)
    w = init_weights(g, 0)
    ex = SliceExecutor(g, w, a.batch, precision=a.dtype)
    ex.input_buf(g.input).copy_(torch.randn(ex.input_buf(g.input).shape, device="cuda"))
    sep = torch.zeros(1, device="cuda")
    for _ in range(3):
        ex._launch(0)
    torch.cuda.synchronize()
    meta = []
    for i, st in enumerate(ex.steps):
        with single_step(ex, i):
            ex._launch(0)
            torch.cuda.synchronize()
            t_ms = None
            if a.meta:
                gg = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gg):
                    for _ in range(20):
                        ex._launch(0)
                t_ms = time_fn(lambda: gg.replay(), reps=5, warm=2) / 20
            torch.cuda.synchronize()
            torch.cuda._sleep(64)               # opening separator
            for _ in range(REPS):
                ex._launch(0)
            torch.cuda._sleep(64)               # closing separator
            torch.cuda.synchronize()
        outs = [st.out] + ([st.p["out2"]] if st.p.get("out2") else [])
        act = sum(_bytes_of(ex, g, n, a.batch) for n in list(st.ins) + outs)
        meta.append({"i": i, "kind": st.kind, "out": st.out, "ms": t_ms, "flop": step_flop(g, st, a.batch),
                     "act_bytes": act, "weight_bytes": _weight_bytes(g, st, 4 if a.dtype == "fp32" else 2),
                     "cfg": ex.cfg.get(i), "wino_flop": _wino_flop(ex, i),
                     "wino4_flop": _wino4_flop(ex, i)})
    if a.meta:
        with open(a.meta, "w") as f:
            json.dump({"model": a.model, "batch": a.batch, "reps": REPS, "dtype": a.dtype, "steps": meta}, f,
                      indent=1)


def _read_counters(d):
    """{dispatch_id: (kernel_name, {counter: value})} from every counter CSV under d."""
    out = {}
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(p) as f:
            for r in csv.DictReader(f):
                did = int(r["Dispatch_Id"])
                name, cnt = out.setdefault(did, (r["Kernel_Name"], {}))
                cnt[r["Counter_Name"]] = cnt.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out


def _segments(disp, n_steps):
    """Per step: summed counters of the dispatches between its opening and closing separator."""
    seq = [disp[k] for k in sorted(disp)]
    seps = [j for j, (name, _) in enumerate(seq) if SEP_NAME in name]
    if len(seps) < 2 * n_steps:
        raise SystemExit(f"found {len(seps)} separators, expected {2 * n_steps}")
    seps = seps[-2 * n_steps:]
    segs = []
    for s0, s1 in zip(seps[0::2], seps[1::2]):
        acc, names = {}, set()
        for name, cnt in seq[s0 + 1:s1]:
            names.add(name.split("(")[0][:80])
            for k, v in cnt.items():
                acc[k] = acc.get(k, 0.0) + v
        segs.append((acc, sorted(names), s1 - s0 - 1))
    return segs


def table(a):
    meta = json.load(open(a.meta))
    steps = meta["steps"]
    peak = PEAK_FP32 if meta.get("dtype") == "fp32" else PEAK_BF16
    reps = meta["reps"]
    merged = [dict() for _ in steps]
    kernels = [None] * len(steps)
    for d in sorted(glob.glob(os.path.join(a.table, "g*"))):
        disp = _read_counters(d)
        if not disp:
            continue
        for i, (acc, names, nd) in enumerate(_segments(disp, len(steps))):
            for k, v in acc.items():
                merged[i][k] = v / reps
            kernels[i] = {"kernels": names, "dispatches_per_launch": nd / reps}
    rows = []
    tot = {"ms": 0.0, "flop": 0, "fabric": 0.0, "compulsory": 0}
    for st, c, kn in zip(steps, merged, kernels):
        rd = c.get("TCC_EA0_RDREQ_sum")
        wr = c.get("TCC_EA0_WRREQ_sum")
        wr64 = c.get("TCC_EA0_WRREQ_64B_sum")
        fabric = None
        if rd is not None and wr is not None:
            wbytes = (wr64 * 64 + (wr - wr64) * 32) if wr64 is not None else wr * 64
            fabric = rd * 128 + wbytes
        comp = st["act_bytes"] + st["weight_bytes"]
        t = st["ms"] * 1e-3 if st["ms"] else None
        floor = max(st["flop"] / peak, comp / HBM_BW)           # compulsory traffic only
        wf = st.get("wino_flop")
        wfloor = max(wf / peak, comp / HBM_BW) if wf else None    # the Winograd kernel's own work floor
        w4 = st.get("wino4_flop")
        w4floor = max(w4 / peak, comp / HBM_BW) if w4 else None   # F(4x4, 3x3) work floor
        row = {"i": st["i"], "kind": st["kind"], "out": st["out"], "cfg": st["cfg"], "ms": st["ms"],
               "gflop": round(st["flop"] / 1e9, 3),
               "tflops": round(st["flop"] / t / 1e12, 1) if t and st["flop"] else None,
               "compulsory_MB": round(comp / 1e6, 2),
               "fabric_MB": round(fabric / 1e6, 2) if fabric is not None else None,
               "fabric_TBps": round(fabric / t / 1e12, 2) if (fabric and t) else None,
               "floor_ms": round(floor * 1e3, 4),
               "bound": "compute" if st["flop"] / peak >= comp / HBM_BW else "memory",
               "mfma_util": round(st["flop"] / t / peak, 3) if t and st["flop"] else None,
               "of_floor": round(t / floor, 2) if t and floor else None,
               "wino_floor_ms": round(wfloor * 1e3, 4) if wfloor else None,
               "of_wino_floor": round(t / wfloor, 2) if t and wfloor else None,
               "wino4_floor_ms": round(w4floor * 1e3, 4) if w4floor else None}
        gui = c.get("GRBM_GUI_ACTIVE")
        mfma = c.get("SQ_VALU_MFMA_BUSY_CYCLES")
        if gui and mfma is not None:
            # SQ_VALU_MFMA_BUSY_CYCLES sums MFMA-busy cycles over SIMDs; GRBM_GUI_ACTIVE sums the
            # kernel's active cycles over the 8 XCDs -> busy share of the 1024 SIMDs
            row["mfma_busy"] = round(mfma / (gui / 8 * 1024), 3)
        for k in ("SQ_LDS_BANK_CONFLICT", "SQ_WAIT_INST_LDS", "TCC_HIT_sum", "TCC_MISS_sum"):
            if k in c:
                row[k] = round(c[k])
        if kn:
            row.update(kn)
        rows.append(row)
        if st["ms"]:
            tot["ms"] += st["ms"]
        tot["flop"] += st["flop"]
        tot["fabric"] += fabric or 0
        tot["compulsory"] += comp
    hdr = f"{'i':>3} {'kind':10} {'out':24} {'ms':>7} {'TF/s':>6} {'compMB':>7} {'fabMB':>7} {'TB/s':>5} " \
          f"{'floor':>7} {'x':>5} {'wfloor':>7} {'xw':>5} {'w4floor':>7} {'mfma':>5} bound"
    print(hdr)
    for r in rows:
        wfl = f"{r['wino_floor_ms']:7.4f}" if r.get("wino_floor_ms") else f"{'-':>7}"
        w4l = f"{r['wino4_floor_ms']:7.4f}" if r.get("wino4_floor_ms") else f"{'-':>7}"
        print(f"{r['i']:3d} {r['kind']:10} {r['out'][:24]:24} {r['ms'] or 0:7.4f} {str(r['tflops']):>6} "
              f"{r['compulsory_MB']:7.2f} {str(r['fabric_MB']):>7} {str(r['fabric_TBps']):>5} {r['floor_ms']:7.4f} "
              f"{str(r['of_floor']):>5} {wfl} {str(r.get('of_wino_floor') or '-'):>5} {w4l} "
              f"{str(r.get('mfma_busy')):>5} {r['bound']}")
    floor_sum = sum(r["floor_ms"] for r in rows)
    wrows = [r for r in rows if r.get("wino_floor_ms")]
    if wrows:
        print(f"winograd 3x3: {len(wrows)} convs, {sum(r['ms'] or 0 for r in wrows):.4f} ms against a Winograd-work "
              f"floor of {sum(r['wino_floor_ms'] for r in wrows):.4f} ms")
    w4rows = [r for r in rows if r.get("wino4_floor_ms")]
    if w4rows:
        print(f"3x3 stride-1: {len(w4rows)} convs, {sum(r['ms'] or 0 for r in w4rows):.4f} ms against an F(4x4, 3x3) "
              f"floor of {sum(r['wino4_floor_ms'] for r in w4rows):.4f} ms")
    print(f"sum: {tot['ms']:.4f} ms, {tot['flop'] / 1e9:.1f} GFLOP, fabric {tot['fabric'] / 1e6:.1f} MB, "
          f"compulsory {tot['compulsory'] / 1e6:.1f} MB, floors {floor_sum:.4f} ms "
          f"(peak {peak / 1e12:.0f} TF/s, {HBM_BW / 1e12:.1f} TB/s)")
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"model": meta["model"], "batch": meta["batch"], "dtype": meta.get("dtype", "bf16"),
                       "peak_flops": peak, "hbm_bw": HBM_BW,
                       "rows": rows, "total": tot}, f, indent=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--run", action="store_true")
    ap.add_argument("--meta", default="")
    ap.add_argument("--table", default="", help="directory holding the g1, g2 ... rocprofv3 output dirs")
    ap.add_argument("--json", default="")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    a = ap.parse_args()
    if a.run:
        run(a)
    if a.table:
        table(a)


if __name__ == "__main__":
    main()
