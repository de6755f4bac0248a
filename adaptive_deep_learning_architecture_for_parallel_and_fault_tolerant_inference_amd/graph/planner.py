"""Cost model and balanced pipeline partition planner.

The reference takes `part_at` from the user verbatim (`test/test.py:15-18`)
and binds slice *i* to worker *i* (`src/dispatcher.py:55-63`), or, in the
gen-2 design, to any live worker per hop (`src/dispatcher.py:176-201`).  On
repartition after a worker joins/leaves we must choose cuts
ourselves, so this module provides:

* a per-layer cost model (MFMA-rate compute + HBM traffic, both per image),
  optionally replaced by measured per-layer times from the runtime;
* `plan_cuts(g, k)`: the min-max-stage DP over *articulation* cut points
  (layers whose ancestor set is exactly the topological prefix, e.g.
  ``pool1_pool`` and every ``*_out``), adding each boundary's transfer time on
  one xGMI link.
"""
from __future__ import annotations

import json
from dataclasses import dataclass, replace
from pathlib import Path
from typing import Dict, List, Optional, Sequence, Tuple

from .ir import Graph

# measured per-layer costs (tools/profile_r50.py --calib) and link rates
# (parallel/check.py --p2p-bw) for gfx950; the analytic model is the fallback
CALIB_FILE = Path(__file__).resolve().parent.parent / "tuning" / "gfx950_layer_costs.json"
LINK_FILE = Path(__file__).resolve().parent.parent / "tuning" / "gfx950_links.json"

# MI355X ballpark figures (MI355X_MICROARCH.md): dense bf16 MFMA ~2.5 PF,
# achievable HBM ~6.3 TB/s, one xGMI link ~150 GB/s.
@dataclass
class HwModel:
    # sustained rate of our fused implicit-GEMM convs: per-layer MI355X measurements
    # at bs=32 run at 0.16-0.55 PF (profiles/r50_bs32_steps_v14.json); 0.35 PF is
    # their FLOP-weighted mean (the round-1 guess of 1.1 PF made late stages look
    # twice as cheap as they are)
    mfma_flops: float = 0.35e15
    hbm_bw: float = 5.0e12                # measured 1x1-conv streaming rate (3.7-5.5 TB/s)
    link_bw: float = 150e9                # replaced by the measured RCCL p2p rate when present
    launch_s: float = 1.5e-6              # kernel boundary inside a hipGraph
    act_bytes: int = 2                    # bf16 activations (for_precision: 4 for fp32 frontiers)


# the fp32 path's sustained conv rate: the fp32 matrix cores peak at 1/16 of bf16 (157 TF); the tuned fp32
# ResNet-50 forward sums 247 GFLOP in 2.26-2.30 ms at bs=32 (profiles/r4/roofline_r50_fp32_bs32.txt), ~0.11 PF
FP32_MFMA_FLOPS = 0.11e15


def for_precision(hw: "HwModel", precision: str) -> "HwModel":
    """The model for a job's activation precision: fp32 frontiers cross a cut at 4 bytes per element (twice
    the bf16 bytes the link terms were first written for) and fp32 convs run at the fp32 matrix rate."""
    if precision == "fp32":
        return replace(hw, act_bytes=4, mfma_flops=min(hw.mfma_flops, FP32_MFMA_FLOPS))
    if precision == "bf16":
        return replace(hw, act_bytes=2)
    return hw


def _calib_key(g: Graph, batch: int, precision: str) -> str:
    return f"{g.name}|{len(g.order)}|b{batch}|{precision}"


def save_calibration(g: Graph, batch: int, precision: str, steps: Sequence[dict],
                     graph_ms: Optional[float] = None) -> Dict[str, float]:
    """Store measured per-step times as per-layer seconds: a fused step's time goes
    to the last layer it covers (cut candidates are fusion-group ends, so a step
    never straddles one)."""
    costs: Dict[str, float] = {}
    for st in steps:
        covers = [c for c in st.get("covers", []) if c in g.layers] or [st["out"].split("#")[0]]
        last = max(covers, key=lambda c: g.order.index(c))
        costs[last] = costs.get(last, 0.0) + float(st["ms"]) * 1e-3
    try:
        table = json.loads(CALIB_FILE.read_text())
    except (OSError, ValueError):
        table = {}
    table[_calib_key(g, batch, precision)] = {"costs_s": costs, "graph_ms": graph_ms}
    CALIB_FILE.parent.mkdir(parents=True, exist_ok=True)
    CALIB_FILE.write_text(json.dumps(table, indent=1, sort_keys=True))
    return costs


def load_calibration(g: Graph, batch: int, precision: str = "bf16") -> Optional[Dict[str, float]]:
    """Measured per-layer seconds for (model, batch, precision), if profiled."""
    try:
        ent = json.loads(CALIB_FILE.read_text()).get(_calib_key(g, batch, precision))
    except (OSError, ValueError):
        return None
    if not ent:
        return None
    costs = {n: 0.0 for n in g.order}
    costs.update({k: float(v) for k, v in ent["costs_s"].items() if k in costs})
    return costs


def measured_link_bw() -> Optional[float]:
    """RCCL p2p bytes/s between neighbouring MI355X (parallel/check.py --p2p-bw)."""
    try:
        return float(json.loads(LINK_FILE.read_text())["link_bw"])
    except (OSError, ValueError, KeyError):
        return None


def default_hw() -> HwModel:
    hw = HwModel()
    bw = measured_link_bw()
    if bw:
        hw.link_bw = bw
    return hw


def layer_costs(g: Graph, batch: int = 32, hw: Optional[HwModel] = None) -> Dict[str, float]:
    """Estimated seconds per layer for a batch (roofline max of compute / memory)."""
    hw = hw or HwModel()
    out = {}
    for n in g.order:
        L = g.layers[n]
        if L.op in ("input",):
            out[n] = 0.0
            continue
        macs = g.layer_macs(n) * batch
        byts = sum(g.tensor_bytes(i, hw.act_bytes) for i in L.inputs) * batch + g.tensor_bytes(n, hw.act_bytes) * batch
        if L.op in ("bn", "relu", "zeropad"):
            # fused into the producing conv / pool at runtime
            out[n] = 0.0
            continue
        if L.op == "add":
            byts = g.tensor_bytes(n, hw.act_bytes) * batch   # residual read inside the conv epilogue
            out[n] = byts / hw.hbm_bw
            continue
        t = max(2.0 * macs / hw.mfma_flops, byts / hw.hbm_bw) + hw.launch_s
        out[n] = t
    return out


def articulation_points(g: Graph) -> List[str]:
    """Layers `c` such that ancestors(c) == topological prefix up to c (single-tensor cuts
    whose stage cost is a contiguous prefix-sum range)."""
    res = []
    seen = set()
    # running check: a layer is an articulation point iff no layer after it
    # consumes a layer before-or-at it other than itself.
    order = g.order
    idx = {n: i for i, n in enumerate(order)}
    # last_use[i] = max index of any consumer of layer i
    cons = g.consumers()
    last_use = [max((idx[c] for c in cons[n]), default=i) for i, n in enumerate(order)]
    running_max = -1
    for i, n in enumerate(order):
        # all layers < i must have their last use <= i... except layer i itself
        if i > 0 and running_max <= i and g.layers[n].op != "input" and n != g.output:
            res.append(n)
        running_max = max(running_max, last_use[i])
        seen.add(n)
    # verify (cheap for <=600 layers)
    verified = []
    for n in res:
        anc = g.ancestors(n)
        if anc == set(order[: idx[n] + 1]):
            verified.append(n)
    return verified


def prefix_points(g: Graph) -> List[str]:
    """Layers `c` whose ancestor set is exactly the topological prefix up to c:
    a cut there makes every stage a contiguous range of the order (so prefix
    sums give stage costs), but unlike an articulation point more than one
    tensor may cross it (a residual branch in flight: the multi-tensor frontier
    of BASELINE config 2)."""
    order = g.order
    out = []
    seen = set()
    for i, n in enumerate(order):
        seen.add(n)
        if g.layers[n].op == "input" or n == g.output:
            continue
        anc = g.ancestors(n)
        if len(anc) == i + 1 and anc == seen:
            out.append(n)
    return out


def crossing_bytes(g: Graph, cut: str, act_bytes: int = 2) -> int:
    """Bytes per image of every tensor produced up to `cut` and consumed after it."""
    idx = {n: i for i, n in enumerate(g.order)}
    i = idx[cut]
    cons = g.consumers()
    return sum(g.tensor_bytes(t, act_bytes) for t in g.order[: i + 1]
               if any(idx[c] > i for c in cons.get(t, [])))


def default_candidates(g: Graph, fine: bool = True) -> List[str]:
    """Articulation points at fusion-group ends: cutting there never splits a
    conv+BN+add+ReLU (or dwconv+BN+ReLU6) epilogue across stages.  ResNet:
    ``pool1_pool`` and the ``*_out`` block outputs; MobileNetV2: the block
    outputs (``*_add`` or ``*_project_BN``); DenseNet: the ``*_concat`` /
    ``pool*_pool`` tensors; VGG: the conv outputs and pools.  A tensor whose
    only consumer is a ZeroPadding2D is skipped (the pad folds into the next op).
    With `fine`, cuts inside a residual block (after its ``_1_relu`` /
    ``_2_relu``: the block input crosses too) are candidates as well."""
    cons = g.consumers()

    def group_end(n: str) -> bool:
        L = g.layers[n]
        c = cons.get(n, [])
        nxt = g.layers[c[0]].op if len(c) == 1 else None
        if nxt == "zeropad":
            return False
        if L.op in ("relu", "maxpool", "avgpool", "concat"):
            return True
        if L.op == "add":
            return nxt != "relu"
        if L.op == "bn":
            return nxt not in ("relu", "add")
        if L.op in ("conv", "dwconv"):
            return L.attrs.get("activation") == "relu"
        return False
    pts = prefix_points(g) if fine else articulation_points(g)
    return [n for n in pts if group_end(n)]


def plan_cuts(g: Graph, stages: int, batch: int = 32, hw: Optional[HwModel] = None,
              costs: Optional[Dict[str, float]] = None,
              candidates: Optional[Sequence[str]] = None, precision: str = "bf16",
              calibrated: bool = True, objective: str = "throughput") -> Tuple[List[str], List[float]]:
    """Min-max DP: returns (part_at, per-stage estimated seconds).  Layer costs:
    `costs` if given, else the measured calibration for (model, batch,
    precision) when one exists, else the analytic roofline model.

    objective "throughput": a stage's period is max(compute, receive, send) on
    its link (the three overlap on separate streams); plans whose period is set
    by a link tie on it and are then ranked by their slowest *compute* stage.
    objective "compute": links are ignored (one device, or links much faster
    than the stages)."""
    if stages < 1:
        raise ValueError("stages must be >= 1")
    hw = for_precision(hw or default_hw(), precision)
    if costs is None and calibrated:
        costs = load_calibration(g, batch, precision)
    costs = costs or layer_costs(g, batch, hw)
    if stages == 1:
        return [], [sum(costs.values())]
    cands = list(candidates) if candidates is not None else default_candidates(g)
    order = g.order
    idx = {n: i for i, n in enumerate(order)}
    cands = sorted(set(cands), key=lambda n: idx[n])
    if len(cands) < stages - 1:
        raise ValueError(f"only {len(cands)} cut candidates for {stages} stages")
    prefix = [0.0]
    for n in order:
        prefix.append(prefix[-1] + costs.get(n, 0.0))
    total = prefix[-1]
    # positions: 0 = start, cands..., end
    pos = [-1] + [idx[c] for c in cands] + [len(order) - 1]
    if objective not in ("throughput", "compute"):
        raise ValueError(f"objective must be throughput or compute, got {objective!r}")
    link = objective == "throughput"
    comm = [0.0] + [crossing_bytes(g, c, hw.act_bytes) * batch / hw.link_bw if link else 0.0 for c in cands] + [0.0]

    def compute(a: int, b: int) -> float:   # stage from after pos[a] to pos[b] inclusive
        return prefix[pos[b] + 1] - prefix[pos[a] + 1]

    def seg(a: int, b: int) -> float:
        # receive / compute / send run on separate HIP streams over a stream of
        # micro-batches, so a stage's steady-state period is the max of the three.
        return max(compute(a, b), comm[a], comm[b])

    P = len(pos)
    INF = (float("inf"), float("inf"))
    # dp[k][j]: best (max period, max compute) covering up to pos[j] with k stages
    dp = [[INF] * P for _ in range(stages + 1)]
    arg = [[-1] * P for _ in range(stages + 1)]
    dp[0][0] = (0.0, 0.0)
    for k in range(1, stages + 1):
        for j in range(1, P):
            best, barg = INF, -1
            for i in range(0, j):
                if dp[k - 1][i] == INF:
                    continue
                v = (max(dp[k - 1][i][0], seg(i, j)), max(dp[k - 1][i][1], compute(i, j)))
                if v < best:
                    best, barg = v, i
            dp[k][j] = best
            arg[k][j] = barg
    # reconstruct
    j = P - 1
    cuts = []
    k = stages
    per = []
    while k > 0:
        i = arg[k][j]
        per.append(seg(i, j))
        if i > 0:
            cuts.append(cands[i - 1])
        j = i
        k -= 1
    cuts.reverse()
    per.reverse()
    if len(cuts) != stages - 1:
        raise RuntimeError("planner failed to place all cuts")
    return cuts, per


def balance_ratio(per_stage: Sequence[float]) -> float:
    """max stage / ideal (1.0 = perfect)."""
    tot = sum(per_stage)
    return max(per_stage) / (tot / len(per_stage)) if tot > 0 else 1.0
