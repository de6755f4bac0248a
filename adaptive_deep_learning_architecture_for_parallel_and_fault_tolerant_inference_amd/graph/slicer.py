"""Graph slicer with multi-tensor cut frontiers.

Reference semantics (`src/dag_util.py:50-62`, `src/dispatcher.py:39-53`):
part *p* spans from the output of ``part_at[p-1]`` (exclusive) to
``part_at[p]`` (inclusive); part 1 starts at the input layer, the last part
ends at the model output.  The reference walks backwards from ``end`` with a
memoised DFS and raises when a branch bypasses ``start``
(`src/dag_util.py:38-43`), i.e. it only supports single-tensor cuts.

We generalise with *ancestor-closure* semantics: part *p* is every layer that
``part_at[p]`` (or the output) depends on and no earlier part already owns.
The *frontier* between part *p* and *p+1* is every tensor produced in parts
``<= p`` that some part ``> p`` consumes; tensors needed further downstream
are relayed through intermediate stages.  For a single-tensor cut this is
exactly the reference partition; for BASELINE config 2
(``part_at=['conv3_block1_1_conv']``) the frontier is
``[conv2_block3_out, conv3_block1_1_conv]``.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Sequence, Tuple

from .ir import Graph, Layer


@dataclass
class Slice:
    """One pipeline stage: a sub-graph with named frontier inputs/outputs."""
    index: int                  # 0-based stage index
    name: str                   # "part{index+1}" like the reference
    layers: List[str]           # owned layers, topological order
    inputs: List[str]           # frontier tensors received (graph input for stage 0)
    outputs: List[str]          # frontier tensors sent downstream (final output for last stage)
    relay: List[str] = field(default_factory=list)   # inputs forwarded unchanged to outputs
    start: str = ""
    end: str = ""

    @property
    def single_tensor(self) -> bool:
        return len(self.inputs) <= 1 and len(self.outputs) <= 1


def partition(g: Graph, part_at: Sequence[str]) -> List[Slice]:
    """Cut `g` at the named layers; returns len(part_at)+1 slices."""
    for n in part_at:
        if n not in g.layers:
            raise KeyError(f"cut layer {n!r} is not in {g.name}")
    ends = list(part_at) + [g.output]
    owner: Dict[str, int] = {}
    for p, end in enumerate(ends):
        anc = g.ancestors(end)
        claimed = [n for n in anc if n not in owner]
        if not claimed:
            raise ValueError(f"cut {end!r} (part {p+1}) is empty: it is already owned by an earlier part; "
                             "cut layers must be in increasing topological order")
        for n in claimed:
            owner[n] = p
    # layers that are not ancestors of the output (dead branches) are dropped
    nparts = len(ends)
    cons = g.consumers()
    # tensors crossing the boundary after part p
    stage_layers: List[List[str]] = [[] for _ in range(nparts)]
    for n in g.order:
        if n in owner:
            stage_layers[owner[n]].append(n)
    boundary: List[List[str]] = []
    for p in range(nparts - 1):
        crossing = []
        for n in g.order:
            if n in owner and owner[n] <= p:
                if any(owner.get(c, -1) > p for c in cons[n]):
                    crossing.append(n)
        boundary.append(crossing)
    slices = []
    for p in range(nparts):
        ins = [g.input] if p == 0 else list(boundary[p - 1])
        outs = [g.output] if p == nparts - 1 else list(boundary[p])
        relay = [t for t in ins if t in outs]
        start = g.input if p == 0 else part_at[p - 1]
        slices.append(Slice(p, f"part{p+1}", stage_layers[p], ins, outs, relay, start, ends[p]))
    return slices


def subgraph(g: Graph, s: Slice) -> Graph:
    """Materialise a slice as a standalone Graph whose inputs are `input` layers
    named after the frontier tensors they stand for."""
    sg = Graph(f"{g.name}:{s.name}")
    for t in s.inputs:
        L = g.layers[t]
        sg.layers[t] = Layer(t, "input", [], {"shape": tuple(L.out_shape), "stands_for": L.op}, tuple(L.out_shape))
        sg.order.append(t)
        sg.input_names.append(t)
    for n in s.layers:
        if n in sg.layers:          # stage-0 graph input
            continue
        L = g.layers[n]
        sg.layers[n] = Layer(L.name, L.op, list(L.inputs), dict(L.attrs), tuple(L.out_shape))
        sg.order.append(n)
    sg.output_names = list(s.outputs)
    return sg


def frontier_bytes(g: Graph, names: Sequence[str], dtype_bytes: int = 2) -> int:
    return sum(g.tensor_bytes(n, dtype_bytes) for n in names)


def is_single_tensor_cut(g: Graph, name: str) -> bool:
    s = partition(g, [name])
    return len(s[0].outputs) == 1


def validate_slices(g: Graph, slices: List[Slice]) -> None:
    """Every layer needed for the output is owned exactly once; every consumed
    tensor is produced in-slice or arrives on the frontier."""
    owned = {}
    for s in slices:
        for n in s.layers:
            if n in owned:
                raise AssertionError(f"{n} owned twice")
            owned[n] = s.index
    for n in g.ancestors(g.output):
        if n not in owned:
            raise AssertionError(f"{n} not owned by any slice")
    for s in slices:
        avail = set(s.inputs) | set(s.layers)
        for n in s.layers:
            for i in g.layers[n].inputs:
                if i not in avail:
                    raise AssertionError(f"slice {s.name}: {n} consumes {i} which is not available")
        for o in s.outputs:
            if o not in avail:
                raise AssertionError(f"slice {s.name}: output {o} not available")
    for a, b in zip(slices, slices[1:]):
        if a.outputs != b.inputs:
            raise AssertionError(f"{a.name}.outputs != {b.name}.inputs")
