"""DAG slicing helpers with the reference's API (`src/dag_util.py:1-62`).

* `get_previous(model, name)` -> names of the layers feeding `name`
  (`src/dag_util.py:3-7`);
* `traverse_improved(model, name, start, part_name, inpt, tensor_cache)` ->
  memoised backwards DFS from `name` that stops at `start`
  (`src/dag_util.py:10-48`); in our IR a "tensor" is the producing layer's
  name, and the cache collects the layers the part needs;
* `construct_model(model, start, end, part_name)` -> a `Model` computing
  `end` from `start` (`src/dag_util.py:50-62`).

Difference by design: the reference raises when a skip branch bypasses
`start` (single-tensor cuts only, `src/dag_util.py:38-43`).  We accept such
cuts by turning every bypassing tensor into an extra part input (the
multi-tensor frontier) unless ``strict=True`` asks for the
reference behaviour.
"""
from __future__ import annotations

from typing import Dict, List, Optional

from .graph.ir import Graph, Layer
from .graph.slicer import Slice, subgraph
from .models.model import Model


def _graph(model) -> Graph:
    return model.graph if isinstance(model, Model) else model


def get_previous(model, name: str) -> List[str]:
    return list(_graph(model).get_layer(name).inputs)


def traverse_improved(model, name: str, start: str, part_name: str, inpt: Optional[str],
                      tensor_cache: Dict[str, str], strict: bool = False, frontier: Optional[List[str]] = None) -> str:
    """Collect into `tensor_cache` every layer needed to compute `name` from `start`.

    Returns the tensor name for `name`.  Reaching a graph input other than via
    `start` raises (strict) or records the tensor as an extra frontier input.
    """
    g = _graph(model)
    if name == start:
        return start
    if name == part_name:
        return inpt
    if name in tensor_cache:
        return tensor_cache[name]
    L = g.get_layer(name)
    if L.op == "input":
        if strict:
            raise RuntimeError(f"Error calling layer {name}: branch bypasses the cut at {start!r}; "
                               "the original model's connection involves a merge that the single-tensor cut "
                               "cannot express")
        if frontier is not None and name not in frontier:
            frontier.append(name)
        tensor_cache[name] = name
        return name
    for prev in get_previous(g, name):            # memoised DFS towards `start` (src/dag_util.py:23-40)
        traverse_improved(g, prev, start, part_name, inpt, tensor_cache, strict, frontier)
    tensor_cache[name] = name
    return name


def construct_model(model, start: str, end: str, part_name: str = "part_begin", strict: bool = False) -> Model:
    """Sub-model computing `end` from the output of `start` (exclusive)."""
    g = _graph(model)
    weights = model.weights if isinstance(model, Model) else {}
    start_anc = g.ancestors(start) if g.layers[start].op != "input" else {start}
    if start == g.input:
        start_anc = {start}
    need = g.ancestors(end)
    own = [n for n in g.order if n in need and n not in start_anc]
    inputs = []
    for n in own:
        for i in g.layers[n].inputs:
            if i not in own and i not in inputs:
                inputs.append(i)
    if strict and inputs != [start]:
        raise RuntimeError(f"cut {start!r} -> {end!r} needs frontier {inputs}, not a single tensor")
    if end == start:
        raise ValueError("empty part")
    # when the part starts at the graph input, the input layer itself is the input
    s = Slice(0, part_name, own, inputs or [start], [end], [], start, end)
    sg = subgraph(g, s)
    sg.name = part_name
    wnames = {n for n, _ in g.weight_specs(own)}
    return Model(sg, {k: v for k, v in weights.items() if k in wnames}, name=part_name)
