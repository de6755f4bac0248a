"""fp32 PyTorch oracle for the graph IR (test oracle + CPU plumbing path).

Implements Keras inference semantics layer by layer (NHWC tensors, HWIO
kernels, zero padding, BN with moving statistics, Dense (in,out)).  It is
what `test/local_infer.py` computes with `model.predict` in the reference,
and what every HIP kernel is checked against.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.nn.functional as F

from ..graph.ir import Graph


class ReferenceExecutor:
    def __init__(self, g: Graph, weights: Dict[str, np.ndarray], device="cpu", dtype=torch.float32):
        self.g = g
        self.device = torch.device(device)
        self.dtype = dtype
        self.w: Dict[str, torch.Tensor] = {}
        for n in g.order:
            L = g.layers[n]
            for wname, _ in L.weight_shapes(g.in_shapes(n)) if L.op != "input" else []:
                self.w[wname] = torch.from_numpy(np.asarray(weights[wname], np.float32)).to(self.device, dtype)

    def _layer(self, L, ins: List[torch.Tensor]) -> torch.Tensor:
        a = L.attrs
        if L.op == "zeropad":
            (t, b), (l, r) = a["pad"]
            return F.pad(ins[0], (0, 0, l, r, t, b))
        if L.op == "conv":
            x = ins[0].permute(0, 3, 1, 2)
            k = self.w[f"{L.name}/kernel"].permute(3, 2, 0, 1)
            bias = self.w.get(f"{L.name}/bias")
            s = a.get("stride", 1)
            if a.get("padding", "valid") == "same":
                kh, kw = a["kernel"]
                H, W = x.shape[2], x.shape[3]
                oh, ow = -(-H // s), -(-W // s)
                ph = max((oh - 1) * s + kh - H, 0)
                pw = max((ow - 1) * s + kw - W, 0)
                x = F.pad(x, (pw // 2, pw - pw // 2, ph // 2, ph - ph // 2))
            y = F.conv2d(x, k, bias, stride=s)
            return y.permute(0, 2, 3, 1)
        if L.op == "bn":
            g_, b_, m_, v_ = (self.w[f"{L.name}/{n}"] for n in ("gamma", "beta", "moving_mean", "moving_variance"))
            return (ins[0] - m_) / torch.sqrt(v_ + a.get("epsilon", 1e-3)) * g_ + b_
        if L.op == "relu":
            return torch.relu(ins[0])
        if L.op == "add":
            y = ins[0]
            for t in ins[1:]:
                y = y + t
            return y
        if L.op == "maxpool":
            x = ins[0].permute(0, 3, 1, 2)
            y = F.max_pool2d(x, a["pool"], a["stride"])
            return y.permute(0, 2, 3, 1)
        if L.op == "gap":
            return ins[0].mean(dim=(1, 2))
        if L.op == "dense":
            y = ins[0] @ self.w[f"{L.name}/kernel"]
            if f"{L.name}/bias" in self.w:
                y = y + self.w[f"{L.name}/bias"]
            if a.get("activation") == "softmax":
                y = torch.softmax(y, dim=-1)
            return y
        if L.op == "softmax":
            return torch.softmax(ins[0], dim=-1)
        raise ValueError(f"unsupported op {L.op}")

    @torch.no_grad()
    def run(self, inputs: Dict[str, torch.Tensor], outputs: Optional[Sequence[str]] = None,
            keep_all: bool = False) -> Dict[str, torch.Tensor]:
        g = self.g
        outputs = list(outputs or g.output_names)
        vals: Dict[str, torch.Tensor] = {}
        for n, t in inputs.items():
            vals[n] = t.to(self.device, self.dtype)
        cons = g.consumers()
        remaining = {n: len(cons[n]) for n in g.order}
        for n in g.order:
            if n in vals:
                continue
            L = g.layers[n]
            if L.op == "input":
                raise KeyError(f"missing input {n}")
            vals[n] = self._layer(L, [vals[i] for i in L.inputs])
            if not keep_all:
                for i in L.inputs:
                    remaining[i] -= 1
                    if remaining[i] == 0 and i not in outputs:
                        vals.pop(i, None)
        return {o: vals[o] for o in outputs} if not keep_all else vals

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        return self.run({self.g.input: x})[self.g.output]
