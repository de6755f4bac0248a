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

from ..graph.ir import Graph, _pair, same_pads


def _same(x: torch.Tensor, kh: int, kw: int, s: int, value: float = 0.0) -> torch.Tensor:
    """TF 'same' padding of an NCHW tensor (the odd pixel goes after)."""
    t, b = same_pads(x.shape[2], kh, s)
    l, r = same_pads(x.shape[3], kw, s)
    return F.pad(x, (l, r, t, b), value=value)


def _act(y: torch.Tensor, act, alpha: float = 0.3) -> torch.Tensor:
    """Keras activations by name (tf.keras 2.15 definitions)."""
    if act in (None, "linear"):
        return y
    if act == "relu":
        return torch.relu(y)
    if act == "relu6":
        return torch.clamp(y, 0.0, 6.0)
    if act == "softmax":
        return torch.softmax(y, dim=-1)
    if act in ("swish", "silu"):
        return y * torch.sigmoid(y)
    if act == "sigmoid":
        return torch.sigmoid(y)
    if act == "tanh":
        return torch.tanh(y)
    if act == "hard_sigmoid":
        return torch.clamp(0.2 * y + 0.5, 0.0, 1.0)
    if act == "hard_swish":
        return y * torch.clamp(y + 3.0, 0.0, 6.0) / 6.0
    if act == "gelu":
        return F.gelu(y)
    if act == "elu":
        return F.elu(y)
    if act == "selu":
        return F.selu(y)
    if act == "softplus":
        return F.softplus(y)
    if act == "leaky_relu":
        return F.leaky_relu(y, alpha)
    raise ValueError(f"unsupported activation {act!r}")


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
            if L.op == "rescale":           # per-channel Rescaling factors: device tensors made once (graph capture)
                for k in ("scale", "offset"):
                    if isinstance(L.attrs.get(k), (list, tuple)):
                        self.w[f"{n}/#{k}"] = torch.tensor(L.attrs[k], dtype=dtype, device=self.device)

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
                x = _same(x, *a["kernel"], s)
            y = F.conv2d(x, k, bias, stride=s)
            return _act(y.permute(0, 2, 3, 1), a.get("activation"), a.get("alpha", 0.3))
        if L.op == "dwconv":
            x = ins[0].permute(0, 3, 1, 2)
            c = x.shape[1]
            k = self.w[f"{L.name}/depthwise_kernel"].permute(2, 3, 0, 1)      # (C, 1, kh, kw)
            bias = self.w.get(f"{L.name}/bias")
            s = a.get("stride", 1)
            if a.get("padding", "valid") == "same":
                x = _same(x, *a["kernel"], s)
            y = F.conv2d(x, k, bias, stride=s, groups=c)
            return _act(y.permute(0, 2, 3, 1), a.get("activation"))
        if L.op == "bn":
            m_, v_ = self.w[f"{L.name}/moving_mean"], self.w[f"{L.name}/moving_variance"]
            g_ = self.w.get(f"{L.name}/gamma", 1.0)         # scale=False / center=False defaults
            b_ = self.w.get(f"{L.name}/beta", 0.0)
            return (ins[0] - m_) / torch.sqrt(v_ + a.get("epsilon", 1e-3)) * g_ + b_
        if L.op == "relu":
            y = torch.relu(ins[0])
            return y if a.get("max_value") is None else torch.clamp(y, max=float(a["max_value"]))
        if L.op == "identity":
            return ins[0]
        if L.op == "act":
            return _act(ins[0], a["fn"], a.get("alpha", 0.3))
        if L.op == "binary":
            x, y = ins
            if y.dim() != x.dim():                      # one channel row per image
                y = y.reshape((y.shape[0],) + (1,) * (x.dim() - 2) + (y.shape[-1],))
            fn = a["fn"]
            if fn == "mul":
                return x * y
            if fn == "sub":
                return x - y
            if fn == "max":
                return torch.maximum(x, y)
            if fn == "min":
                return torch.minimum(x, y)
            if fn == "avg":
                return 0.5 * (x + y)
            raise ValueError(f"binary {fn}")
        if L.op == "gmp":
            y = ins[0].amax(dim=(1, 2))
            return y.reshape(y.shape[0], 1, 1, -1) if a.get("keepdims") else y
        if L.op == "reshape":
            return ins[0].reshape((ins[0].shape[0],) + tuple(L.out_shape))
        if L.op == "rescale":
            sc, of = a.get("scale", 1.0), a.get("offset", 0.0)
            if isinstance(sc, (list, tuple)):
                sc = self.w[f"{L.name}/#scale"]
            if isinstance(of, (list, tuple)):
                of = self.w[f"{L.name}/#offset"]
            return ins[0] * sc + of
        if L.op == "normalization":
            m, v = self.w[f"{L.name}/mean"], self.w[f"{L.name}/variance"]
            return (ins[0] - m) / torch.clamp(torch.sqrt(v), min=1e-7)
        if L.op == "flatten":
            return ins[0].reshape(ins[0].shape[0], -1)
        if L.op == "concat":
            return torch.cat(ins, dim=-1)
        if L.op == "add":
            y = ins[0]
            for t in ins[1:]:
                y = y + t
            return y
        if L.op in ("maxpool", "avgpool"):
            x = ins[0].permute(0, 3, 1, 2)
            kh, kw = _pair(a["pool"])
            s = a["stride"]
            if L.op == "maxpool":
                if a.get("padding", "valid") == "same":
                    x = _same(x, kh, kw, s, value=float("-inf"))
                y = F.max_pool2d(x, (kh, kw), s)
            elif a.get("padding", "valid") == "same":
                # mean over the in-image part of each window (TF excludes the padding)
                ones = torch.ones_like(x[:, :1])
                num = F.avg_pool2d(_same(x, kh, kw, s), (kh, kw), s, divisor_override=1)
                den = F.avg_pool2d(_same(ones, kh, kw, s), (kh, kw), s, divisor_override=1)
                y = num / den
            else:
                y = F.avg_pool2d(x, (kh, kw), s)
            return y.permute(0, 2, 3, 1)
        if L.op == "gap":
            y = ins[0].mean(dim=(1, 2))
            return y.reshape(y.shape[0], 1, 1, -1) if a.get("keepdims") else y
        if L.op == "dense":
            y = ins[0] @ self.w[f"{L.name}/kernel"]
            if f"{L.name}/bias" in self.w:
                y = y + self.w[f"{L.name}/bias"]
            return _act(y, a.get("activation"))
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
