"""Native CPU execution path: a compiled fp32 plan run by the `_cpu` extension.

The reference's baseline (`/root/reference/test/local_infer.py:18-28`) and
any worker without an accelerator (`/root/reference/src/node.py:177`) run
`model.predict` on TF's CPU kernels in float32.  Here the same graph slice is
compiled by `runtime/plan.py` (``device_fusions=False``: BN folded into the
conv weights, bias / residual Add / activation in the conv epilogue, pads
folded into convs and pools) and every step runs as one OpenMP C++ call of
`csrc/cpu/cpu_ops.cpp` on NHWC float32 numpy arrays.  PyTorch is not on this
path (`ops/reference.py` stays the test oracle), and there is no fallback:
a step kind without a native op raises at construction.

Used by `Model.predict(device="cpu")`, `StageCompute` on a CPU device
(runtime/stage.py) and therefore every CPU DEFER stage (BASELINE config 1).
"""
from __future__ import annotations

import threading
from typing import Dict, List, Optional, Sequence

import numpy as np

from ..graph.ir import Graph, bn_params
from ..ops.conv import fold_bn
from .plan import Step, compile_plan

_mod = None
_lock = threading.Lock()

_BINARY = {"add": 0, "mul": 1, "sub": 2, "max": 3, "min": 4, "avg": 5}


def native():
    """The `_cpu` extension (built in-tree by `_build.build_cpu`); raises if missing."""
    global _mod
    with _lock:
        if _mod is None:
            from .. import _cpu  # noqa: PLC0415
            _mod = _cpu
    return _mod


def _pad_cout(k: np.ndarray, cob: int) -> np.ndarray:
    """HWIO kernel with cout padded to a multiple of the native channel block (zero filters)."""
    co = k.shape[-1]
    cop = -(-co // cob) * cob
    if cop == co:
        return np.ascontiguousarray(k, np.float32)
    out = np.zeros(k.shape[:-1] + (cop,), np.float32)
    out[..., :co] = k
    return out


class CpuExecutor:
    """Runs one (sub)graph on the host CPU with the native `_cpu` ops (fp32)."""

    KINDS = ("conv", "dwconv", "maxpool", "avgpool", "bn", "add", "relu", "act", "binary", "affine", "gmp", "copy",
             "concat", "gap", "dense", "softmax", "pad")

    def __init__(self, g: Graph, weights: Dict[str, np.ndarray], outputs: Optional[Sequence[str]] = None):
        self.g = g
        self.outputs = list(outputs or g.output_names)
        self.steps: List[Step] = compile_plan(g, self.outputs, fp32=True, device_fusions=False)
        bad = sorted({st.kind for st in self.steps if st.kind not in self.KINDS})
        if bad:
            raise NotImplementedError(f"native CPU path has no op for {bad} (model {g.name})")
        self.mod = native()
        self._pack(weights)
        self._logits: Optional[np.ndarray] = None
        last: Dict[str, int] = {}
        for i, st in enumerate(self.steps):
            for t in st.ins:
                last[t] = i
        self._last_use = last

    # ------------------------------------------------------------ weights
    def _folded(self, weights, p):
        bn, eps = None, 1e-3
        if p.get("bn"):
            bn = bn_params(weights, p["bn"])
            eps = self.g.layers[p["bn"]].attrs.get("epsilon", 1e-3)
        return fold_bn(weights[f"{p['conv']}/kernel"], weights.get(f"{p['conv']}/bias"), bn, eps)

    def _pack(self, weights: Dict[str, np.ndarray]) -> None:
        cob = int(self.mod.COB)
        self.packed: Dict[int, tuple] = {}
        for i, st in enumerate(self.steps):
            if st.kind == "conv":
                k, b = self._folded(weights, st.p)
                self.packed[i] = (_pad_cout(k, cob), np.ascontiguousarray(b, np.float32))
            elif st.kind == "dense":
                name = st.p.get("layer", st.out)
                k = np.asarray(weights[f"{name}/kernel"], np.float32)
                b = np.asarray(weights.get(f"{name}/bias", np.zeros(k.shape[1], np.float32)), np.float32)
                self.packed[i] = (_pad_cout(k.reshape(1, 1, *k.shape), cob), np.ascontiguousarray(b))
            elif st.kind == "dwconv":
                p = st.p
                k = weights[f"{p['conv']}/depthwise_kernel"][..., 0]          # (kh, kw, C), multiplier 1
                bn, eps = None, 1e-3
                if p["bn"]:
                    bn = bn_params(weights, p["bn"])
                    eps = self.g.layers[p["bn"]].attrs.get("epsilon", 1e-3)
                kf, bf = fold_bn(k[:, :, None, :], weights.get(f"{p['conv']}/bias"), bn, eps)
                self.packed[i] = (np.ascontiguousarray(kf[:, :, 0, :]), np.ascontiguousarray(bf, np.float32))
            elif st.kind == "bn":
                bp = bn_params(weights, st.p["bn"])
                gm, bt, mu, var = (np.asarray(bp[n], np.float64) for n in
                                   ("gamma", "beta", "moving_mean", "moving_variance"))
                eps = self.g.layers[st.p["bn"]].attrs.get("epsilon", 1e-3)
                sc = gm / np.sqrt(var + eps)
                self.packed[i] = (sc.astype(np.float32), (bt - mu * sc).astype(np.float32))
            elif st.kind == "affine":            # Keras Rescaling / Normalization: y = x * scale + shift
                L = self.g.layers[st.p["layer"]]
                c = L.out_shape[-1]
                if L.op == "rescale":
                    sc = np.broadcast_to(np.asarray(L.attrs.get("scale", 1.0), np.float64), (c,))
                    sh = np.broadcast_to(np.asarray(L.attrs.get("offset", 0.0), np.float64), (c,))
                else:
                    mu = weights[f"{L.name}/mean"].astype(np.float64)
                    sd = np.maximum(np.sqrt(weights[f"{L.name}/variance"].astype(np.float64)), 1e-7)
                    sc, sh = 1.0 / sd, -mu / sd
                self.packed[i] = (np.ascontiguousarray(sc, np.float32), np.ascontiguousarray(sh, np.float32))

    # ------------------------------------------------------------ run
    def _shape(self, name: str, batch: int):
        return (batch,) + tuple(self.g.layers[name.split("#")[0]].out_shape)

    def _step(self, i: int, st: Step, vals: Dict[str, np.ndarray], batch: int) -> np.ndarray:
        m = self.mod
        p = st.p
        ins = [vals[t] for t in st.ins]
        y = np.empty(self._shape(st.out, batch), np.float32)
        k = st.kind
        if k == "conv":
            w, b = self.packed[i]
            (pt, _), (pl, _) = p["pads"]
            if ins[0].ndim != 4:                # a Reshape((1, 1, C)) aliased onto a GAP row (squeeze-excite)
                ins[0] = ins[0].reshape((batch,) + tuple(self.g.layers[self.g.layers[p["conv"]].inputs[0]].out_shape))
            m.conv2d(ins[0], w, b, y, int(p["stride"]), int(pt), int(pl), int(p["relu"]), 0.3,
                     ins[1] if p.get("residual") else None)
        elif k == "dwconv":
            w, b = self.packed[i]
            (pt, _), (pl, _) = p["pads"]
            m.dwconv2d(ins[0], w, b, y, int(p["stride"]), int(pt), int(pl), int(p["relu"]), 0.3)
        elif k in ("maxpool", "avgpool"):
            kh, kw = (p["pool"], p["pool"]) if isinstance(p["pool"], int) else tuple(p["pool"])
            (pt, _), (pl, _) = p["pads"]
            m.pool2d(ins[0], y, 0 if k == "maxpool" else 1, int(kh), int(kw), int(p["stride"]), int(pt), int(pl),
                     bool(p.get("pad_zero", True)))
        elif k in ("bn", "affine"):
            sc, sh = self.packed[i]
            m.affine(ins[0], sc, sh, y, int(p.get("relu", 0)), 0.3)
        elif k == "add":
            m.binary(ins[0], ins[1], y, 0, int(p["relu"]), 0.3)
        elif k == "relu":
            m.activation(ins[0], y, int(p["mode"]), 0.3)
        elif k == "act":
            m.activation(ins[0], y, int(p["mode"]), float(p.get("alpha", 0.3)))
        elif k == "binary":
            m.binary(ins[0], ins[1], y, _BINARY[p["fn"]], int(p["act"]), 0.3)
        elif k in ("gap", "gmp"):
            m.global_pool(ins[0], y, 0 if k == "gap" else 1)
        elif k == "copy":
            y[...] = ins[0].reshape(y.shape)
        elif k == "concat":
            m.concat(list(ins), y)
        elif k == "pad":
            (t, _), (l, _) = p["pad"]
            m.zero_pad(ins[0], y, int(t), int(l))
        elif k == "dense":
            w, b = self.packed[i]
            x = np.ascontiguousarray(ins[0]).reshape(batch, 1, 1, -1)
            z = np.empty((batch, 1, 1, p["units"]), np.float32)
            m.conv2d(x, w, b, z, 1, 0, 0, int(p["relu"]), 0.3, None)
            z = z.reshape(batch, p["units"])
            if p["softmax"]:
                self._logits = z.copy()
                m.softmax(z, y.reshape(batch, -1))
            else:
                y[...] = z.reshape(y.shape)
        elif k == "softmax":
            m.softmax(ins[0], y)
        else:                                           # pragma: no cover - filtered in __init__
            raise NotImplementedError(k)
        return y

    def run(self, inputs: Dict[str, np.ndarray], outputs: Optional[Sequence[str]] = None) -> Dict[str, np.ndarray]:
        vals: Dict[str, np.ndarray] = {n: np.ascontiguousarray(np.asarray(v, np.float32)) for n, v in inputs.items()}
        batch = next(iter(vals.values())).shape[0]
        keep = set(outputs or self.outputs)
        for i, st in enumerate(self.steps):
            vals[st.out] = self._step(i, st, vals, batch)
            for t in set(st.ins):
                if self._last_use.get(t) == i and t not in keep and t not in inputs:
                    vals.pop(t, None)
        out = {}
        for o in (outputs or self.outputs):
            out[o] = vals[o] if o in vals else vals[o]
        return out

    def logits(self) -> Optional[np.ndarray]:
        """Pre-softmax logits of the last run (a Dense(softmax) head), for numerics checks."""
        return self._logits

    def __call__(self, x: np.ndarray) -> np.ndarray:
        return self.run({self.g.input: x})[self.g.output]
