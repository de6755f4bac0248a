"""Named-layer graph IR.

The reference cuts a Keras functional graph at named layers
(`src/dag_util.py:3-62`, `src/dispatcher.py:39-53`).  We do not depend on
Keras: models are described by this small IR whose layer names, layer order
and per-layer weight lists are byte-identical to the Keras
`applications.resnet` graphs, so `part_at` lists and Keras `get_weights()`
lists port over 1:1.

Shapes are per-image NHWC (``(H, W, C)``) or ``(C,)``; the batch dimension is
implicit.  Layers are stored in Keras creation order, which is a valid
topological order.
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

# op kinds understood by the runtime
OPS = (
    "input",      # graph input, attrs: shape
    "zeropad",    # attrs: pad=((t,b),(l,r))
    "conv",       # attrs: filters, kernel=(kh,kw), stride, padding('valid'|'same'), use_bias, activation
    "dwconv",     # DepthwiseConv2D, multiplier 1: kernel, stride, padding, use_bias, activation
    "bn",         # attrs: epsilon
    "relu",       # attrs: max_value (None | 6.0: Keras ReLU(6.))
    "add",
    "concat",     # channel concat (Keras Concatenate(axis=-1))
    "maxpool",    # attrs: pool, stride, padding
    "avgpool",    # attrs: pool, stride, padding (padding excluded from the mean)
    "gap",        # global average pool
    "flatten",    # NHWC -> (H*W*C,) in Keras channels_last order
    "identity",   # Dropout / Activation('linear') at inference
    "dense",      # attrs: units, activation(None|'relu'|'softmax'|any ACTIVATIONS), use_bias
    "softmax",
    "act",        # Keras Activation / LeakyReLU: attrs fn (ACTIVATIONS), alpha (LeakyReLU slope)
    "binary",     # Multiply / Subtract / Maximum / Minimum / Average: attrs fn; the 2nd input may be one
                  # channel row per image (squeeze-excite broadcast)
    "gmp",        # GlobalMaxPooling2D
    "reshape",    # attrs: shape (element order unchanged: NHWC row-major)
    "rescale",    # Keras Rescaling: attrs scale, offset (scalars or per-channel lists)
    "normalization",  # Keras Normalization(axis=-1): weights mean, variance, count
)

# activations the runtime executes (fused into conv / dense / eltwise epilogues,
# csrc/kernels/common.h ActMode), by their Keras names
ACTIVATIONS = ("linear", "relu", "relu6", "swish", "silu", "sigmoid", "tanh", "hard_sigmoid", "hard_swish", "gelu",
               "elu", "selu", "softplus", "leaky_relu")
# Keras activation name -> kernel ActMode (csrc/kernels/common.h); leaky_relu also takes its slope
ACT_MODE = {None: 0, "linear": 0, "relu": 1, "relu6": 2, "swish": 3, "silu": 3, "sigmoid": 4, "tanh": 5,
            "hard_sigmoid": 6, "hard_swish": 7, "gelu": 8, "elu": 9, "selu": 10, "softplus": 11, "leaky_relu": 12}


def bn_params(weights, name: str) -> Dict:
    """gamma / beta / moving statistics of BN layer `name`, with Keras' defaults
    (gamma 1, beta 0) for a layer built with scale=False / center=False."""
    import numpy as np
    mu = weights[f"{name}/moving_mean"]
    return {"gamma": weights.get(f"{name}/gamma", np.ones_like(mu)),
            "beta": weights.get(f"{name}/beta", np.zeros_like(mu)),
            "moving_mean": mu, "moving_variance": weights[f"{name}/moving_variance"]}


def same_pads(size: int, k: int, s: int) -> Tuple[int, int]:
    """TF/Keras 'same' padding of one spatial dim: (before, after), the odd pixel after."""
    out = -(-size // s)
    total = max((out - 1) * s + k - size, 0)
    return total // 2, total - total // 2


def _pair(v) -> Tuple[int, int]:
    return (v, v) if isinstance(v, int) else (int(v[0]), int(v[1]))


@dataclass
class Layer:
    name: str
    op: str
    inputs: List[str]
    attrs: Dict = field(default_factory=dict)
    out_shape: Tuple[int, ...] = ()

    # ---- weights (Keras get_weights() order) ----
    def weight_shapes(self, in_shapes: Sequence[Tuple[int, ...]]) -> List[Tuple[str, Tuple[int, ...]]]:
        """Return [(weight_name, shape)] in Keras order.

        conv: kernel HWIO + bias; bn: gamma, beta, moving_mean, moving_variance;
        dense: kernel (in, out) + bias.
        """
        if self.op == "conv":
            kh, kw = self.attrs["kernel"]
            cin = in_shapes[0][-1]
            out = [(f"{self.name}/kernel", (kh, kw, cin, self.attrs["filters"]))]
            if self.attrs.get("use_bias", True):
                out.append((f"{self.name}/bias", (self.attrs["filters"],)))
            return out
        if self.op == "bn":
            # Keras omits gamma for scale=False (InceptionV3) and beta for center=False
            c = in_shapes[0][-1]
            keep = (("gamma", self.attrs.get("scale", True)), ("beta", self.attrs.get("center", True)),
                    ("moving_mean", True), ("moving_variance", True))
            return [(f"{self.name}/{n}", (c,)) for n, k in keep if k]
        if self.op == "dwconv":
            kh, kw = self.attrs["kernel"]
            cin = in_shapes[0][-1]
            out = [(f"{self.name}/depthwise_kernel", (kh, kw, cin, 1))]
            if self.attrs.get("use_bias", True):
                out.append((f"{self.name}/bias", (cin,)))
            return out
        if self.op == "normalization":
            c = in_shapes[0][-1]
            return [(f"{self.name}/mean", (c,)), (f"{self.name}/variance", (c,)), (f"{self.name}/count", ())]
        if self.op == "dense":
            cin = in_shapes[0][-1]
            out = [(f"{self.name}/kernel", (cin, self.attrs["units"]))]
            if self.attrs.get("use_bias", True):
                out.append((f"{self.name}/bias", (self.attrs["units"],)))
            return out
        return []

    def macs(self, in_shapes: Sequence[Tuple[int, ...]]) -> int:
        """Multiply-accumulates per image."""
        if self.op == "conv":
            kh, kw = self.attrs["kernel"]
            oh, ow, co = self.out_shape
            return oh * ow * co * kh * kw * in_shapes[0][-1]
        if self.op == "dwconv":
            kh, kw = self.attrs["kernel"]
            oh, ow, co = self.out_shape
            return oh * ow * co * kh * kw
        if self.op == "dense":
            return in_shapes[0][-1] * self.attrs["units"]
        return 0

    def to_json(self) -> Dict:
        return {"name": self.name, "op": self.op, "inputs": list(self.inputs),
                "attrs": _jsonable(self.attrs), "out_shape": list(self.out_shape)}

    @staticmethod
    def from_json(d: Dict) -> "Layer":
        attrs = dict(d.get("attrs", {}))
        for k in ("kernel", "pad", "pool"):
            if k in attrs and isinstance(attrs[k], list):
                attrs[k] = _tuplify(attrs[k])
        return Layer(d["name"], d["op"], list(d["inputs"]), attrs, tuple(d.get("out_shape", ())))


def _tuplify(x):
    if isinstance(x, list):
        return tuple(_tuplify(v) for v in x)
    return x


def _jsonable(attrs: Dict) -> Dict:
    def conv(v):
        if isinstance(v, tuple):
            return [conv(x) for x in v]
        return v
    return {k: conv(v) for k, v in attrs.items()}


class Graph:
    """An ordered DAG of named layers (one output tensor per layer)."""

    def __init__(self, name: str = "model"):
        self.name = name
        self.layers: Dict[str, Layer] = {}
        self.order: List[str] = []
        self.input_names: List[str] = []
        self.output_names: List[str] = []
        self._consumers: Optional[Dict[str, List[str]]] = None

    # ---------------------------------------------------------------- build
    def add(self, layer: Layer) -> str:
        if layer.name in self.layers:
            raise ValueError(f"duplicate layer name {layer.name!r}")
        for i in layer.inputs:
            if i not in self.layers:
                raise ValueError(f"layer {layer.name!r} consumes unknown tensor {i!r}")
        layer.out_shape = tuple(layer.out_shape) or self._infer_shape(layer)
        self.layers[layer.name] = layer
        self.order.append(layer.name)
        if layer.op == "input":
            self.input_names.append(layer.name)
        self._consumers = None
        return layer.name

    def _infer_shape(self, layer: Layer) -> Tuple[int, ...]:
        ins = [self.layers[i].out_shape for i in layer.inputs]
        a = layer.attrs
        if layer.op == "input":
            return tuple(a["shape"])
        if layer.op == "zeropad":
            (t, b), (l, r) = a["pad"]
            h, w, c = ins[0]
            return (h + t + b, w + l + r, c)
        if layer.op in ("conv", "dwconv"):
            h, w, c = ins[0]
            kh, kw = a["kernel"]
            s = a.get("stride", 1)
            co = a["filters"] if layer.op == "conv" else c
            if a.get("padding", "valid") == "same":
                return (-(-h // s), -(-w // s), co)
            return ((h - kh) // s + 1, (w - kw) // s + 1, co)
        if layer.op in ("bn", "relu", "softmax", "identity", "act", "rescale", "normalization"):
            return ins[0]
        if layer.op == "binary":
            return ins[0]
        if layer.op == "reshape":
            shp = tuple(int(d) for d in a["shape"])
            n_in = n_out = 1
            for d in ins[0]:
                n_in *= d
            for d in shp:
                n_out *= d
            if n_in != n_out:
                raise ValueError(f"reshape {layer.name}: {ins[0]} -> {shp}")
            return shp
        if layer.op == "flatten":
            n = 1
            for d in ins[0]:
                n *= d
            return (n,)
        if layer.op == "concat":
            if len(ins) < 2 or any(len(s) != 3 or s[:2] != ins[0][:2] for s in ins):
                raise ValueError(f"concat {layer.name}: inputs {ins} do not share H x W")
            return ins[0][:2] + (sum(s[2] for s in ins),)
        if layer.op == "add":
            if any(s != ins[0] for s in ins):
                raise ValueError(f"add {layer.name}: mismatched shapes {ins}")
            return ins[0]
        if layer.op in ("maxpool", "avgpool"):
            h, w, c = ins[0]
            (ph, pw), s = _pair(a["pool"]), a["stride"]
            if a.get("padding", "valid") == "same":
                return (-(-h // s), -(-w // s), c)
            return ((h - ph) // s + 1, (w - pw) // s + 1, c)
        if layer.op in ("gap", "gmp"):
            return (1, 1, ins[0][-1]) if a.get("keepdims") else (ins[0][-1],)
        if layer.op == "dense":
            return (a["units"],)
        raise ValueError(f"unknown op {layer.op}")

    # -------------------------------------------------------------- queries
    def __getitem__(self, name: str) -> Layer:
        return self.layers[name]

    def get_layer(self, name: str) -> Layer:
        if name not in self.layers:
            raise KeyError(f"no layer named {name!r} in {self.name}")
        return self.layers[name]

    def __len__(self) -> int:
        return len(self.order)

    def index(self, name: str) -> int:
        return self.order.index(name)

    @property
    def output(self) -> str:
        return self.output_names[0] if self.output_names else self.order[-1]

    @property
    def input(self) -> str:
        return self.input_names[0]

    def consumers(self) -> Dict[str, List[str]]:
        if self._consumers is None:
            c: Dict[str, List[str]] = {n: [] for n in self.order}
            for n in self.order:
                for i in self.layers[n].inputs:
                    c[i].append(n)
            self._consumers = c
        return self._consumers

    def in_shapes(self, name: str) -> List[Tuple[int, ...]]:
        return [self.layers[i].out_shape for i in self.layers[name].inputs]

    def weight_specs(self, names: Optional[Iterable[str]] = None) -> List[Tuple[str, Tuple[int, ...]]]:
        names = self.order if names is None else list(names)
        out = []
        for n in names:
            out.extend(self.layers[n].weight_shapes(self.in_shapes(n)))
        return out

    def count_params(self) -> int:
        total = 0
        for _, shp in self.weight_specs():
            p = 1
            for d in shp:
                p *= d
            total += p
        return total

    def layer_macs(self, name: str) -> int:
        return self.layers[name].macs(self.in_shapes(name))

    def total_macs(self) -> int:
        return sum(self.layer_macs(n) for n in self.order)

    def ancestors(self, name: str, inclusive: bool = True) -> set:
        """All layers that `name` transitively depends on."""
        seen = set()
        stack = [name]
        while stack:
            n = stack.pop()
            if n in seen:
                continue
            seen.add(n)
            stack.extend(self.layers[n].inputs)
        if not inclusive:
            seen.discard(name)
        return seen

    def tensor_bytes(self, name: str, dtype_bytes: int = 2) -> int:
        p = 1
        for d in self.layers[name].out_shape:
            p *= d
        return p * dtype_bytes

    # ------------------------------------------------------- serialization
    def to_json(self) -> str:
        return json.dumps({
            "format": "adapt-graph-v1",
            "name": self.name,
            "layers": [self.layers[n].to_json() for n in self.order],
            "inputs": self.input_names,
            "outputs": self.output_names,
        })

    @staticmethod
    def from_json(s: str) -> "Graph":
        d = json.loads(s)
        if d.get("format") != "adapt-graph-v1":
            raise ValueError("not an adapt-graph-v1 document")
        g = Graph(d["name"])
        for ld in d["layers"]:
            layer = Layer.from_json(ld)
            # sub-graph inputs may reference tensors produced elsewhere; they
            # are declared as 'input' layers by the slicer, so add() succeeds.
            g.layers[layer.name] = layer
            g.order.append(layer.name)
        g.input_names = list(d["inputs"])
        g.output_names = list(d["outputs"])
        return g

    def to_dot(self, show_shapes: bool = True) -> str:
        """Graphviz DOT of the layer DAG (the reference renders each slice with
        `tf.keras.utils.plot_model`, `src/node.py:49`); slice inputs that stand for
        another slice's tensors are drawn dashed."""
        def q(s: str) -> str:
            return '"' + s.replace('"', r'\"') + '"'
        lines = [f"digraph {q(self.name)} {{", "  rankdir=TB;", '  node [shape=record, fontsize=10];']
        for n in self.order:
            L = self.layers[n]
            label = f"{n}|{L.op}" + (f"|{tuple(L.out_shape)}" if show_shapes else "")
            style = ", style=dashed" if L.op == "input" and L.attrs.get("stands_for", "input") != "input" else ""
            lines.append(f"  {q(n)} [label={q('{' + label + '}')}{style}];")
        for n in self.order:
            for i in self.layers[n].inputs:
                lines.append(f"  {q(i)} -> {q(n)};")
        lines.append("}")
        return "\n".join(lines)

    def summary(self) -> str:
        lines = [f"Model: {self.name}", f"{'Layer':40s} {'Op':8s} {'Output':>18s} {'Params':>10s}"]
        for n in self.order:
            L = self.layers[n]
            p = 0
            for _, shp in L.weight_shapes(self.in_shapes(n)):
                q = 1
                for d in shp:
                    q *= d
                p += q
            lines.append(f"{n:40s} {L.op:8s} {str(L.out_shape):>18s} {p:>10d}")
        lines.append(f"Total params: {self.count_params():,}")
        return "\n".join(lines)
