"""ResNet v1 (50/101/152) graph builders with Keras layer names.

The reference serves `tf.keras.applications.ResNet50(weights='imagenet')`
(`test/test.py:13`, `test/local_infer.py:8`); BASELINE.json also names
ResNet-152.  We rebuild the same graph in our IR: identical layer names
(`conv{s}_block{b}_{0..3}_{conv,bn}`, `_relu`, `_add`, `_out`), identical
creation order (so `part_at` lists and Keras `get_weights()` lists map 1:1),
Conv2D `use_bias=True`, BN epsilon 1.001e-5, NHWC / HWIO layouts.

Parameter totals (checked by tests): R50 25,636,712; R152 60,419,944.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np

from ..graph.ir import Graph, Layer

BN_EPS = 1.001e-5

STACKS = {
    "resnet50": (3, 4, 6, 3),
    "resnet101": (3, 4, 23, 3),
    "resnet152": (3, 8, 36, 3),
    "resnet_tiny": (1, 1, 1, 1),     # same layer naming/structure; for fast CPU tests
    "resnet_mini": (2, 2, 2, 2),
}


def _block1(g: Graph, x: str, filters: int, stride: int, conv_shortcut: bool, name: str) -> str:
    if conv_shortcut:
        sc = g.add(Layer(f"{name}_0_conv", "conv", [x],
                         {"filters": 4 * filters, "kernel": (1, 1), "stride": stride, "padding": "valid", "use_bias": True}))
        sc = g.add(Layer(f"{name}_0_bn", "bn", [sc], {"epsilon": BN_EPS}))
    else:
        sc = x
    y = g.add(Layer(f"{name}_1_conv", "conv", [x],
                    {"filters": filters, "kernel": (1, 1), "stride": stride, "padding": "valid", "use_bias": True}))
    y = g.add(Layer(f"{name}_1_bn", "bn", [y], {"epsilon": BN_EPS}))
    y = g.add(Layer(f"{name}_1_relu", "relu", [y]))
    y = g.add(Layer(f"{name}_2_conv", "conv", [y],
                    {"filters": filters, "kernel": (3, 3), "stride": 1, "padding": "same", "use_bias": True}))
    y = g.add(Layer(f"{name}_2_bn", "bn", [y], {"epsilon": BN_EPS}))
    y = g.add(Layer(f"{name}_2_relu", "relu", [y]))
    y = g.add(Layer(f"{name}_3_conv", "conv", [y],
                    {"filters": 4 * filters, "kernel": (1, 1), "stride": 1, "padding": "valid", "use_bias": True}))
    y = g.add(Layer(f"{name}_3_bn", "bn", [y], {"epsilon": BN_EPS}))
    y = g.add(Layer(f"{name}_add", "add", [sc, y]))
    return g.add(Layer(f"{name}_out", "relu", [y]))


def _stack1(g: Graph, x: str, filters: int, blocks: int, stride1: int, name: str) -> str:
    x = _block1(g, x, filters, stride1, True, f"{name}_block1")
    for i in range(2, blocks + 1):
        x = _block1(g, x, filters, 1, False, f"{name}_block{i}")
    return x


def build_resnet(depth: str = "resnet50", classes: int = 1000, input_shape=(224, 224, 3),
                 input_name: str = "input_1") -> Graph:
    """Build a ResNet v1 graph; `depth` in {'resnet50','resnet101','resnet152'}."""
    depth = depth.lower().replace("-", "")
    if depth not in STACKS:
        raise ValueError(f"unknown ResNet depth {depth!r}; choose from {sorted(STACKS)}")
    g = Graph(depth)
    x = g.add(Layer(input_name, "input", [], {"shape": tuple(input_shape)}))
    x = g.add(Layer("conv1_pad", "zeropad", [x], {"pad": ((3, 3), (3, 3))}))
    x = g.add(Layer("conv1_conv", "conv", [x],
                    {"filters": 64, "kernel": (7, 7), "stride": 2, "padding": "valid", "use_bias": True}))
    x = g.add(Layer("conv1_bn", "bn", [x], {"epsilon": BN_EPS}))
    x = g.add(Layer("conv1_relu", "relu", [x]))
    x = g.add(Layer("pool1_pad", "zeropad", [x], {"pad": ((1, 1), (1, 1))}))
    x = g.add(Layer("pool1_pool", "maxpool", [x], {"pool": 3, "stride": 2, "padding": "valid"}))
    b2, b3, b4, b5 = STACKS[depth]
    x = _stack1(g, x, 64, b2, 1, "conv2")
    x = _stack1(g, x, 128, b3, 2, "conv3")
    x = _stack1(g, x, 256, b4, 2, "conv4")
    x = _stack1(g, x, 512, b5, 2, "conv5")
    x = g.add(Layer("avg_pool", "gap", [x]))
    x = g.add(Layer("predictions", "dense", [x], {"units": classes, "activation": "softmax", "use_bias": True}))
    g.output_names = [x]
    return g


def ResNet50(**kw) -> Graph:
    return build_resnet("resnet50", **kw)


def ResNet101(**kw) -> Graph:
    return build_resnet("resnet101", **kw)


def ResNet152(**kw) -> Graph:
    return build_resnet("resnet152", **kw)


# ------------------------------------------------------------------ weights
def init_weights(g: Graph, seed: int = 0, layers: Optional[List[str]] = None) -> Dict[str, np.ndarray]:
    """Seeded random init in Keras layouts (conv HWIO, dense (in,out)).

    He-normal conv kernels, Glorot-uniform dense, BN statistics near identity
    (gamma of the last BN in each residual branch is damped so activations stay
    O(1) through 50-150 layers of random weights).  Per-layer seeding makes the
    weights of a layer independent of which slice materialises them.
    """
    names = g.order if layers is None else layers
    out: Dict[str, np.ndarray] = {}
    for n in names:
        L = g.layers[n]
        specs = L.weight_shapes(g.in_shapes(n))
        if not specs:
            continue
        rng = np.random.default_rng([seed, _stable_hash(n)])
        if L.op == "conv":
            kh, kw, cin, cout = specs[0][1]
            std = np.sqrt(2.0 / (kh * kw * cin))
            out[specs[0][0]] = (rng.standard_normal((kh, kw, cin, cout)) * std).astype(np.float32)
            if len(specs) > 1:
                out[specs[1][0]] = (rng.standard_normal(cout) * 0.01).astype(np.float32)
        elif L.op == "dwconv":
            kh, kw, cin, mult = specs[0][1]
            std = np.sqrt(2.0 / (kh * kw))
            out[specs[0][0]] = (rng.standard_normal((kh, kw, cin, mult)) * std).astype(np.float32)
            if len(specs) > 1:
                out[specs[1][0]] = (rng.standard_normal(cin * mult) * 0.01).astype(np.float32)
        elif L.op == "bn":
            c = specs[0][1][0]
            # last BN of a residual branch (ResNet `_3_bn`, MobileNetV2 `project_BN`) damped
            damp = 0.2 if n.endswith("_3_bn") or n.endswith("project_BN") else 1.0
            vals = {"gamma": (damp * rng.uniform(0.8, 1.2, c)).astype(np.float32),
                    "beta": (rng.standard_normal(c) * 0.05).astype(np.float32),
                    "moving_mean": (rng.standard_normal(c) * 0.05).astype(np.float32),
                    "moving_variance": rng.uniform(0.5, 1.5, c).astype(np.float32)}
            for wname, _ in specs:                 # scale=False / center=False drop gamma / beta
                out[wname] = vals[wname.rsplit("/", 1)[1]]
        elif L.op == "normalization":
            c = specs[0][1][0]
            out[specs[0][0]] = (rng.standard_normal(c) * 0.1).astype(np.float32)
            out[specs[1][0]] = rng.uniform(0.5, 1.5, c).astype(np.float32)
            out[specs[2][0]] = np.array(1000.0, np.float32)
        elif L.op == "dense":
            cin, units = specs[0][1]
            lim = np.sqrt(6.0 / (cin + units))
            out[specs[0][0]] = rng.uniform(-lim, lim, (cin, units)).astype(np.float32)
            if len(specs) > 1:
                out[specs[1][0]] = np.zeros(units, np.float32)
    return out


def _stable_hash(s: str) -> int:
    h = 2166136261
    for ch in s.encode():
        h = ((h ^ ch) * 16777619) & 0xFFFFFFFF
    return h


def get_weights(g: Graph, weights: Dict[str, np.ndarray], layers: Optional[List[str]] = None) -> List[np.ndarray]:
    """Keras `model.get_weights()`-ordered list for `layers` (default: all)."""
    return [weights[name] for name, _ in g.weight_specs(layers)]


def set_weights(g: Graph, arrays: List[np.ndarray], layers: Optional[List[str]] = None) -> Dict[str, np.ndarray]:
    """Inverse of get_weights: map a Keras-ordered list back to names (shape-checked)."""
    specs = g.weight_specs(layers)
    if len(specs) != len(arrays):
        raise ValueError(f"expected {len(specs)} weight arrays, got {len(arrays)}")
    out = {}
    for (name, shp), arr in zip(specs, arrays):
        if tuple(arr.shape) != tuple(shp):
            raise ValueError(f"{name}: expected shape {shp}, got {arr.shape}")
        out[name] = np.require(arr, np.float32, ["C"])      # keeps 0-d weights (Normalization count) 0-d
    return out
