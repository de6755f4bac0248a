"""Keras functional-model JSON <-> our graph IR.

The reference ships every slice to its worker as ``model.to_json()`` and
rebuilds it with ``tf.keras.models.model_from_json`` (`src/dispatcher.py:
234-236`, `src/node.py:40,77`), and its dispatcher accepts any Keras
functional model (`src/dispatcher.py:39-53`).  This module reads that JSON
(no TensorFlow involved) into our IR so an existing Keras architecture, plus
its ``get_weights()`` list, runs on our engine unchanged; and writes our
graphs back out in the same format.

Both serialisations are understood:

* Keras 2 / tf.keras 2.x (the reference's TF 2.15): ``inbound_nodes`` is a
  list of nodes, each a list of ``[layer_name, node_index, tensor_index,
  kwargs]``; ``InputLayer`` carries ``batch_input_shape``.
* Keras 3: each node is ``{"args": [...], "kwargs": {...}}`` whose tensors
  are ``{"class_name": "__keras_tensor__", "config": {"keras_history":
  [layer, node, index]}}``; ``InputLayer`` carries ``batch_shape``.

Supported layer classes are the ones the runtime executes (graph/ir.py
OPS); anything else raises ``NotImplementedError`` naming the layer.  Only
``channels_last`` data, single-output layers and one call per layer (no
shared layers, as in the reference's `src/dag_util.py:23-25`).
"""
from __future__ import annotations

import json
from typing import Any, Dict, List, Tuple

from .ir import ACTIVATIONS, Graph, Layer, _pair

_BINARY = {"Multiply": "mul", "Subtract": "sub", "Maximum": "max", "Minimum": "min", "Average": "avg"}


def _inbound_names(layer: Dict[str, Any]) -> List[str]:
    nodes = layer.get("inbound_nodes") or []
    if not nodes:
        return []
    if len(nodes) > 1:
        raise NotImplementedError(f"layer {layer.get('name')!r} is called more than once (shared layer)")
    node = nodes[0]
    if isinstance(node, dict):                       # Keras 3
        names: List[str] = []

        def walk(v):
            if isinstance(v, dict):
                if v.get("class_name") == "__keras_tensor__":
                    names.append(v["config"]["keras_history"][0])
                else:
                    for x in v.values():
                        walk(x)
            elif isinstance(v, (list, tuple)):
                for x in v:
                    walk(x)
        walk(node.get("args", []))
        return names
    return [entry[0] for entry in node]               # Keras 2: [[name, node, tensor, kwargs], ...]


def _padding2d(p) -> Tuple[Tuple[int, int], Tuple[int, int]]:
    if isinstance(p, int):
        return ((p, p), (p, p))
    a, b = p
    if isinstance(a, int):
        return ((a, a), (b, b))
    return ((int(a[0]), int(a[1])), (int(b[0]), int(b[1])))


def _stride(cfg: Dict[str, Any], name: str) -> int:
    sh, sw = _pair(cfg.get("strides", 1))
    if sh != sw:
        raise NotImplementedError(f"{name}: unequal strides {sh}x{sw}")
    return sh


def _check_channels_last(cfg: Dict[str, Any], name: str) -> None:
    if cfg.get("data_format", "channels_last") not in (None, "channels_last"):
        raise NotImplementedError(f"{name}: data_format {cfg['data_format']!r}")


def _activation(act, name: str):
    """A Keras activation config (a name, or a serialized function in Keras 3) -> our name."""
    if isinstance(act, dict):
        act = act.get("config", {}).get("name", act.get("class_name"))
    if act in (None, "linear"):
        return None
    if act not in ACTIVATIONS and act != "softmax":
        raise NotImplementedError(f"{name}: activation {act!r}")
    return act


def _layers_from_keras(cls: str, cfg: Dict[str, Any], name: str, inputs: List[str]) -> List[Layer]:
    """Most classes map to one IR layer; SeparableConv2D lowers to a depthwise + a pointwise conv (same
    get_weights() order: depthwise_kernel, pointwise_kernel, bias), the pointwise one keeping the Keras name."""
    if cls == "SeparableConv2D":
        _check_channels_last(cfg, name)
        if int(cfg.get("depth_multiplier", 1)) != 1 or _pair(cfg.get("dilation_rate", 1)) != (1, 1):
            raise NotImplementedError(f"{name}: SeparableConv2D with depth_multiplier / dilation")
        dw = Layer(f"{name}/depthwise", "dwconv", inputs,
                   {"kernel": _pair(cfg["kernel_size"]), "stride": _stride(cfg, name),
                    "padding": cfg.get("padding", "valid"), "use_bias": False})
        a = {"filters": int(cfg["filters"]), "kernel": (1, 1), "stride": 1, "padding": "valid",
             "use_bias": bool(cfg.get("use_bias", True))}
        act = _activation(cfg.get("activation"), name)
        if act:
            a["activation"] = act
        return [dw, Layer(name, "conv", [dw.name], a)]
    return [_layer_from_keras(cls, cfg, name, inputs)]


def _layer_from_keras(cls: str, cfg: Dict[str, Any], name: str, inputs: List[str]) -> Layer:
    if cls == "InputLayer":
        shp = cfg.get("batch_input_shape") or cfg.get("batch_shape")
        return Layer(name, "input", [], {"shape": tuple(int(d) for d in shp[1:])})
    _check_channels_last(cfg, name)
    if cls == "ZeroPadding2D":
        return Layer(name, "zeropad", inputs, {"pad": _padding2d(cfg["padding"])})
    if cls in ("Conv2D", "DepthwiseConv2D"):
        if _pair(cfg.get("dilation_rate", 1)) != (1, 1) or cfg.get("groups", 1) != 1:
            raise NotImplementedError(f"{name}: dilated / grouped convolution")
        a = {"kernel": _pair(cfg["kernel_size"]), "stride": _stride(cfg, name),
             "padding": cfg.get("padding", "valid"), "use_bias": bool(cfg.get("use_bias", True))}
        act = _activation(cfg.get("activation", "linear"), name)
        if act == "softmax":
            raise NotImplementedError(f"{name}: softmax on a convolution")
        if act:
            a["activation"] = act
        if cls == "Conv2D":
            a["filters"] = int(cfg["filters"])
            return Layer(name, "conv", inputs, a)
        if int(cfg.get("depth_multiplier", 1)) != 1:
            raise NotImplementedError(f"{name}: depth_multiplier != 1")
        return Layer(name, "dwconv", inputs, a)
    if cls == "BatchNormalization":
        axis = cfg.get("axis", -1)
        axis = axis[0] if isinstance(axis, list) else axis
        if axis not in (-1, 3):
            raise NotImplementedError(f"{name}: BatchNormalization needs axis=-1")
        a = {"epsilon": float(cfg.get("epsilon", 1e-3))}
        for k in ("center", "scale"):
            if not cfg.get(k, True):
                a[k] = False
        return Layer(name, "bn", inputs, a)
    if cls == "ReLU":
        if float(cfg.get("threshold", 0.0) or 0.0) != 0.0:
            raise NotImplementedError(f"{name}: thresholded ReLU")
        mv = cfg.get("max_value")
        slope = float(cfg.get("negative_slope", 0.0) or 0.0)
        if slope:
            if mv is not None:
                raise NotImplementedError(f"{name}: ReLU with both max_value and negative_slope")
            return Layer(name, "act", inputs, {"fn": "leaky_relu", "alpha": slope})
        if mv is not None and float(mv) != 6.0:
            raise NotImplementedError(f"{name}: ReLU(max_value={mv})")
        return Layer(name, "relu", inputs, {"max_value": float(mv)} if mv is not None else {})
    if cls == "LeakyReLU":
        alpha = cfg.get("alpha", cfg.get("negative_slope", 0.3))
        return Layer(name, "act", inputs, {"fn": "leaky_relu", "alpha": float(alpha)})
    if cls == "Activation":
        act = _activation(cfg["activation"], name)
        if act is None:
            return Layer(name, "identity", inputs)
        if act == "relu":
            return Layer(name, "relu", inputs)
        if act == "softmax":
            return Layer(name, "softmax", inputs)
        return Layer(name, "act", inputs, {"fn": act})
    if cls in _BINARY:
        if len(inputs) != 2:
            raise NotImplementedError(f"{name}: {cls} of {len(inputs)} inputs")
        return Layer(name, "binary", inputs, {"fn": _BINARY[cls]})
    if cls == "GlobalMaxPooling2D":
        return Layer(name, "gmp", inputs, {"keepdims": True} if cfg.get("keepdims") else {})
    if cls == "Reshape":
        return Layer(name, "reshape", inputs, {"shape": tuple(int(d) for d in cfg["target_shape"])})
    if cls == "Rescaling":
        return Layer(name, "rescale", inputs, {"scale": cfg.get("scale", 1.0), "offset": cfg.get("offset", 0.0)})
    if cls == "Normalization":
        axis = cfg.get("axis", -1)
        axis = axis[0] if isinstance(axis, list) and len(axis) == 1 else axis
        if axis not in (-1, 3) or cfg.get("invert"):
            raise NotImplementedError(f"{name}: Normalization needs axis=-1")
        return Layer(name, "normalization", inputs)
    if cls == "Softmax":
        return Layer(name, "softmax", inputs)
    if cls == "Add":
        return Layer(name, "add", inputs)
    if cls == "Concatenate":
        if cfg.get("axis", -1) not in (-1, 3):
            raise NotImplementedError(f"{name}: concat axis {cfg.get('axis')}")
        return Layer(name, "concat", inputs)
    if cls in ("MaxPooling2D", "AveragePooling2D"):
        pool = _pair(cfg.get("pool_size", 2))
        strides = cfg.get("strides") or cfg.get("pool_size", 2)
        sh, sw = _pair(strides)
        if sh != sw:
            raise NotImplementedError(f"{name}: unequal pooling strides")
        return Layer(name, "maxpool" if cls == "MaxPooling2D" else "avgpool", inputs,
                     {"pool": pool if pool[0] != pool[1] else pool[0], "stride": sh,
                      "padding": cfg.get("padding", "valid")})
    if cls == "GlobalAveragePooling2D":
        return Layer(name, "gap", inputs, {"keepdims": True} if cfg.get("keepdims") else {})
    if cls == "Flatten":
        return Layer(name, "flatten", inputs)
    if cls in ("Dropout", "SpatialDropout2D", "GaussianDropout", "GaussianNoise", "ActivityRegularization"):
        return Layer(name, "identity", inputs)
    if cls == "Dense":
        act = _activation(cfg.get("activation", "linear"), name)
        a = {"units": int(cfg["units"]), "use_bias": bool(cfg.get("use_bias", True))}
        if act:
            a["activation"] = act
        return Layer(name, "dense", inputs, a)
    raise NotImplementedError(f"layer {name!r}: Keras class {cls!r} is not supported by the runtime")


def from_keras_json(s) -> Graph:
    """Parse ``model.to_json()`` output (str or already-decoded dict) into a Graph."""
    d = json.loads(s) if isinstance(s, (str, bytes)) else s
    if d.get("class_name") not in ("Functional", "Model"):
        raise NotImplementedError(f"only functional models are supported (got {d.get('class_name')!r})")
    cfg = d["config"]
    g = Graph(cfg.get("name", "model"))
    for ld in cfg["layers"]:
        name = ld.get("name") or ld["config"]["name"]
        for layer in _layers_from_keras(ld["class_name"], ld["config"], name, _inbound_names(ld)):
            g.add(layer)

    def names(v) -> List[str]:
        if isinstance(v, list) and v and isinstance(v[0], str):
            return [v[0]]                                   # a single [name, node, tensor]
        return [e[0] for e in v]
    g.input_names = names(cfg["input_layers"])
    g.output_names = names(cfg["output_layers"])
    return g


# ------------------------------------------------------------------ export
def _keras_layer(L: Layer, g: Graph) -> Dict[str, Any]:
    a = L.attrs
    cfg: Dict[str, Any] = {"name": L.name, "trainable": True, "dtype": "float32"}
    if L.op == "input":
        cls = "InputLayer"
        cfg = {"batch_input_shape": [None] + list(a["shape"]), "dtype": "float32", "sparse": False,
               "ragged": False, "name": L.name}
    elif L.op == "zeropad":
        cls = "ZeroPadding2D"
        cfg.update(padding=[list(p) for p in a["pad"]], data_format="channels_last")
    elif L.op in ("conv", "dwconv"):
        cls = "Conv2D" if L.op == "conv" else "DepthwiseConv2D"
        cfg.update(kernel_size=list(_pair(a["kernel"])), strides=[a.get("stride", 1)] * 2,
                   padding=a.get("padding", "valid"), data_format="channels_last", dilation_rate=[1, 1],
                   activation=a.get("activation") or "linear", use_bias=a.get("use_bias", True))
        if L.op == "conv":
            cfg.update(filters=a["filters"], groups=1)
        else:
            cfg.update(depth_multiplier=1)
    elif L.op == "bn":
        cls = "BatchNormalization"
        cfg.update(axis=[3], momentum=0.99, epsilon=a.get("epsilon", 1e-3), center=a.get("center", True),
                   scale=a.get("scale", True))
    elif L.op == "relu":
        if a.get("max_value") is None:
            cls = "Activation"
            cfg.update(activation="relu")
        else:
            cls = "ReLU"
            cfg.update(max_value=a["max_value"], negative_slope=0.0, threshold=0.0)
    elif L.op == "add":
        cls = "Add"
    elif L.op == "concat":
        cls = "Concatenate"
        cfg.update(axis=-1)
    elif L.op in ("maxpool", "avgpool"):
        cls = "MaxPooling2D" if L.op == "maxpool" else "AveragePooling2D"
        cfg.update(pool_size=list(_pair(a["pool"])), strides=[a["stride"]] * 2, padding=a.get("padding", "valid"),
                   data_format="channels_last")
    elif L.op in ("gap", "gmp"):
        cls = "GlobalAveragePooling2D" if L.op == "gap" else "GlobalMaxPooling2D"
        cfg.update(data_format="channels_last", keepdims=bool(a.get("keepdims", False)))
    elif L.op == "act":
        if a["fn"] == "leaky_relu":
            cls = "LeakyReLU"
            cfg.update(alpha=a.get("alpha", 0.3))
        else:
            cls = "Activation"
            cfg.update(activation=a["fn"])
    elif L.op == "binary":
        cls = {v: k for k, v in _BINARY.items()}[a["fn"]]
    elif L.op == "reshape":
        cls = "Reshape"
        cfg.update(target_shape=list(a["shape"]))
    elif L.op == "rescale":
        cls = "Rescaling"
        cfg.update(scale=a.get("scale", 1.0), offset=a.get("offset", 0.0))
    elif L.op == "normalization":
        cls = "Normalization"
        cfg.update(axis=[-1], invert=False)
    elif L.op == "flatten":
        cls = "Flatten"
        cfg.update(data_format="channels_last")
    elif L.op == "identity":
        cls = "Activation"
        cfg.update(activation="linear")
    elif L.op == "dense":
        cls = "Dense"
        cfg.update(units=a["units"], activation=a.get("activation") or "linear", use_bias=a.get("use_bias", True))
    elif L.op == "softmax":
        cls = "Activation"
        cfg.update(activation="softmax")
    else:
        raise NotImplementedError(L.op)
    inbound = [[[i, 0, 0, {}] for i in L.inputs]] if L.inputs else []
    return {"class_name": cls, "config": cfg, "name": L.name, "inbound_nodes": inbound}


def to_keras_json(g: Graph) -> str:
    """Our graph as Keras 2 functional-model JSON (``model.to_json()`` layout)."""
    layers = [_keras_layer(g.layers[n], g) for n in g.order]
    outs = g.output_names or [g.order[-1]]
    return json.dumps({"class_name": "Functional",
                       "config": {"name": g.name, "trainable": True, "layers": layers,
                                  "input_layers": [[n, 0, 0] for n in g.input_names],
                                  "output_layers": [[n, 0, 0] for n in outs]},
                       "keras_version": "2.15.0", "backend": "tensorflow"})
