"""`Model`: a graph + its weights, with the slice of the Keras Model API the
reference uses (`get_layer`, `layers`, `input`/`output`, `get_weights`,
`set_weights`, `to_json`, `summary`, `predict`, `count_params`;
`src/dispatcher.py:43-48,235-243`, `test/test.py:13-14`)."""
from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np

from ..graph.ir import Graph, Layer


class Model:
    def __init__(self, graph: Graph, weights: Dict[str, np.ndarray], name: Optional[str] = None):
        self.graph = graph
        self.weights = weights
        self.name = name or graph.name
        self._executors = {}

    # ------------------------------------------------ Keras-like surface
    @property
    def layers(self) -> List[Layer]:
        return [self.graph.layers[n] for n in self.graph.order]

    def get_layer(self, name: str) -> Layer:
        return self.graph.get_layer(name)

    @property
    def input(self) -> str:
        return self.graph.input

    @property
    def output(self) -> str:
        return self.graph.output

    def get_weights(self) -> List[np.ndarray]:
        return [self.weights[n] for n, _ in self.graph.weight_specs()]

    def set_weights(self, arrays: List[np.ndarray]) -> None:
        from .resnet import set_weights
        self.weights = set_weights(self.graph, arrays)
        self._executors.clear()

    def to_json(self) -> str:
        return self.graph.to_json()

    def to_keras_json(self) -> str:
        """Keras functional-model JSON (what the reference's `model.to_json()` ships)."""
        from ..graph.keras_json import to_keras_json
        return to_keras_json(self.graph)

    @staticmethod
    def from_keras_json(s, weights=None, seed: int = 0) -> "Model":
        """`tf.keras.models.model_from_json` analogue (`src/node.py:40,77`): a Keras
        JSON architecture plus, optionally, its `get_weights()` list (or a
        name -> array dict); random-init (seeded) when no weights are given."""
        from ..graph.keras_json import from_keras_json
        from .resnet import init_weights, set_weights
        g = from_keras_json(s)
        if weights is None:
            w = init_weights(g, seed)
        elif isinstance(weights, dict):
            w = dict(weights)
        else:
            w = set_weights(g, list(weights))
        return Model(g, w)

    def plot_model(self, to_file: str = "model.png", show_shapes: bool = True) -> str:
        """`tf.keras.utils.plot_model` analogue (`src/node.py:49`): DOT source, rendered when Graphviz is present."""
        from ..utils.plot import plot_model
        return plot_model(self, to_file, show_shapes)

    def summary(self, print_fn=print) -> str:
        s = self.graph.summary()
        if print_fn:
            print_fn(s)
        return s

    def count_params(self) -> int:
        return self.graph.count_params()

    # ------------------------------------------------------------ compute
    def predict(self, x: np.ndarray, device: Optional[str] = None, batch: Optional[int] = None,
                precision: str = "fp32") -> np.ndarray:
        """Single-device inference (`test/local_infer.py:22`): our HIP runtime on
        a GPU (precision "bf16" or "fp32", the reference's Keras float32), the
        native OpenMP fp32 path on CPU.  Inputs are NHWC float32 images."""
        import torch
        x = np.asarray(x, np.float32)
        if device is None:
            device = "cuda" if torch.cuda.is_available() else "cpu"
        if device == "cpu":
            # the native OpenMP path (runtime/cpu_executor.py); PyTorch is only the test oracle
            from ..runtime.cpu_executor import CpuExecutor
            ex = self._executors.get("cpu")
            if ex is None:
                ex = self._executors["cpu"] = CpuExecutor(self.graph, self.weights)
            return ex(x)
        from ..runtime.executor import SliceExecutor
        b = batch or x.shape[0]
        key = (device, b, precision)
        ent = self._executors.get(key)
        if ent is None:
            # one hipGraph per (device, batch) and a pinned result buffer: a request is
            # H2D -> graph replay -> async D2H -> one sync (the reference re-enters TF's
            # per-layer dispatch on every `model.predict`, test/local_infer.py:22)
            ex = SliceExecutor(self.graph, self.weights, b, device=device, precision=precision)
            ex.capture()
            yout = ex.output_buf(ex.outputs[0])
            ent = self._executors[key] = (ex, torch.empty(yout.shape, dtype=yout.dtype, pin_memory=True))
        ex, hout = ent
        xin = ex.input_buf(self.graph.input)
        outs = []
        for i in range(0, x.shape[0], b):
            chunk = x[i:i + b]
            n = chunk.shape[0]
            if n < b:
                chunk = np.concatenate([chunk, np.zeros((b - n,) + chunk.shape[1:], np.float32)])
            xin.copy_(torch.from_numpy(np.ascontiguousarray(chunk)))     # straight from the caller's array
            y = ex.forward(0)[ex.outputs[0]]
            hout.copy_(y, non_blocking=True)
            torch.cuda.current_stream(ex.device).synchronize()
            outs.append(hout[:n].float().numpy().copy())
        return np.concatenate(outs)

    def __call__(self, x, **kw):
        return self.predict(x, **kw)


def resnet(depth: str = "resnet50", seed: int = 0, weights: Optional[Dict[str, np.ndarray]] = None, **kw) -> Model:
    """`ResNet50(weights=...)` analogue: random-init (seeded) or given weights.
    Any family of `models/zoo.py` is accepted by name too (vgg16, mobilenet_v2, densenet121, ...)."""
    from .resnet import init_weights
    from .zoo import build_model
    g = build_model(depth, **kw)
    return Model(g, weights if weights is not None else init_weights(g, seed))


def application(name: str, seed: int = 0, weights: Optional[Dict[str, np.ndarray]] = None, **kw) -> Model:
    """`tf.keras.applications.<Name>(...)` analogue for every family we build."""
    return resnet(name, seed=seed, weights=weights, **kw)
