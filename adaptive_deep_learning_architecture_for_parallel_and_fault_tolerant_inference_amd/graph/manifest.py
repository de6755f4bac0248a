"""Slice ("checkpoint") format: manifest + ordered weight list, on the wire and on disk.

Reference format (`src/dispatcher.py:223-264`, `src/node.py:65-119`), per slice:

1. framed UTF-8 Keras JSON architecture,
2. framed ASCII partition index (sent with chunk_size=1),
3. u64 big-endian weight-array count,
4. per array: framed ``lz4(zfp(ndarray))`` in Keras ``get_weights()`` order,
5. one ACK byte ``0x06`` back from the worker.

We keep that information content and order: a JSON manifest (our graph IR
of the slice + frontier tensor specs + per-array name/shape/dtype/xxh32), the
ASCII index, the count and the encoded arrays (codec selectable, reference
default ``zfp+lz4``), then the ACK.  On disk a slice is ``<name>.json`` +
``<name>.safetensors`` (loaded with the non-executing safetensors loader).
"""
from __future__ import annotations

import json
import os
import socket
import struct
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np

from .. import codec as codec_mod
from ..native import runtime
from ..node_state import socket_recv, socket_send
from .ir import Graph
from .slicer import Slice, subgraph

ACK = b"\x06"
NAK = b"\x15"
FORMAT = "adapt-slice-v1"


@dataclass
class SliceManifest:
    model: str
    part_index: int                 # 1-based like the reference ("part{p+1}")
    part_name: str
    graph_json: str                 # sub-graph (inputs are 'input' layers named after frontier tensors)
    inputs: List[Dict]              # [{"name", "shape", "dtype"}] per image
    outputs: List[Dict]
    weights: List[Dict] = field(default_factory=list)   # [{"name","shape","dtype","xxh32"}] get_weights() order
    start: str = ""
    end: str = ""
    extra: Dict = field(default_factory=dict)

    def to_json(self) -> str:
        return json.dumps({"format": FORMAT, "model": self.model, "part_index": self.part_index,
                           "part_name": self.part_name, "graph": json.loads(self.graph_json),
                           "inputs": self.inputs, "outputs": self.outputs, "weights": self.weights,
                           "start": self.start, "end": self.end, "extra": self.extra})

    @staticmethod
    def from_json(s) -> "SliceManifest":
        d = json.loads(s)
        if d.get("format") != FORMAT:
            raise ValueError(f"not an {FORMAT} manifest")
        return SliceManifest(d["model"], d["part_index"], d["part_name"], json.dumps(d["graph"]), d["inputs"],
                             d["outputs"], d.get("weights", []), d.get("start", ""), d.get("end", ""),
                             d.get("extra", {}))

    def graph(self) -> Graph:
        return Graph.from_json(self.graph_json)

    @property
    def weight_names(self) -> List[str]:
        return [w["name"] for w in self.weights]


def _tensor_spec(g: Graph, name: str) -> Dict:
    L = g.layers[name]
    dtype = "float32" if (name in g.input_names or L.op in ("dense", "softmax")) else "bfloat16"
    return {"name": name, "shape": list(L.out_shape), "dtype": dtype}


def build_manifest(g: Graph, s: Slice, weights: Dict[str, np.ndarray]) -> (SliceManifest, List[np.ndarray]):
    sg = subgraph(g, s)
    arrays = []
    wspecs = []
    for name, shp in g.weight_specs(s.layers):
        a = np.require(weights[name], np.float32, ["C"])       # (ascontiguousarray makes 0-d 1-d)
        if tuple(a.shape) != tuple(shp):
            raise ValueError(f"{name}: shape {a.shape} != {shp}")
        arrays.append(a)
        wspecs.append({"name": name, "shape": list(shp), "dtype": "float32",
                       "xxh32": int(runtime().xxh32(a.reshape(-1).view(np.uint8)))})
    m = SliceManifest(g.name, s.index + 1, s.name, sg.to_json(),
                      [_tensor_spec(g, t) for t in s.inputs], [_tensor_spec(g, t) for t in s.outputs],
                      wspecs, s.start, s.end)
    return m, arrays


def verify_arrays(m: SliceManifest, arrays: Sequence[np.ndarray]) -> None:
    if len(arrays) != len(m.weights):
        raise ValueError(f"expected {len(m.weights)} arrays, got {len(arrays)}")
    for spec, a in zip(m.weights, arrays):
        if list(a.shape) != list(spec["shape"]):
            raise ValueError(f"{spec['name']}: shape {a.shape} != {spec['shape']}")
        h = int(runtime().xxh32(np.require(a, None, ["C"]).reshape(-1).view(np.uint8)))
        if "xxh32" in spec and h != spec["xxh32"]:
            raise ValueError(f"{spec['name']}: checksum mismatch")


def arrays_to_dict(m: SliceManifest, arrays: Sequence[np.ndarray]) -> Dict[str, np.ndarray]:
    return {spec["name"]: a for spec, a in zip(m.weights, arrays)}


# ------------------------------------------------------------------- wire
def send_weights(weights: Sequence[np.ndarray], sock: socket.socket, chunk_size: int, codec: str = "zfp+lz4") -> None:
    """u64 BE count + one framed encoded array each (`src/dispatcher.py:76-89`)."""
    runtime().send_all(sock.fileno(), struct.pack(">Q", len(weights)), 8, -1)
    for a in weights:
        socket_send(codec_mod.encode(a, codec), sock, chunk_size)


def recv_weights(sock: socket.socket, chunk_size: int) -> List[np.ndarray]:
    hdr = runtime().recv_exact(sock.fileno(), 8, -1)
    if hdr is None:
        raise ConnectionError("closed before weight count")
    (n,) = struct.unpack(">Q", hdr)
    out = []
    for _ in range(n):
        buf = socket_recv(sock, chunk_size)
        if not buf:
            raise ConnectionError("closed inside weight list")
        out.append(codec_mod.decode(buf))
    return out


def send_slice(sock: socket.socket, m: SliceManifest, arrays: Sequence[np.ndarray], chunk_size: int = 512000,
               codec: str = "zfp+lz4") -> None:
    socket_send(m.to_json().encode(), sock, chunk_size)
    socket_send(str(m.part_index).encode(), sock, 1)          # reference sends the index with chunk_size=1
    send_weights(arrays, sock, chunk_size, codec)


def recv_slice(sock: socket.socket, chunk_size: int = 512000):
    mj = socket_recv(sock, chunk_size)
    if not mj:
        raise ConnectionError("closed before manifest")
    idx = socket_recv(sock, 1)
    if not idx:
        raise ConnectionError("closed before partition index")
    m = SliceManifest.from_json(mj)
    if int(idx.decode()) != m.part_index:
        raise ValueError("partition index does not match manifest")
    arrays = recv_weights(sock, chunk_size)
    verify_arrays(m, arrays)
    return m, arrays


# ------------------------------------------------------------------- disk
def save_slice(path_prefix: str, m: SliceManifest, arrays: Sequence[np.ndarray]) -> None:
    from safetensors.numpy import save_file
    os.makedirs(os.path.dirname(os.path.abspath(path_prefix)), exist_ok=True)
    with open(path_prefix + ".json", "w") as f:
        f.write(m.to_json())
    save_file({f"{i:05d}": np.require(a, None, ["C"]) for i, a in enumerate(arrays)}, path_prefix + ".safetensors",
              metadata={"format": FORMAT, "order": json.dumps(m.weight_names)})


def load_slice(path_prefix: str):
    from safetensors.numpy import load_file
    with open(path_prefix + ".json") as f:
        m = SliceManifest.from_json(f.read())
    t = load_file(path_prefix + ".safetensors")
    arrays = [t[f"{i:05d}"] for i in range(len(m.weights))]
    verify_arrays(m, arrays)
    return m, arrays


def save_model(path: str, g: Graph, weights: Dict[str, np.ndarray]) -> None:
    """Whole-model checkpoint: graph JSON + safetensors in get_weights() order."""
    from safetensors.numpy import save_file
    with open(path + ".graph.json", "w") as f:
        f.write(g.to_json())
    names = [n for n, _ in g.weight_specs()]
    save_file({n: np.require(weights[n], np.float32, ["C"]) for n in names}, path + ".safetensors",
              metadata={"format": "adapt-model-v1"})


def load_model(path: str):
    from safetensors.numpy import load_file
    with open(path + ".graph.json") as f:
        g = Graph.from_json(f.read())
    return g, dict(load_file(path + ".safetensors"))


def load_keras_weight_list(g: Graph, path: str) -> Dict[str, np.ndarray]:
    """Map a Keras `model.get_weights()` list saved as .npz (arr_0..arr_N, no
    pickles: allow_pickle=False) onto our layer names."""
    from ..models.resnet import set_weights
    with np.load(path, allow_pickle=False) as z:
        keys = sorted(z.files, key=lambda k: int(k.split("_")[-1]) if k.split("_")[-1].isdigit() else k)
        arrays = [z[k] for k in keys]
    return set_weights(g, arrays)
