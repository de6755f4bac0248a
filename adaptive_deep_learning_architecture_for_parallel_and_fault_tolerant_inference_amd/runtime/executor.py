"""Slice executor: compiled plan + packed weights + static buffers + hipGraphs.

The reference's worker hot loop is `to_send.get() -> model.predict(inpt)`
(`src/node.py:173-179`): TF re-dispatches ~177 ops per request from Python.
Here a slice is compiled once for a fixed micro-batch:

1. `compile_plan` fuses Keras layers into kernel steps (runtime/plan.py);
2. conv weights are BN-folded and packed to bf16 ``[Npad][Kpad]`` once and
   stay resident in HBM (repartition = pointer swap);
3. activations get liveness-reused static buffers (an R50 bs=32 slice's
   working set stays inside the 256 MiB Infinity Cache);
4. the step list is captured into one hipGraph per *buffer set* and replayed
   per micro-batch.  ``num_sets=2`` double-buffers the slice's frontier
   inputs/outputs so RCCL receives the next micro-batch and sends the
   previous one while this one computes (parallel/pipeline.py).

All compute goes through our gfx950 kernels (ops/*.py); torch provides the
allocator and the stream / graph API only.
"""
from __future__ import annotations

import json
import math
import os
import threading
from collections import ChainMap
from pathlib import Path
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..graph.ir import Graph, bn_params
from ..ops import conv as conv_ops
from ..ops import eltwise as E
from ..ops._lib import private_stream
from .plan import Step, compile_plan

TUNING_FILE = Path(__file__).resolve().parent.parent / "tuning" / "gfx950_conv.json"
_tuning_lock = threading.Lock()
_tuning_cache: Optional[Dict[str, List]] = None


def load_tuning() -> Dict[str, List]:
    global _tuning_cache
    with _tuning_lock:
        if _tuning_cache is None:
            try:
                _tuning_cache = json.loads(TUNING_FILE.read_text())
            except (OSError, ValueError):
                _tuning_cache = {}
        return _tuning_cache


def save_tuning(entries: Dict[str, List]) -> None:
    global _tuning_cache
    with _tuning_lock:
        cur = {}
        try:
            cur = json.loads(TUNING_FILE.read_text())
        except (OSError, ValueError):
            pass
        cur.update(entries)
        TUNING_FILE.parent.mkdir(parents=True, exist_ok=True)
        TUNING_FILE.write_text(json.dumps(cur, indent=1, sort_keys=True))
        _tuning_cache = cur


def conv_key(B, H, W, Cin, pc) -> str:
    return f"{B}x{H}x{W}x{Cin}|{pc.kh}x{pc.kw}s{pc.stride}p{pc.pad_t}{pc.pad_l}{pc.pad_b}{pc.pad_r}|{pc.cout}"


def _nbytes(shape, dtype) -> int:
    return int(np.prod(shape)) * torch.empty((), dtype=dtype).element_size()


class SliceExecutor:
    """Runs one (sub)graph for a fixed batch on one device with our HIP kernels."""

    FP32_KINDS = ("conv", "pair", "dense", "maxpool", "gap", "softmax", "add", "bn", "relu", "pad", "copy",
                  "dwconv", "avgpool", "concat", "act", "binary", "affine", "stem_f32")

    def __init__(self, g: Graph, weights: Dict[str, np.ndarray], batch: int, device="cuda",
                 outputs: Optional[Sequence[str]] = None, tune: bool = False, num_sets: int = 1,
                 precision: str = "fp32", private_sets: bool = False):
        """precision: "bf16" (bf16 activations / weights, fp32 accumulation: the
        fast path) or "fp32" (fp32 activations and weights on the fp32 matrix
        cores: the reference's Keras float32 numerics, csrc/kernels/conv_f32.hip).
        private_sets: every buffer set also gets its own internal activation arena
        and scratch (split-K workspace, stream-K counters, head / GAP partials), so
        the sets' graphs may replay concurrently on different streams (a serving
        stage keeps two micro-batches in flight); by default the sets share them
        and replay one after the other."""
        if precision not in ("bf16", "fp32"):
            raise ValueError(f"precision must be bf16 or fp32, got {precision!r}")
        self.g = g
        self.batch = batch
        self.device = torch.device(device)
        self.outputs = list(outputs or g.output_names)
        self.num_sets = num_sets
        self.private_sets = bool(private_sets) and num_sets > 1
        self.precision = precision
        self.fp32 = precision == "fp32"
        self.steps: List[Step] = compile_plan(g, self.outputs, fp32=self.fp32)
        if self.fp32:
            bad = sorted({st.kind for st in self.steps if st.kind not in self.FP32_KINDS})
            if bad:
                raise NotImplementedError(f"fp32 execution has no kernels for {bad} (model {g.name})")
        self._graphs: List[Optional[torch.cuda.CUDAGraph]] = [None] * num_sets
        self._pack_weights(weights)
        self._alloc()
        self._select_configs(tune)

    # ------------------------------------------------------------ shapes
    def shape_of(self, name: str) -> Tuple[int, ...]:
        base = name.split("#")[0]
        shp = tuple(self.g.layers[base].out_shape)
        # activations are stored with channels padded to a multiple of 8 (16-byte
        # vectors); only the user's fp32 image keeps its true channel count
        if len(shp) == 3 and shp[-1] % 8 and self.dtype_of(name) != torch.float32 and not self.fp32:
            shp = shp[:-1] + (((shp[-1] + 7) // 8) * 8,)
        return (self.batch,) + shp

    def dtype_of(self, name: str):
        if self.fp32:
            return torch.float32
        base = name.split("#")[0]
        L = self.g.layers[base]
        if (L.op == "input" and base == name and len(L.out_shape) == 3
                and L.attrs.get("stands_for", "input") == "input"):
            return torch.float32          # user image input (Keras float32 NHWC)
        if L.op == "softmax" or (L.op == "dense" and L.attrs.get("activation") in (None, "linear", "softmax")):
            return torch.float32          # logits / probabilities; a Dense(relu, ...) feeds the next GEMM in bf16
        return torch.bfloat16

    # ----------------------------------------------------------- weights
    def _pack_weights(self, weights: Dict[str, np.ndarray]) -> None:
        self.packed: Dict[int, object] = {}
        dev = self.device
        if self.fp32:
            self._pack_weights_f32(weights)
            return
        for i, st in enumerate(self.steps):
            if st.kind == "conv":
                p = st.p
                kf, bf = self._folded(weights, p)
                cin_pad = ((kf.shape[2] + 7) // 8) * 8
                if kf.shape[-1] % 8 and not p.get("sibling"):
                    # output channels padded to the 16-byte activation layout with zero filters
                    # (EfficientNet's 4- / 6-channel squeeze-excite convs)
                    extra = 8 - kf.shape[-1] % 8
                    kf = np.concatenate([kf, np.zeros(kf.shape[:3] + (extra,), kf.dtype)], axis=-1)
                    bf = np.concatenate([bf, np.zeros(extra, bf.dtype)])
                n_split = 0
                if p.get("sibling"):                  # merged sibling convs: one GEMM, N = N0 + N1
                    k2, b2 = self._folded(weights, p["sibling"])
                    n_split = kf.shape[-1]
                    kf, bf = np.concatenate([kf, k2], axis=-1), np.concatenate([bf, b2])
                pc = conv_ops.pack_conv(kf, bf, p["stride"], p["pads"], dev, cin_pad=cin_pad)
                pc.n_split = n_split
                self.packed[i] = pc
            elif st.kind == "bottleneck":
                p = st.p
                k1, b1 = self._folded(weights, p["c1"])
                k2, b2 = self._folded(weights, p["c2"])
                k3, b3 = self._folded(weights, p["c3"])
                kp = bp = None
                if p["proj"] is not None:
                    kp, bp = self._folded(weights, p["proj"])
                self.packed[i] = conv_ops.pack_bottleneck(k1, b1, k2, b2, k3, b3, kp, bp, device=dev)
            elif st.kind == "pair":
                p = st.p
                k3, b3 = self._folded(weights, p["c3"])
                k1, b1 = self._folded(weights, p["c1"])
                self.packed[i] = conv_ops.pack_pair(k3, b3, k1, b1, device=dev)
            elif st.kind == "stem":
                p = st.p
                k = weights[f"{p['conv']}/kernel"]
                bn = None
                eps = 1e-3
                if p["bn"]:
                    bn = bn_params(weights, p["bn"])
                    eps = self.g.layers[p["bn"]].attrs.get("epsilon", 1e-3)
                kf, bf = conv_ops.fold_bn(k, weights.get(f"{p['conv']}/bias"), bn, eps)
                self.packed[i] = conv_ops.pack_stem(kf, bf, p["pads"], dev)
            elif st.kind == "dense":
                name = st.p.get("layer", st.out)
                k = weights[f"{name}/kernel"]                     # (in, out)
                b = weights.get(f"{name}/bias", np.zeros(k.shape[1], np.float32))
                self.packed[i] = conv_ops.pack_conv(k.reshape(1, 1, k.shape[0], k.shape[1]), b, 1,
                                                    ((0, 0), (0, 0)), dev)
            elif st.kind == "dwconv":
                p = st.p
                k = weights[f"{p['conv']}/depthwise_kernel"][..., 0]          # (kh, kw, C), multiplier 1
                bn = None
                eps = 1e-3
                if p["bn"]:
                    bn = bn_params(weights, p["bn"])
                    eps = self.g.layers[p["bn"]].attrs.get("epsilon", 1e-3)
                # as an HWIO kernel with one input channel: BN scales the last (channel) axis
                kf, bf = conv_ops.fold_bn(k[:, :, None, :], weights.get(f"{p['conv']}/bias"), bn, eps)
                kf = kf[:, :, 0, :]
                cp = ((kf.shape[-1] + 7) // 8) * 8
                wp = np.zeros(kf.shape[:2] + (cp,), np.float32)
                wp[..., :kf.shape[-1]] = kf
                bp = np.zeros(cp, np.float32)
                bp[:bf.shape[0]] = bf
                self.packed[i] = (torch.tensor(wp, device=dev), torch.tensor(bp, device=dev))
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
                cp = ((c + 7) // 8) * 8
                scp, shp = np.zeros(cp, np.float32), np.zeros(cp, np.float32)   # padding channels stay 0
                scp[:c], shp[:c] = sc, sh
                self.packed[i] = (torch.tensor(scp, device=dev), torch.tensor(shp, device=dev))
            elif st.kind == "bn":
                name = st.p["bn"]
                bp_ = bn_params(weights, name)
                gm, bt, mu, var = (np.asarray(bp_[n], np.float64) for n in
                                   ("gamma", "beta", "moving_mean", "moving_variance"))
                eps = self.g.layers[name].attrs.get("epsilon", 1e-3)
                s = gm / np.sqrt(var + eps)
                self.packed[i] = (torch.tensor(s, dtype=torch.float32, device=dev),
                                  torch.tensor(bt - mu * s, dtype=torch.float32, device=dev))

    def _pack_weights_f32(self, weights: Dict[str, np.ndarray]) -> None:
        dev = self.device
        for i, st in enumerate(self.steps):
            if st.kind == "conv":
                kf, bf = self._folded(weights, st.p)
                n_split = 0
                if st.p.get("sibling"):                # merged sibling 1x1 convs: one GEMM, N = N0 + N1
                    k2, b2 = self._folded(weights, st.p["sibling"])
                    n_split = kf.shape[-1]
                    kf, bf = np.concatenate([kf, k2], axis=-1), np.concatenate([bf, b2])
                self.packed[i] = conv_ops.pack_conv_f32(kf, bf, st.p["stride"], st.p["pads"], dev)
                self.packed[i].n_split = n_split
            elif st.kind == "stem_f32":
                kf, bf = self._folded(weights, st.p)
                self.packed[i] = conv_ops.pack_stem_f32(kf, bf, st.p["pads"], dev)
            elif st.kind == "pair":
                k3, b3 = self._folded(weights, st.p["c3"])
                k1, b1 = self._folded(weights, st.p["c1"])
                self.packed[i] = conv_ops.pack_pair_f32(k3, b3, k1, b1, device=dev)
            elif st.kind == "dense":
                name = st.p.get("layer", st.out)
                k = weights[f"{name}/kernel"]
                b = weights.get(f"{name}/bias", np.zeros(k.shape[1], np.float32))
                self.packed[i] = conv_ops.pack_conv_f32(k.reshape(1, 1, k.shape[0], k.shape[1]), b, 1,
                                                        ((0, 0), (0, 0)), dev)
            elif st.kind == "bn":
                bp_ = bn_params(weights, st.p["bn"])
                gm, bt, mu, var = (np.asarray(bp_[n], np.float64) for n in
                                   ("gamma", "beta", "moving_mean", "moving_variance"))
                eps = self.g.layers[st.p["bn"]].attrs.get("epsilon", 1e-3)
                sc = gm / np.sqrt(var + eps)
                self.packed[i] = (torch.tensor(sc, dtype=torch.float32, device=dev),
                                  torch.tensor(bt - mu * sc, dtype=torch.float32, device=dev))
            elif st.kind == "dwconv":
                p = st.p
                k = weights[f"{p['conv']}/depthwise_kernel"][..., 0]          # (kh, kw, C), multiplier 1
                bn = None
                eps = 1e-3
                if p["bn"]:
                    bn = bn_params(weights, p["bn"])
                    eps = self.g.layers[p["bn"]].attrs.get("epsilon", 1e-3)
                kf, bf = conv_ops.fold_bn(k[:, :, None, :], weights.get(f"{p['conv']}/bias"), bn, eps)
                self.packed[i] = (torch.tensor(np.ascontiguousarray(kf[:, :, 0, :]), dtype=torch.float32, device=dev),
                                  torch.tensor(bf, dtype=torch.float32, device=dev))
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
                self.packed[i] = (torch.tensor(np.ascontiguousarray(sc), dtype=torch.float32, device=dev),
                                  torch.tensor(np.ascontiguousarray(sh), dtype=torch.float32, device=dev))

    def _folded(self, weights: Dict[str, np.ndarray], p: Dict):
        """BN-folded (kernel HWIO, bias) of a conv step's parameters."""
        cname = p["conv"]
        bn = None
        eps = 1e-3
        if p["bn"]:
            bn = bn_params(weights, p["bn"])
            eps = self.g.layers[p["bn"]].attrs.get("epsilon", 1e-3)
        return conv_ops.fold_bn(weights[f"{cname}/kernel"], weights.get(f"{cname}/bias"), bn, eps)

    # ----------------------------------------------------------- buffers
    def _alloc(self) -> None:
        """Per-set frontier buffers + liveness-reused internal activation buffers."""
        dev = self.device
        in_names = list(self.g.input_names)
        # relay outputs (slice inputs forwarded unchanged) get their own output buffers
        self.relay = [o for o in self.outputs if o in in_names]
        self.sets: List[Dict[str, torch.Tensor]] = []
        for _ in range(self.num_sets):
            s = {}
            for n in in_names:
                s[n] = torch.zeros(self.shape_of(n), dtype=self.dtype_of(n), device=dev)
            for o in self.outputs:
                key = o + "#out" if o in in_names else o
                s[key] = torch.empty(self.shape_of(o), dtype=self.dtype_of(o), device=dev)
            self.sets.append(s)
        self._alloc_private()
        self._priv: List[Dict[str, object]] = []
        self._bound = 0
        if self.private_sets:
            self._priv.append(self._private_state())
            for _ in range(1, self.num_sets):
                self._alloc_private()
                self._priv.append(self._private_state())
            self._bound = self.num_sets - 1        # the live attributes are the last set's
            self._bind(0)

    _PRIVATE = ("internal", "_arena", "_logits", "_dense_part", "_gap_part", "_ws", "_ctr", "_ws_side", "_ctr_side")

    def _private_state(self) -> Dict[str, object]:
        return {k: getattr(self, k) for k in self._PRIVATE}

    def _bind(self, set_idx: int) -> None:
        """private_sets: make set `set_idx`'s arena and scratch the current ones (the
        bound set's workspace, possibly grown meanwhile by _ensure_ws, is saved first)."""
        if not self.private_sets:
            return
        self._priv[self._bound].update(self._private_state())
        for k, v in self._priv[set_idx].items():
            setattr(self, k, v)
        self._bound = set_idx

    def _alloc_private(self) -> None:
        """The internal activation arena and the per-launch scratch of one set (or
        of all sets together, without private_sets)."""
        dev = self.device
        keep = set(self.outputs)
        last_use: Dict[str, int] = {}
        for i, st in enumerate(self.steps):
            for t in st.ins:
                last_use[t] = i
        # independent branches run on a side stream: their inputs stay live until the join
        self._side = self._side_schedule()
        for i, j in self._side.items():
            for t in self.steps[i].ins:
                last_use[t] = max(last_use.get(t, j), j)
        owner: Dict[str, torch.Tensor] = {}          # internal tensor -> arena block backing it
        free: List[torch.Tensor] = []
        self.internal: Dict[str, torch.Tensor] = {}
        self._arena: List[torch.Tensor] = []
        for i, st in enumerate(self.steps):
            for name in [st.out] + ([st.p["out2"]] if st.p.get("out2") else []):
                if name in keep:
                    continue
                shp, dt = self.shape_of(name), self.dtype_of(name)
                nb = _nbytes(shp, dt)
                cand = [k for k, b in enumerate(free) if b.numel() >= nb]
                if cand:
                    k = min(cand, key=lambda q: free[q].numel())
                    b = free.pop(k)
                else:
                    b = torch.empty(max(nb, 1 << 16), dtype=torch.uint8, device=dev)
                    self._arena.append(b)
                self.internal[name] = b[:nb].view(dt).view(shp)
                owner[name] = b
            for tname in set(st.ins):
                if last_use.get(tname) == i and tname not in keep and tname in owner:
                    free.append(owner.pop(tname))
        self._logits: Dict[int, torch.Tensor] = {}
        self._dense_part: Dict[int, torch.Tensor] = {}
        for i, st in enumerate(self.steps):
            if (st.kind == "dense" and self.batch <= 32 and not st.p.get("relu") and not self.fp32
                    and self.dtype_of(st.out) == torch.float32):          # head.hip writes fp32 logits / probs
                # small-M head GEMM (csrc/kernels/head.hip): split-K scratch
                pc = self.packed[i]
                n = E.dense_small_scratch(self.batch, pc.cout, pc.K)
                self._dense_part[i] = torch.empty(n, dtype=torch.float32, device=dev)
            elif (st.kind == "dense" and self.batch <= 32 and not st.p.get("relu") and self.fp32
                  and self.device.type == "cuda" and os.environ.get("ADAPT_F32_HEAD", "1") == "1"):
                # fp32 small-M head (head.hip dense_partial_f32_kernel + finish): logits + softmax in 2 launches
                pc = self.packed[i]
                self._dense_part[i] = torch.empty(E.dense_small_f32_scratch(self.batch, pc.cout, pc.Kpad),
                                                  dtype=torch.float32, device=dev)
            if st.kind == "dense" and st.p["softmax"]:
                # pre-softmax logits stay readable (`logits()`): numerics checks compare them
                self._logits[i] = torch.empty((self.batch, st.p["units"]), dtype=torch.float32, device=dev)
        self._gap_part: Dict[int, torch.Tensor] = {}
        for i, st in enumerate(self.steps):
            if st.kind == "gap" and self.device.type == "cuda":
                shp = self.shape_of(st.ins[0])
                if len(shp) == 4:
                    need = E.gap_scratch_elems(shp[0], shp[1] * shp[2], shp[3])
                    if need:
                        self._gap_part[i] = torch.empty(need, dtype=torch.float32, device=dev)
        self._ws: Optional[torch.Tensor] = None
        self._ctr: Optional[torch.Tensor] = None
        self._ws_side: Optional[torch.Tensor] = None
        self._ctr_side: Optional[torch.Tensor] = None
        if not hasattr(self, "_side_stream"):
            self._side_stream: Optional[torch.cuda.Stream] = None

    def _side_schedule(self) -> Dict[int, int]:
        """{step i: join step j} for convs that form an independent branch: the
        first of several consumers of their input whose only consumer comes
        later than the next step (ResNet: the projection shortcut X_0 of each
        stage's first block runs beside X_1 -> X_2 and joins at X_3's residual
        add).  Run on a second HIP stream inside the same hipGraph.

        Opt-in (ADAPT_BRANCH_STREAMS=1): measured on MI355X at bs=32 the
        concurrent branch slows the slice down (0.877 vs 0.815 ms/batch): both
        sides are bandwidth-bound and the shortcut conv steals the CUs the
        critical path needs."""
        if self.device.type != "cuda" or os.environ.get("ADAPT_BRANCH_STREAMS", "0") != "1":
            return {}
        cons: Dict[str, List[int]] = {}
        for i, st in enumerate(self.steps):
            for t in set(st.ins):
                cons.setdefault(t, []).append(i)
        side: Dict[int, int] = {}
        for i, st in enumerate(self.steps):
            if st.kind != "conv" or st.out in self.outputs or st.p.get("out2"):
                continue
            c_in = cons.get(st.ins[0], [])
            users = cons.get(st.out, [])
            if len(c_in) >= 2 and c_in[0] == i and len(users) == 1 and users[0] > i + 1:
                side[i] = users[0]
        return side

    def bufs(self, set_idx: int = 0):
        internal = self._priv[set_idx]["internal"] if self.private_sets and set_idx != self._bound else self.internal
        return ChainMap(self.sets[set_idx], internal)

    @property
    def inputs(self) -> Dict[str, torch.Tensor]:
        return {n: self.sets[0][n] for n in self.g.input_names}

    def input_buf(self, name: str, set_idx: int = 0) -> torch.Tensor:
        return self.sets[set_idx][name]

    def output_buf(self, name: str, set_idx: int = 0) -> torch.Tensor:
        s = self.sets[set_idx]
        return s[name + "#out"] if name in self.relay else s[name]

    def workspace_bytes(self) -> int:
        arenas = [p["_arena"] for p in self._priv] if self.private_sets else [self._arena]
        n = sum(b.numel() for a in arenas for b in a)
        n += sum(t.numel() * t.element_size() for s in self.sets for t in s.values())
        return n

    # ---------------------------------------------------- tile configs
    def _conv_geom(self, i: int):
        st = self.steps[i]
        x = self.bufs(0)[st.ins[0]]
        if st.kind == "dense":                     # a GEMM over the flattened input (Flatten aliases into it)
            x = x.reshape(self.batch, -1)
        if x.dim() == 2:
            B, H, W, C = x.shape[0], 1, 1, x.shape[1]
        else:
            B, H, W, C = x.shape
        pc = self.packed[i]
        OH, OW = pc.out_hw(H, W)
        return B, H, W, C, OH, OW, pc

    def _ensure_ws(self) -> None:
        need = ctr = 0
        for i, (cfg, ks) in self.cfg.items():
            if self.fp32:
                if cfg in conv_ops.WINO4S_F32_CFGS:        # V and the split-K partials, whatever the split
                    B, H, W, C, OH, OW, pc = self._conv_geom(i)
                    need = max(need, conv_ops.wino4s_ws_elems(B, H, W, C, pc.cout, ks))
                    ctr = max(ctr, conv_ops.f32_counter_elems(cfg, ks, B, H, W, OH, OW, pc.cout, pc.Kpad))
                    continue
                if ks != 1:
                    B, H, W, C, OH, OW, pc = self._conv_geom(i)
                    need = max(need, conv_ops.workspace_elems_f32(B * OH * OW, pc.cout, pc.Kpad, cfg, ks))
                    ctr = max(ctr, conv_ops.f32_counter_elems(cfg, ks, B, H, W, OH, OW, pc.cout, pc.Kpad))
                continue
            if ks != 1:
                B, H, W, C, OH, OW, pc = self._conv_geom(i)
                need = max(need, conv_ops.workspace_elems(B * OH * OW, pc.cout, pc.Kpad, cfg, ks))
                if ks < 0:
                    ctr = max(ctr, conv_ops.sk_plan(B * OH * OW, pc.cout, pc.Kpad, cfg, -ks)[0])
        if need and (self._ws is None or self._ws.numel() < need):
            self._ws = torch.empty(need, dtype=torch.float32, device=self.device)
            if self._side:                     # side-stream convs must not share scratch with the main stream
                self._ws_side = torch.empty(need, dtype=torch.float32, device=self.device)
        if ctr and (self._ctr is None or self._ctr.numel() < ctr):
            # stream-K arrival counters: zero once, every launch leaves them zero
            self._ctr = torch.zeros(ctr, dtype=torch.int32, device=self.device)
            if self._side:
                self._ctr_side = torch.zeros(ctr, dtype=torch.int32, device=self.device)

    def _select_configs(self, tune: bool) -> None:
        table = load_tuning()
        self.cfg: Dict[int, Tuple[int, int]] = {}
        for i, st in enumerate(self.steps):
            if st.kind not in ("conv", "dense") or i in self._dense_part:    # small-M heads: head.hip
                continue
            B, H, W, C, OH, OW, pc = self._conv_geom(i)
            if self.fp32:
                key = "f32|" + conv_key(B, H, W, C, pc)
                cfg, ks = table[key][:2] if key in table else conv_ops.choose_cfg_f32(B * OH * OW, pc.cout, pc.Kpad)
                self.cfg[i] = (int(cfg), int(ks))
                continue
            if pc.cout % 8:
                raise NotImplementedError(f"{st.kind} {st.out}: {pc.cout} output channels (the MFMA GEMM path "
                                          f"needs a multiple of 8)")
            key = conv_key(B, H, W, C, pc)
            if key in table:
                cfg, ks = table[key][:2]
            else:
                cfg, ks = conv_ops.choose_cfg(B * OH * OW, pc.cout, pc.Kpad)
            self.cfg[i] = (int(cfg), int(ks))
        self._ensure_ws()
        if tune:
            self.autotune_f32() if self.fp32 else self.autotune(verbose=os.environ.get("ADAPT_TUNE_VERBOSE", "0") == "1")

    @staticmethod
    def _time_graph(fn, reps: int) -> float:
        """ms per call of `fn`, `reps` calls captured in one hipGraph (device time only)."""
        fn()
        torch.cuda.synchronize()
        gg = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gg):
            for _ in range(reps):
                fn()
        gg.replay()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(3):
            gg.replay()
        e.record()
        e.synchronize()
        return s.elapsed_time(e) / (3 * reps)

    def autotune_f32(self, reps: int = 10, persist: bool = True, refine: int = 3,
                     verbose: bool = False) -> Dict[str, List]:
        """fp32 path: time every (tile cfg, split-K) of conv_f32.hip per conv
        problem in isolation and keep the fastest ("f32|" keys in the table);
        then (refine > 1) re-decide each problem among its `refine` best isolated
        candidates by replaying the whole captured slice, as the bf16 tuner does
        (round 5: the 98-row GEMM tile cfg 307 is 5 % slower than the ring kernel
        in isolation and 10 us per batch faster in the model)."""
        results: Dict[str, List] = {}
        done: Dict[str, Tuple[int, int]] = {}
        ranked: Dict[str, List[Tuple[float, int, int]]] = {}
        prev = dict(load_tuning())
        for i, st in enumerate(self.steps):
            if st.kind not in ("conv", "dense") or i in self._dense_part:
                continue
            B, H, W, C, OH, OW, pc = self._conv_geom(i)
            M, N = B * OH * OW, pc.cout
            key = "f32|" + conv_key(B, H, W, C, pc)
            if key in done:
                self.cfg[i] = done[key]
                continue
            x = torch.randn(self.bufs(0)[st.ins[0]].shape, device=self.device)
            ns = pc.n_split                       # merged sibling convs write two outputs
            out = torch.empty(M * (ns or N), dtype=torch.float32, device=self.device)
            out2 = torch.empty(M * (N - ns), dtype=torch.float32, device=self.device) if ns else None
            ktiles = pc.Kpad // conv_ops.F32_BK
            best = None
            for cfg in (list(conv_ops.F32_TILES) + list(conv_ops.WINO_F32_CFGS) + list(conv_ops.WINO4S_F32_CFGS)
                        + list(conv_ops.PW_F32_CFGS) + list(conv_ops.F32S_CFGS)):
                if (not conv_ops.f32_cfg_supported(cfg, C, pc.cout, pc) or cfg in conv_ops.WINO_MEASURE_CFGS
                        or cfg in conv_ops.F32_UNTUNED):
                    continue
                if cfg in conv_ops.WINO4S_F32_CFGS:       # F(4x4) transform + GEMM: split-K, fused fixup
                    sp = [k for k in conv_ops.wino4s_splits(C) if k > 1]
                    tiles, kts, sks = int(conv_ops.kernels().wino4s_blocks(cfg, B, H, W, N)), C // 16, \
                        tuple(-k for k in sp)
                elif cfg in conv_ops.PW_F32_CFGS:            # persistent pointwise: whole K, one launch
                    tiles, kts, sks = 0, 1, ()
                elif cfg in conv_ops.F32S_CFGS:             # big-tile 1x1 GEMM: tiles, or stream-K over 256
                    tiles, kts, sks = conv_ops.f32s_tiles(cfg, M, N), C // 32, (-1,)
                elif cfg in conv_ops.WINO_F32_CFGS:         # Winograd F(2x2,3x3): split-K over 16-channel chunks
                    nwm, fn = conv_ops.WINO_F32_CFGS[cfg]
                    tiles = math.ceil(B * ((OH + 1) // 2) * ((OW + 1) // 2) / (16 * nwm)) * (N // (16 * fn))
                    kts, sks = C // 16, (-2, -4)          # fused split-K (fixup in the kernel, <= 4 splits)
                    if cfg in conv_ops.WINO_SK_CFGS:       # stream-K twins: 1 or 2 x 256 blocks only
                        kts, sks = C // 16, (conv_ops.WINO_SK_BASE - 1, conv_ops.WINO_SK_BASE - 2)
                    if cfg in conv_ops.WINO_PU_CFGS:       # persistent: whole K in one launch
                        kts, sks = 1, ()
                else:
                    bm, bn = conv_ops.F32_TILES[cfg]
                    tiles = math.ceil(M / bm) * math.ceil(N / bn)
                    kts = ktiles
                    sks = (-1, -2) if cfg in conv_ops.F32G_CFGS else ()
                for ks in ((1,) if cfg in conv_ops.PW_F32_CFGS or cfg in conv_ops.F32S_CFGS else
                           (1, 2, 4, 8, 16) if cfg not in conv_ops.WINO_SK_CFGS else ()) + sks:
                    # split-K / stream-K only where the tiles alone leave CUs idle
                    if ks > 1 and (kts // ks < 2 or tiles >= 2 * conv_ops.NUM_CUS):
                        continue
                    if ks < 0 and tiles >= 4 * conv_ops.NUM_CUS:
                        continue
                    if -100 < ks < 0 and cfg in conv_ops.WINO_F32_CFGS and (kts // -ks < 2 or tiles >= 2 * conv_ops.NUM_CUS):
                        continue
                    nws = (conv_ops.wino4s_ws_elems(B, H, W, C, N, ks) if cfg in conv_ops.WINO4S_F32_CFGS
                           else conv_ops.workspace_elems_f32(M, N, pc.Kpad, cfg, ks))
                    ws = torch.empty(nws, dtype=torch.float32, device=self.device) if nws else None
                    nctr = conv_ops.f32_counter_elems(cfg, ks, B, H, W, OH, OW, N, pc.Kpad)
                    ctr = torch.zeros(nctr, dtype=torch.int32, device=self.device) if nctr else None
                    try:
                        t = self._time_graph(lambda: conv_ops.conv_forward_f32(x, pc, out, cfg=cfg, ksplit=ks,
                                                                               workspace=ws, counters=ctr,
                                                                               out2=out2), reps)
                    except (RuntimeError, ValueError):
                        continue
                    ranked.setdefault(key, []).append((t, cfg, ks))
                    if best is None or t < best[0]:
                        best = (t, cfg, ks)
            if best:
                results[key] = [best[1], best[2], round(best[0] * 1000, 2)]
                done[key] = (best[1], best[2])
                self.cfg[i] = (best[1], best[2])
                if verbose:
                    print(f"autotune {key}: cfg {best[1]} ksplit {best[2]} {best[0] * 1000:.2f} us", flush=True)
        self._ensure_ws()
        refine = int(os.environ.get("ADAPT_TUNE_REFINE", refine))
        if refine > 1 and ranked:
            self._refine_in_graph(ranked, results, refine, prev, verbose, prefix="f32|")
        if persist:
            save_tuning(results)
        return results

    def autotune(self, reps: int = 20, persist: bool = True, refine: int = 3, verbose: bool = False) -> Dict[str, List]:
        """Time every (tile cfg, split-K) candidate per conv problem in isolation,
        then (refine > 1) re-decide each problem among its `refine` best
        candidates by replaying the WHOLE captured slice: isolated timings miss
        how a kernel's tail and grid overlap with its neighbours."""
        results: Dict[str, List] = {}
        done: Dict[str, Tuple[int, int]] = {}
        ranked: Dict[str, List[Tuple[float, int, int]]] = {}
        prev = dict(load_tuning())              # the table in force: a known-good starting point
        for i, st in enumerate(self.steps):
            if st.kind not in ("conv", "dense") or i in self._dense_part:
                continue
            B, H, W, C, OH, OW, pc = self._conv_geom(i)
            M, N = B * OH * OW, pc.cout
            key = conv_key(B, H, W, C, pc)
            if key in done:
                self.cfg[i] = done[key]
                continue
            x = torch.randn(self.bufs(0)[st.ins[0]].shape, device=self.device).to(torch.bfloat16)
            ns = pc.n_split                       # merged sibling convs write two outputs
            out = torch.empty(M * (ns or N), dtype=torch.bfloat16, device=self.device)
            extra = {"out2": torch.empty(M * (N - ns), dtype=torch.bfloat16, device=self.device)} if ns else {}
            best = None
            ktiles = pc.Kpad // conv_ops.BK
            resident = (list(conv_ops.PW_CFGS) + list(conv_ops.PS_CFGS) + list(conv_ops.RR3_CFGS)
                        + list(conv_ops.CS3_CFGS))
            for cfg in list(conv_ops.CFG_TILES) + resident:
                for ks in (1, 2, 3, 4, 6, 8, -1, -2):
                    if cfg in conv_ops.PS_CFGS:              # ks = blocks per CU for the sliced pointwise
                        if ks not in conv_ops.PS_GRIDS:
                            continue
                    elif cfg in resident and ks != 1:
                        continue
                    if ks > 1 and ktiles // ks < 2:
                        continue
                    if ks < 0 and cfg in conv_ops.V1_CFGS:
                        continue
                    try:
                        need = conv_ops.workspace_elems(M, N, pc.Kpad, cfg, ks)
                        ws = torch.empty(need, dtype=torch.float32, device=self.device) if need else None
                        ctr = None
                        if ks < 0:
                            ctr = torch.zeros(conv_ops.sk_plan(M, N, pc.Kpad, cfg, -ks)[0], dtype=torch.int32,
                                              device=self.device)
                        conv_ops.conv_forward(x, pc, out, cfg=cfg, ksplit=ks, workspace=ws, counters=ctr, **extra)
                        torch.cuda.synchronize(self.device)
                        # time device work only: `reps` launches captured in one hipGraph
                        gg = torch.cuda.CUDAGraph()
                        with torch.cuda.graph(gg, stream=self._capture_stream()):
                            for _ in range(reps):
                                conv_ops.conv_forward(x, pc, out, cfg=cfg, ksplit=ks, workspace=ws, counters=ctr,
                                                      **extra)
                        gg.replay()
                        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        s.record()
                        for _ in range(3):
                            gg.replay()
                        e.record()
                        e.synchronize()
                        t = s.elapsed_time(e) / (3 * reps)
                        del gg
                    except (RuntimeError, ValueError):
                        continue
                    ranked.setdefault(key, []).append((t, cfg, ks))
                    if best is None or t < best[0]:
                        best = (t, cfg, ks)
            if best:
                results[key] = [best[1], best[2], round(best[0] * 1000, 2)]
                done[key] = (best[1], best[2])
                self.cfg[i] = (best[1], best[2])
                if verbose:
                    print(f"autotune {key}: cfg {best[1]} ksplit {best[2]} {best[0] * 1000:.2f} us", flush=True)
        self._ensure_ws()
        # ADAPT_TUNE_REFINE: how many of each problem's best isolated candidates
        # are re-timed inside the whole captured slice
        refine = int(os.environ.get("ADAPT_TUNE_REFINE", refine))
        if refine > 1 and ranked:
            self._refine_in_graph(ranked, results, refine, prev, verbose)
        if persist:
            save_tuning(results)
        return results

    def _graph_time(self, rounds: int = 5, reps: int = 10) -> float:
        """Median ms per replay of the whole slice, freshly captured."""
        g = torch.cuda.CUDAGraph()
        s = self._capture_stream()
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            self._launch(0)
        torch.cuda.current_stream(self.device).wait_stream(s)
        torch.cuda.synchronize(self.device)
        with torch.cuda.graph(g, stream=s):
            self._launch(0)
        g.replay()
        times = []
        for _ in range(rounds):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(reps):
                g.replay()
            b.record()
            b.synchronize()
            times.append(a.elapsed_time(b) / reps)
        del g
        return sorted(times)[len(times) // 2]

    def _refine_in_graph(self, ranked, results, top: int, prev: Optional[Dict[str, List]] = None,
                         verbose: bool = False, prefix: str = "") -> None:
        steps_of: Dict[str, List[int]] = {}
        for i, st in enumerate(self.steps):
            if st.kind in ("conv", "dense") and i not in self._dense_part:
                B, H, W, C, OH, OW, pc = self._conv_geom(i)
                steps_of.setdefault(prefix + conv_key(B, H, W, C, pc), []).append(i)
        # start from the previous table where it is still a valid candidate, so a
        # re-tune can only keep or improve the whole-slice time
        for key, idx in steps_of.items():
            old = (prev or {}).get(key)
            if old and any((c, k) == (int(old[0]), int(old[1])) for _, c, k in ranked.get(key, [])):
                for i in idx:
                    self.cfg[i] = (int(old[0]), int(old[1]))
                results[key] = list(old)
        self._ensure_ws()
        base = self._graph_time()
        # most expensive problems first (isolated time x occurrences)
        order = sorted(ranked, key=lambda k: -min(ranked[k])[0] * len(steps_of.get(k, [])))
        for key in order:
            if key not in steps_of:
                continue
            cands = sorted(ranked[key])[:top]
            cur = self.cfg[steps_of[key][0]]
            for t, cfg, ks in cands:
                if (cfg, ks) == cur:
                    continue
                for i in steps_of[key]:
                    self.cfg[i] = (cfg, ks)
                self._ensure_ws()
                tt = self._graph_time()
                if tt < base * 0.997:
                    if verbose:
                        print(f"refine {key}: cfg {cfg} ksplit {ks}: slice {base:.4f} -> {tt:.4f} ms", flush=True)
                    base, cur = tt, (cfg, ks)
                    results[key] = [cfg, ks, round(t * 1000, 2)]
                else:
                    for i in steps_of[key]:
                        self.cfg[i] = cur
        self._ensure_ws()
        self.tuned_graph_ms = base

    # -------------------------------------------------------------- run
    def _launch(self, set_idx: int = 0, stream=None) -> None:
        if self.private_sets:
            self._bind(set_idx)
            self._ensure_ws()              # this set's workspace, sized for the configs in force
        b = self.bufs(set_idx)
        # ADAPT_DEBUG_SYNC=1: synchronize after every step so a faulting or
        # failing kernel is reported with its step (the AMD_SERIALIZE_KERNEL
        # idea at plan level; never active under hipGraph capture)
        debug = os.environ.get("ADAPT_DEBUG_SYNC", "0") == "1" and not torch.cuda.is_current_stream_capturing()
        main = stream if stream is not None else torch.cuda.current_stream(self.device)
        side = self._side
        joins: Dict[int, List[int]] = {}
        for a, j in side.items():
            joins.setdefault(j, []).append(a)
        if side and self._side_stream is None:
            self._side_stream = private_stream(self.device)
        done: Dict[int, torch.cuda.Event] = {}
        main_stream = stream
        for i, st in enumerate(self.steps):
            if debug and i:
                self._debug_check(i - 1)
            for a in joins.get(i, []):
                main.wait_event(done[a])              # join: the branch result is ready
            stream, ws, ctr = main_stream, self._ws, self._ctr
            if i in side:                             # fork: the branch starts after everything before it
                fork = torch.cuda.Event()
                fork.record(main)
                self._side_stream.wait_event(fork)
                stream, ws, ctr = self._side_stream, self._ws_side, self._ctr_side
            k = st.kind
            if self.fp32:
                self._launch_f32(i, st, b, stream, ws)
            elif k == "pack":
                E.input_pack(b[st.ins[0]], b[st.out], stream=stream)
            elif k == "bottleneck":
                conv_ops.bottleneck_forward(b[st.ins[0]], self.packed[i], b[st.out], stream=stream)
            elif k == "pair":
                conv_ops.pair_forward(b[st.ins[0]], b[st.ins[1]], self.packed[i], b[st.out], b[st.p["out2"]],
                                      stream=stream)
            elif k == "stem":
                conv_ops.stem_forward(b[st.ins[0]], self.packed[i], b[st.out], pool=st.p["pool"],
                                      pool_pad=st.p["pool_pad"], stream=stream)
            elif k == "conv":
                cfg, ks = self.cfg[i]
                res = b[st.ins[1]] if len(st.ins) > 1 else None
                out2 = b[st.p["out2"]] if st.p.get("out2") else None
                conv_ops.conv_forward(b[st.ins[0]], self.packed[i], b[st.out], residual=res, relu=st.p["relu"],
                                      cfg=cfg, ksplit=ks, workspace=ws, stream=stream, counters=ctr,
                                      out2=out2, relu2=st.p.get("relu2", False))
            elif k == "maxpool":
                (pt, _), (pl, _) = st.p["pads"]
                E.maxpool(b[st.ins[0]], b[st.out], st.p["pool"], st.p["stride"], pt, pl, st.p.get("pad_zero", True),
                          stream=stream)
            elif k == "avgpool":
                E.avgpool(b[st.ins[0]], b[st.out], st.p["pool"], st.p["stride"], st.p["pads"], stream=stream)
            elif k == "dwconv":
                w, bias = self.packed[i]
                E.dwconv(b[st.ins[0]], w, bias, b[st.out], st.p["stride"], st.p["pads"], act=st.p["relu"],
                         stream=stream)
            elif k == "act":
                E.act(b[st.ins[0]], b[st.out], st.p["mode"], st.p["alpha"], stream=stream)
            elif k == "binary":
                E.binary(b[st.ins[0]], b[st.ins[1]], b[st.out], st.p["fn"], st.p["act"], stream=stream)
            elif k == "gmp":
                E.gmp(b[st.ins[0]], b[st.out], stream=stream)
            elif k == "affine":
                sc, sh = self.packed[i]
                E.bn_act(b[st.ins[0]], sc, sh, b[st.out], relu=0, stream=stream)
            elif k == "concat":
                E.concat([b[t] for t in st.ins], st.p["channels"], b[st.out], sum(st.p["channels"]), stream=stream)
            elif k == "copy":
                src, dst = b[st.ins[0]], b[st.out]
                if src.numel() != dst.numel() or src.dtype != dst.dtype:
                    raise RuntimeError(f"copy {st.ins[0]} -> {st.out}: {tuple(src.shape)} vs {tuple(dst.shape)}")
                if stream is not None:
                    with torch.cuda.stream(stream):
                        dst.view(-1).copy_(src.view(-1), non_blocking=True)
                else:
                    dst.view(-1).copy_(src.view(-1), non_blocking=True)
            elif k == "bn":
                sc, sh = self.packed[i]
                E.bn_act(b[st.ins[0]], sc, sh, b[st.out], relu=st.p["relu"], stream=stream)
            elif k == "add":
                E.add_act(b[st.ins[0]], b[st.ins[1]], b[st.out], relu=st.p["relu"], stream=stream)
            elif k == "relu":
                E.relu(b[st.ins[0]], b[st.out], mode=st.p.get("mode", 1) or 1, stream=stream)
            elif k == "pad":
                (pt, _), (pl, _) = st.p["pad"]
                E.pad(b[st.ins[0]], b[st.out], pt, pl, stream=stream)
            elif k == "gap":
                E.gap(b[st.ins[0]], out=b[st.out], stream=stream, scratch=self._gap_part.get(i))
            elif k == "dense" and i in self._dense_part:
                x = b[st.ins[0]].reshape(self.batch, -1)
                if st.p["softmax"]:
                    E.dense_small(x, self.packed[i], self._dense_part[i], logits=self._logits[i], probs=b[st.out],
                                  stream=stream)
                else:
                    E.dense_small(x, self.packed[i], self._dense_part[i], logits=b[st.out], stream=stream)
            elif k == "dense":
                cfg, ks = self.cfg[i]
                x = b[st.ins[0]].reshape(self.batch, -1)
                dst = self._logits[i] if st.p["softmax"] else b[st.out]
                conv_ops.conv_forward(x, self.packed[i], dst, relu=st.p.get("relu", 0), cfg=cfg, ksplit=ks,
                                      workspace=self._ws, stream=stream, counters=self._ctr)
                if st.p["softmax"]:
                    E.softmax_rows(dst, b[st.out], stream=stream)
            elif k == "softmax":
                E.softmax_rows(b[st.ins[0]], b[st.out], stream=stream)
            else:
                raise NotImplementedError(k)
            if i in side:
                ev = torch.cuda.Event()
                ev.record(self._side_stream)
                done[i] = ev
        stream = main_stream
        for a in done:                                # every branch joined (normally at its consumer)
            if a not in side or side[a] >= len(self.steps):
                main.wait_event(done[a])
        if debug and self.steps:
            self._debug_check(len(self.steps) - 1)
        # relay frontier tensors: device copy into the output set (no aliasing with the
        # input buffer that the next micro-batch's receive will overwrite)
        for r in self.relay:
            s = self.sets[set_idx]
            if stream is not None:
                with torch.cuda.stream(stream):
                    s[r + "#out"].copy_(s[r], non_blocking=True)
            else:
                s[r + "#out"].copy_(s[r], non_blocking=True)

    def _launch_f32(self, i: int, st: Step, b, stream, ws) -> None:
        """One step of the fp32 path (csrc/kernels/conv_f32.hip)."""
        k = st.kind
        ctr = self._ctr_side if stream is not None and stream is self._side_stream else self._ctr
        if k == "conv":
            cfg, ks = self.cfg[i]
            res = b[st.ins[1]] if len(st.ins) > 1 else None
            out2 = b[st.p["out2"]] if st.p.get("out2") else None
            conv_ops.conv_forward_f32(b[st.ins[0]], self.packed[i], b[st.out], residual=res, relu=st.p["relu"],
                                      cfg=cfg, ksplit=ks, workspace=ws, stream=stream, counters=ctr,
                                      out2=out2, relu2=st.p.get("relu2", 0))
        elif k == "dense" and i in self._dense_part:
            x = b[st.ins[0]].reshape(self.batch, -1)
            if st.p["softmax"]:
                E.dense_small_f32(x, self.packed[i], self._dense_part[i], logits=self._logits[i], probs=b[st.out],
                                  stream=stream)
            else:
                E.dense_small_f32(x, self.packed[i], self._dense_part[i], logits=b[st.out], stream=stream)
        elif k == "dense":
            cfg, ks = self.cfg[i]
            x = b[st.ins[0]].reshape(self.batch, -1)
            dst = self._logits[i] if st.p["softmax"] else b[st.out]
            conv_ops.conv_forward_f32(x, self.packed[i], dst, relu=st.p.get("relu", 0), cfg=cfg, ksplit=ks,
                                      workspace=ws, stream=stream, counters=ctr)
            if st.p["softmax"]:
                E.softmax_rows(dst, b[st.out], stream=stream)
        elif k == "stem_f32":
            conv_ops.stem_f32_forward(b[st.ins[0]], self.packed[i], b[st.out], pool_pad=st.p["pool_pad"],
                                      stream=stream)
        elif k == "pair":
            conv_ops.pair_f32_forward(b[st.ins[0]], b[st.ins[1]], self.packed[i], b[st.out], b[st.p["out2"]],
                                      stream=stream)
        elif k == "maxpool":
            (pt, _), (pl, _) = st.p["pads"]
            E.maxpool_f32(b[st.ins[0]], b[st.out], st.p["pool"], st.p["stride"], pt, pl, st.p.get("pad_zero", True),
                          stream=stream)
        elif k == "gap":
            E.gap_f32(b[st.ins[0]], b[st.out], stream=stream, scratch=self._gap_part.get(i))
        elif k == "softmax":
            E.softmax_rows(b[st.ins[0]], b[st.out], stream=stream)
        elif k == "add":
            E.eltwise_f32(b[st.ins[0]], b[st.out], b=b[st.ins[1]], relu=st.p["relu"], stream=stream)
        elif k == "bn":
            sc, sh = self.packed[i]
            E.eltwise_f32(b[st.ins[0]], b[st.out], scale=sc, shift=sh, relu=st.p["relu"], stream=stream)
        elif k == "relu":
            E.eltwise_f32(b[st.ins[0]], b[st.out], relu=st.p.get("mode", 1) or 1, stream=stream)
        elif k == "pad":
            (pt, _), (pl, _) = st.p["pad"]
            E.pad_f32(b[st.ins[0]], b[st.out], pt, pl, stream=stream)
        elif k == "dwconv":
            w, bias = self.packed[i]
            E.dwconv_f32(b[st.ins[0]], w, bias, b[st.out], st.p["stride"], st.p["pads"], act=st.p["relu"],
                         stream=stream)
        elif k == "avgpool":
            E.avgpool_f32(b[st.ins[0]], b[st.out], st.p["pool"], st.p["stride"], st.p["pads"], stream=stream)
        elif k == "concat":
            E.concat_f32([b[t] for t in st.ins], b[st.out], stream=stream)
        elif k == "act":
            E.affine_act_f32(b[st.ins[0]], b[st.out], act=st.p["mode"], alpha=st.p["alpha"], stream=stream)
        elif k == "binary":
            E.binary_f32(b[st.ins[0]], b[st.ins[1]], b[st.out], st.p["fn"], st.p["act"], stream=stream)
        elif k == "affine":
            sc, sh = self.packed[i]
            E.affine_act_f32(b[st.ins[0]], b[st.out], sc, sh, stream=stream)
        elif k == "copy":
            src, dst = b[st.ins[0]], b[st.out]
            if stream is not None:
                with torch.cuda.stream(stream):
                    dst.view(-1).copy_(src.view(-1), non_blocking=True)
            else:
                dst.view(-1).copy_(src.view(-1), non_blocking=True)
        else:
            raise NotImplementedError(f"fp32 {k}")

    def _debug_check(self, i: int) -> None:
        try:
            torch.cuda.synchronize(self.device)
        except RuntimeError as e:
            st = self.steps[i]
            raise RuntimeError(f"step {i} ({st.kind} -> {st.out}, cfg {self.cfg.get(i)}) failed: {e}") from e

    def capture(self, mode: str = "global") -> None:
        """Record the step list of every buffer set into its own hipGraph.
        mode="thread_local" lets other threads keep launching and synchronising
        while this one captures (a worker preparing its next slice in the
        background of a serving epoch)."""
        s = self._capture_stream()
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for j in range(self.num_sets):
                self._launch(j)                 # warm-up: code-object load, allocator
        torch.cuda.current_stream(self.device).wait_stream(s)
        torch.cuda.synchronize(self.device)
        for j in range(self.num_sets):
            g = torch.cuda.CUDAGraph()
            # a private capture stream: with a pool stream, another thread's work could land in this capture
            with torch.cuda.graph(g, stream=s, capture_error_mode=mode):
                self._launch(j)
            self._graphs[j] = g
        torch.cuda.synchronize(self.device)

    def _capture_stream(self):
        if getattr(self, "_cap_stream", None) is None:
            self._cap_stream = private_stream(self.device)
        return self._cap_stream

    @property
    def captured(self) -> bool:
        return self._graphs[0] is not None

    def forward(self, set_idx: int = 0) -> Dict[str, torch.Tensor]:
        """Run on the current stream using the static buffers of `set_idx`."""
        g = self._graphs[set_idx]
        if g is not None:
            g.replay()
        else:
            self._launch(set_idx)
        return {o: self.output_buf(o, set_idx) for o in self.outputs}

    def logits(self) -> Optional[torch.Tensor]:
        """Pre-softmax logits of the last Dense(softmax) step (None if there is none)."""
        for i in reversed(range(len(self.steps))):
            if i in self._logits:
                return self._logits[i]
        return None

    def run(self, inputs: Dict[str, torch.Tensor], set_idx: int = 0) -> Dict[str, torch.Tensor]:
        for n, t in inputs.items():
            dst = self.sets[set_idx][n]
            if tuple(t.shape) != tuple(dst.shape):
                raise ValueError(f"input {n}: expected {tuple(dst.shape)}, got {tuple(t.shape)}")
            dst.copy_(t, non_blocking=True)
        return self.forward(set_idx)

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        return self.run({self.g.input_names[0]: x})[self.outputs[0]]

    def describe(self) -> str:
        lines = []
        for i, st in enumerate(self.steps):
            extra = f" cfg={self.cfg[i]}" if i in self.cfg else ""
            lines.append(f"{i:3d} {st.kind:8s} {st.out:28s} <- {st.ins}{extra}")
        return "\n".join(lines)
