"""One typed configuration for dispatcher, workers and tools.

The reference hard-codes everything (ports, chunk size, timeouts, worker
list, cut list) and asks users to edit sources.  Here every knob
lives in `AdaptConfig`, resolved in this order (later wins):

    dataclass defaults  <  YAML file (--config)  <  ADAPT_<FIELD> env vars  <  CLI flags

`part_at` accepts a list of layer names, a comma-separated string, or
``"auto:K"`` (balanced planner, K stages).
"""
from __future__ import annotations

import dataclasses
import os
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Union

import yaml


@dataclass
class AdaptConfig:
    # model
    model: str = "resnet50"
    seed: int = 0
    image: List[int] = field(default_factory=lambda: [224, 224, 3])
    classes: int = 1000
    weights: Optional[str] = None            # safetensors checkpoint (graph/manifest.save_model) or Keras .npz list
    # partition / placement
    part_at: Union[List[str], str] = field(default_factory=list)
    batch: int = 1                           # micro-batch size per pipeline message
    elastic: bool = False                    # rebalance on worker join, not only on leave
    replicas: Union[int, str] = "auto"       # PP x DP: pipeline replicas ("auto" = live // stages)
    # data plane
    transport: str = "auto"                  # auto | tcp | rccl | gloo (auto: rccl between distinct local GPUs)
    codec: str = "none"                      # activations on TCP links: none|lz4|zvc|zfp+lz4 (host LZ4 of
                                             # activations: ratio ~1.02 at 0.2 GB/s, so off by default)
    weight_codec: str = "zfp+lz4"            # slice push (reference: zfp+lz4)
    chunk_size: int = 512 * 1000             # socket chunk (src/dispatcher.py:24)
    # control plane
    dispatcher_host: str = "127.0.0.1"
    membership_port: int = 2379
    result_port: int = 6003
    data_port: int = 6000
    config_port: int = 6001
    lease_ttl: float = 1.0
    # flow control / fault handling
    max_inflight: int = 8
    task_timeout: Optional[float] = None       # None: per replica, 10 s GPU / 30 s CPU, scaled by the period
    worker_wait: float = 5.0
    ordered: bool = False
    # worker
    device: Optional[str] = None
    node_id: Optional[str] = None
    graph: bool = True                       # hipGraph capture of each slice
    # observability
    trace: Optional[str] = None              # JSONL span log path
    prometheus_port: Optional[int] = None

    # --------------------------------------------------------------- load
    @classmethod
    def load(cls, path: Optional[str] = None, env: Optional[Dict[str, str]] = None,
             overrides: Optional[Dict[str, Any]] = None) -> "AdaptConfig":
        cfg = cls()
        if path:
            with open(path) as f:
                data = yaml.safe_load(f) or {}
            cfg = cfg.replace(**data)
        env = os.environ if env is None else env
        upd = {}
        for f in dataclasses.fields(cls):
            key = "ADAPT_" + f.name.upper()
            if key in env:
                upd[f.name] = _coerce(env[key], getattr(cfg, f.name))
        cfg = cfg.replace(**upd)
        if overrides:
            cfg = cfg.replace(**{k: v for k, v in overrides.items() if v is not None})
        return cfg

    def replace(self, **kw) -> "AdaptConfig":
        names = {f.name for f in dataclasses.fields(self)}
        bad = set(kw) - names
        if bad:
            raise KeyError(f"unknown config keys {sorted(bad)}")
        return dataclasses.replace(self, **kw)

    def cuts(self, graph=None, precision: str = "fp32") -> List[str]:
        """Resolve `part_at` (list, 'a,b', or 'auto:K') to layer names ('auto:K': the planner's cuts for
        the job's activation precision, DEFER's default fp32)."""
        p = self.part_at
        if isinstance(p, list) and len(p) == 1 and p[0].startswith("auto:"):
            p = p[0]
        if isinstance(p, str):
            if p.startswith("auto:"):
                from ..graph.planner import plan_cuts
                k = int(p.split(":", 1)[1])
                return plan_cuts(graph, k, batch=max(self.batch, 1), precision=precision)[0]
            return [s for s in p.split(",") if s]
        return list(p)

    def to_dict(self) -> Dict[str, Any]:
        return dataclasses.asdict(self)


def _coerce(s: str, like: Any):
    if isinstance(like, bool):
        return s.lower() in ("1", "true", "yes", "on")
    if isinstance(like, int) and not isinstance(like, bool):
        return int(s)
    if isinstance(like, float):
        return float(s)
    if isinstance(like, list):
        return [x for x in s.split(",") if x]
    if like is None:
        for conv in (int, float):
            try:
                return conv(s)
            except ValueError:
                pass
        return s
    return s
