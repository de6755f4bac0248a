"""Tracing, metrics and GPU telemetry.

The reference has `print` statements only.  Here:

* `Tracer` — thread-safe JSONL span log (`span(name, **attrs)`), used for
  per-request timelines (dispatch -> stage compute -> emit) and pipeline
  bubble analysis; spans also open roctx ranges (libroctx64) when
  ``ADAPT_ROCTX=1`` so they show up in rocprofv3 ``--marker-trace``;
* `Metrics` — counters and latency histograms (p50/p90/p99), optional
  Prometheus exporter (`prometheus_client`);
* `gpu_telemetry()` — amdsmi readings (GFX activity, VRAM, power,
  temperature) published into each worker's membership record.
"""
from __future__ import annotations

import ctypes
import json
import os
import threading
import time
from collections import defaultdict
from contextlib import contextmanager
from typing import Dict, List, Optional

# ------------------------------------------------------------------- roctx
_roctx = None


def _roctx_lib():
    global _roctx
    if _roctx is None:
        _roctx = False
        if os.environ.get("ADAPT_ROCTX") == "1":
            for name in ("libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
                try:
                    lib = ctypes.CDLL(name)
                    lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                    lib.roctxRangePushA.restype = ctypes.c_int
                    lib.roctxRangePop.restype = ctypes.c_int
                    _roctx = lib
                    break
                except OSError:
                    continue
    return _roctx or None


@contextmanager
def roctx_range(name: str):
    lib = _roctx_lib()
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib is not None:
            lib.roctxRangePop()


# ------------------------------------------------------------------ tracer
class Tracer:
    def __init__(self, path: Optional[str] = None, enabled: Optional[bool] = None):
        self.path = path or os.environ.get("ADAPT_TRACE")
        self.enabled = bool(self.path) if enabled is None else enabled
        self._lock = threading.Lock()
        self._buf: List[dict] = []
        self._fh = open(self.path, "a") if (self.enabled and self.path) else None

    def event(self, name: str, **attrs) -> None:
        if not self.enabled:
            return
        rec = {"ts": time.time(), "name": name, "tid": threading.get_ident(), **attrs}
        with self._lock:
            if self._fh:
                self._fh.write(json.dumps(rec) + "\n")
            else:
                self._buf.append(rec)

    @contextmanager
    def span(self, name: str, **attrs):
        if not self.enabled:
            with roctx_range(name):
                yield
            return
        t0 = time.time()
        with roctx_range(name):
            try:
                yield
            finally:
                self.event(name, start=t0, dur_ms=(time.time() - t0) * 1e3, **attrs)

    def records(self) -> List[dict]:
        with self._lock:
            return list(self._buf)

    def flush(self) -> None:
        with self._lock:
            if self._fh:
                self._fh.flush()


TRACER = Tracer()


# ----------------------------------------------------------------- metrics
class Metrics:
    def __init__(self):
        self._lock = threading.Lock()
        self.counters: Dict[str, float] = defaultdict(float)
        self.samples: Dict[str, List[float]] = defaultdict(list)
        self._prom = None

    def inc(self, name: str, v: float = 1.0) -> None:
        with self._lock:
            self.counters[name] += v
        if self._prom:
            self._prom_counter(name).inc(v)

    def observe(self, name: str, v: float) -> None:
        with self._lock:
            s = self.samples[name]
            s.append(v)
            if len(s) > 100000:
                del s[: len(s) - 100000]
        if self._prom:
            self._prom_hist(name).observe(v)

    def summary(self) -> Dict[str, dict]:
        import numpy as np
        out = {}
        with self._lock:
            for k, v in self.samples.items():
                if v:
                    a = np.asarray(v)
                    out[k] = {"n": len(a), "mean": float(a.mean()), "p50": float(np.percentile(a, 50)),
                              "p90": float(np.percentile(a, 90)), "p99": float(np.percentile(a, 99))}
            out["counters"] = dict(self.counters)
        return out

    # optional Prometheus exporter
    def serve_prometheus(self, port: int = 9400) -> None:
        import prometheus_client as pc
        self._prom = {"c": {}, "h": {}, "pc": pc}
        pc.start_http_server(port)

    def _prom_counter(self, name):
        pc = self._prom["pc"]
        key = name.replace(".", "_").replace("-", "_")
        if key not in self._prom["c"]:
            self._prom["c"][key] = pc.Counter("adapt_" + key, name)
        return self._prom["c"][key]

    def _prom_hist(self, name):
        pc = self._prom["pc"]
        key = name.replace(".", "_").replace("-", "_")
        if key not in self._prom["h"]:
            self._prom["h"][key] = pc.Histogram("adapt_" + key, name)
        return self._prom["h"][key]


METRICS = Metrics()


# ----------------------------------------------------------- GPU telemetry
_amdsmi_handles = None


def gpu_telemetry(index: int = 0) -> Dict[str, float]:
    """Best-effort amdsmi snapshot of one GPU ({} when unavailable)."""
    global _amdsmi_handles
    try:
        import amdsmi
        if _amdsmi_handles is None:
            amdsmi.amdsmi_init()
            _amdsmi_handles = amdsmi.amdsmi_get_processor_handles()
        h = _amdsmi_handles[index]
        out: Dict[str, float] = {}
        try:
            act = amdsmi.amdsmi_get_gpu_activity(h)
            out["gfx_activity"] = float(act.get("gfx_activity", 0))
            out["umc_activity"] = float(act.get("umc_activity", 0))
        except Exception:  # noqa: BLE001
            pass
        try:
            vr = amdsmi.amdsmi_get_gpu_vram_usage(h)
            out["vram_used_mb"] = float(vr.get("vram_used", 0))
            out["vram_total_mb"] = float(vr.get("vram_total", 0))
        except Exception:  # noqa: BLE001
            pass
        try:
            pw = amdsmi.amdsmi_get_power_info(h)
            out["power_w"] = float(pw.get("current_socket_power", pw.get("average_socket_power", 0)) or 0)
        except Exception:  # noqa: BLE001
            pass
        return out
    except Exception:  # noqa: BLE001 - no amdsmi / no GPU / not permitted
        return {}


class PhaseStamps:
    """Per-phase progress stamps of a multi-process job (bench.py sub-runs,
    parallel/fault_run.py): every `stamp` prints ``[<tag> +<ms>] <phase> k=v``
    to stderr at once and keeps ``{phase: ms}`` for the job's JSON record, so a
    run that hangs on an 8-GPU node leaves the phase it reached in its log.
    `arm_faulthandler(limit_s)` additionally dumps every thread's stack 10 s
    before the caller's time limit (and exits), naming where it stopped."""

    def __init__(self, tag: str, stream=None):
        import sys
        import time
        self.tag = tag
        self.stream = stream if stream is not None else sys.stderr
        self.t0 = time.perf_counter()
        self.phases: Dict[str, float] = {}

    def stamp(self, phase: str, **kw) -> float:
        import time
        ms = (time.perf_counter() - self.t0) * 1e3
        self.phases[phase] = round(ms, 1)
        extra = " ".join(f"{k}={v}" for k, v in kw.items())
        print(f"[{self.tag} +{ms:9.1f} ms] {phase}" + (f" {extra}" if extra else ""), file=self.stream, flush=True)
        return ms

    @staticmethod
    def arm_faulthandler(limit_s: float, margin_s: float = 10.0) -> Optional[float]:
        """Dump all stacks to stderr `margin_s` before `limit_s` (no-op for limit <= margin)."""
        import faulthandler
        if not limit_s or limit_s <= margin_s:
            return None
        faulthandler.dump_traceback_later(limit_s - margin_s, exit=True)
        return limit_s - margin_s
