"""Loader for the in-tree gfx950 kernel library (``_C``).

torch is imported first so our library binds to the HIP runtime torch
already loaded (both link SONAME ``libamdhip64.so.7``).  There is no silent
fallback: on a GPU the kernels must load or `kernels()` raises.
"""
from __future__ import annotations

import importlib
import os
import threading

import torch  # noqa: F401  (must precede the extension import)

_lock = threading.Lock()
_C = None


def kernels():
    """Return the `_C` extension module, building it in-tree if it is missing."""
    global _C
    if _C is not None:
        return _C
    with _lock:
        if _C is not None:
            return _C
        try:
            mod = importlib.import_module("adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd._C")
        except ImportError:
            if os.environ.get("ADAPT_NO_BUILD"):
                raise
            from .. import _build
            _build.build_kernels()
            mod = importlib.import_module("adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd._C")
        _C = mod
    return _C


def private_stream(device) -> "torch.cuda.ExternalStream":
    """A non-blocking HIP stream of the caller's own.  torch.cuda.Stream() hands
    out streams of a shared round-robin pool, so two threads can get the same
    one: a hipGraph captured on a pool stream (a worker preparing its next slice
    in the background) could then take in, or be invalidated by, another
    thread's work.  Every capture runs on one of these.  Like pool streams they
    live as long as the process (one per executor; destroying them under
    PyTorch's current-stream bookkeeping is not worth the risk)."""
    dev = torch.device(device)
    if dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    with torch.cuda.device(dev):
        h = kernels().stream_create()
    return torch.cuda.ExternalStream(h, device=dev)


def stream_handle(stream=None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


def ptr(t) -> int:
    return 0 if t is None else int(t.data_ptr())
