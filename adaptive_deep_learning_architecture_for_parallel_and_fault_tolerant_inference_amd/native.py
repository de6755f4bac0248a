"""Loader for the in-tree host runtime library (``_runtime``: framing, LZ4, zfp).

Built with g++ by `_build.build_runtime()`; there is no pure-Python
fallback for these components (the reference uses python-lz4 / zfpy C
libraries, SURVEY §2.2 — this is our native replacement).
"""
from __future__ import annotations

import importlib
import os
import threading

_lock = threading.Lock()
_mod = None


def runtime():
    global _mod
    if _mod is not None:
        return _mod
    with _lock:
        if _mod is None:
            name = __package__ + "._runtime"
            try:
                _mod = importlib.import_module(name)
            except ImportError:
                if os.environ.get("ADAPT_NO_BUILD"):
                    raise
                from . import _build
                _build.build_runtime()
                _mod = importlib.import_module(name)
    return _mod
