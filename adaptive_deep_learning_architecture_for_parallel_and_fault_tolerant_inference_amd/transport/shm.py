"""Same-host zero-copy ingest: request tensors in POSIX shared memory.

The reference pushes every input image through a TCP socket, zfp+lz4
compressed, from one Python thread (`src/dispatcher.py:99-107`): at bs=32
that is 19.3 MB of fp32 per batch through the loopback stack.  When the
dispatcher and a pipeline's stage 0 share a host, the dispatcher instead
writes the batch into a slot of a shared-memory pool and sends only a small
descriptor (codec id "shm": segment name + offset) over the data link.  Stage
0 maps the segment once, registers the mapping with the HIP runtime (page-
locked, so the host->device copy is an async DMA straight from the slot) and
reads the batch in place.

A slot stays owned by its request until the request completes (result
received or given up): a replay after a failure just re-sends the descriptor.
Segments are plain files under /dev/shm opened with os.open + mmap (not
`multiprocessing.shared_memory`, whose resource tracker would unlink a
segment when an *attaching* worker exits); the dispatcher unlinks its pool on
shutdown.
"""
from __future__ import annotations

import mmap
import os
import threading
import uuid
from typing import Dict, List, Optional, Tuple

import numpy as np

SHM_DIR = "/dev/shm"


def available() -> bool:
    return os.path.isdir(SHM_DIR) and os.access(SHM_DIR, os.W_OK)


class Slot:
    __slots__ = ("pool", "name", "nbytes", "mm", "index")

    def __init__(self, pool: "ShmPool", name: str, nbytes: int, mm: mmap.mmap, index: int):
        self.pool, self.name, self.nbytes, self.mm, self.index = pool, name, nbytes, mm, index

    def view(self, dtype, shape) -> np.ndarray:
        return np.ndarray(shape, dtype=dtype, buffer=self.mm, offset=0)

    def release(self) -> None:
        self.pool.release(self)


class ShmPool:
    """Dispatcher side: slots of `nbytes` (one segment each), recycled."""

    def __init__(self, prefix: Optional[str] = None):
        self.prefix = prefix or f"adapt-{os.getpid()}-{uuid.uuid4().hex[:8]}"
        self._lock = threading.Lock()
        self._free: Dict[int, List[Slot]] = {}
        self._all: List[Slot] = []

    def acquire(self, nbytes: int) -> Slot:
        with self._lock:
            free = self._free.setdefault(nbytes, [])
            if free:
                return free.pop()
            name = f"{self.prefix}-{len(self._all)}"
            path = os.path.join(SHM_DIR, name)
            fd = os.open(path, os.O_CREAT | os.O_EXCL | os.O_RDWR, 0o600)
            try:
                os.ftruncate(fd, nbytes)
                mm = mmap.mmap(fd, nbytes)
            finally:
                os.close(fd)
            s = Slot(self, name, nbytes, mm, len(self._all))
            self._all.append(s)
            return s

    def put(self, arr: np.ndarray) -> Slot:
        """Copy `arr` into a free slot."""
        arr = np.ascontiguousarray(arr)
        s = self.acquire(arr.nbytes)
        np.copyto(s.view(arr.dtype, arr.shape), arr)
        return s

    def release(self, s: Slot) -> None:
        with self._lock:
            self._free.setdefault(s.nbytes, []).append(s)

    def close(self) -> None:
        with self._lock:
            for s in self._all:
                try:
                    s.mm.close()
                except (BufferError, ValueError):
                    pass
                try:
                    os.unlink(os.path.join(SHM_DIR, s.name))
                except FileNotFoundError:
                    pass
            self._all.clear()
            self._free.clear()


class _Attached:
    def __init__(self, name: str):
        path = os.path.join(SHM_DIR, name)
        fd = os.open(path, os.O_RDWR)
        try:
            size = os.fstat(fd).st_size
            self.mm = mmap.mmap(fd, size)
        finally:
            os.close(fd)
        self.size = size
        self.arr = np.frombuffer(self.mm, dtype=np.uint8)
        self.registered = False


class ShmRef:
    """A request tensor that lives in a pool slot: on the wire it is the "shm"
    codec container (segment name + offset), not the bytes."""

    def __init__(self, slot: Slot, dtype, shape: Tuple[int, ...]):
        self.slot, self.dtype, self.shape = slot, np.dtype(dtype), tuple(int(v) for v in shape)

    @property
    def array(self) -> np.ndarray:
        return self.slot.view(self.dtype, self.shape)

    def container(self) -> bytes:
        from .. import codec as C
        return C.wrap(self.slot.name.encode() + b"\0" + (0).to_bytes(8, "little"), "shm", self.dtype, self.shape)


# worker processes on a GPU set this: mapped segments are page-locked for DMA
REGISTER_DEVICE = False
_attached: Dict[str, _Attached] = {}
_att_lock = threading.Lock()


def attach(name: str, register_device: bool = False) -> _Attached:
    """Worker side: map segment `name` (cached per process); with
    `register_device` the mapping is page-locked for the HIP runtime once."""
    with _att_lock:
        a = _attached.get(name)
        if a is None:
            a = _attached[name] = _Attached(name)
    if register_device and not a.registered:
        import torch
        try:
            rc = torch.cuda.cudart().cudaHostRegister(int(a.arr.ctypes.data), a.size, 0)
            a.registered = int(rc) == 0 if not isinstance(rc, tuple) else int(rc[0]) == 0
        except Exception:  # noqa: BLE001 - a pageable copy still works, just slower
            a.registered = False
    return a


def view(name: str, offset: int, dtype, shape: Tuple[int, ...], register_device: bool = False) -> np.ndarray:
    a = attach(name, register_device)
    n = int(np.prod(shape)) * np.dtype(dtype).itemsize
    if offset + n > a.size:
        raise ValueError(f"shm {name}: {offset + n} bytes past its {a.size}-byte segment")
    return a.arr[offset:offset + n].view(dtype).reshape(shape)


def detach_all() -> None:
    with _att_lock:
        for a in _attached.values():
            if a.registered:
                try:
                    import torch
                    torch.cuda.cudart().cudaHostUnregister(int(a.arr.ctypes.data))
                except Exception:  # noqa: BLE001
                    pass
        _attached.clear()
