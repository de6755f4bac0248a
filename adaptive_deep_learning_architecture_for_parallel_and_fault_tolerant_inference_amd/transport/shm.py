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

Stage -> stage links (`LinkPool`): when two consecutive stages of a pipeline
share a host (the same `domain()`), the sending stage copies its frontier
tensors device -> host straight into a page-locked slot and sends only the
descriptor; the receiving stage copies host -> device from its own mapping of
the same pages.  The reference ships every activation through a loopback TCP
socket (`src/node.py:163-179`): the ResNet-50 2-stage frontier is 57 MB per
bs=32 batch.  A link slot carries a 64-byte header whose first byte is the
hand-off flag: the sender sets it when it fills the slot, the receiver clears
it once its copy out of the slot has completed, and the sender only reuses
slots whose flag is clear (so the receiver's pace is the link's
back-pressure).

Device links (`DeviceLinkPool`): when both stages are GPU workers on the host,
the slot's payload lives in device memory instead.  Each slot is a hipMalloc
allocation exported by IPC handle; its shared-memory segment keeps the same
64-byte hand-off header, and the handle is stored after that header.  The
sender copies device -> slot (device to device), and the receiver opens the
handle once per slot and copies slot -> its input buffer.  On one GPU that is
an HBM-to-HBM copy, and across GPUs a peer copy over xGMI.  There is no bounce
through host memory: the host-slot link moves the 2-stage ResNet-50 frontier
(57 MB) over PCIe twice per batch.
"""
from __future__ import annotations

import mmap
import os
import threading
import time
import uuid
from typing import Dict, List, Optional, Tuple

import numpy as np

SHM_DIR = "/dev/shm"


def available() -> bool:
    return os.path.isdir(SHM_DIR) and os.access(SHM_DIR, os.W_OK)


def domain() -> Optional[str]:
    """Identity of this process's /dev/shm: two processes can exchange slots
    iff their domains are equal (same kernel boot and the same tmpfs mount, so
    containers with private /dev/shm mounts do not match)."""
    if not available():
        return None
    try:
        with open("/proc/sys/kernel/random/boot_id") as f:
            boot = f.read().strip()
    except OSError:
        boot = "?"
    st = os.stat(SHM_DIR)
    return f"{boot}:{st.st_dev}"


LINK_HDR = 64          # link slots: byte 0 = hand-off flag, data from this offset


class ShmFull(OSError):
    """/dev/shm could not back a new segment (tmpfs size limit): callers fall back
    to an inline (TCP) or pageable path instead of taking a SIGBUS later."""


def _open_reserved(path: str, nbytes: int) -> mmap.mmap:
    """Create segment `path` of `nbytes` with its pages reserved up front.
    ftruncate alone succeeds past a tmpfs mount's size limit and the first
    write into the missing pages raises SIGBUS; posix_fallocate fails with
    ENOSPC instead, so a full /dev/shm is an exception here."""
    fd = os.open(path, os.O_CREAT | os.O_EXCL | os.O_RDWR, 0o600)
    try:
        os.ftruncate(fd, nbytes)
        try:
            os.posix_fallocate(fd, 0, nbytes)
        except OSError as e:
            try:
                os.unlink(path)
            except FileNotFoundError:
                pass
            raise ShmFull(e.errno, f"/dev/shm cannot hold {nbytes} more bytes: {e.strerror}") from e
        return mmap.mmap(fd, nbytes)
    finally:
        os.close(fd)


class Slot:
    __slots__ = ("pool", "name", "nbytes", "mm", "index", "offset")

    def __init__(self, pool, name: str, nbytes: int, mm: mmap.mmap, index: int, offset: int = 0):
        self.pool, self.name, self.nbytes, self.mm, self.index = pool, name, nbytes, mm, index
        self.offset = offset

    def view(self, dtype, shape) -> np.ndarray:
        return np.ndarray(shape, dtype=dtype, buffer=self.mm, offset=self.offset)

    def release(self) -> None:
        self.pool.release(self)


COPY_THREADS = 4


def _copy(dst: np.ndarray, src: np.ndarray) -> None:
    """dst <- src (same bytes): the native runtime's threaded copy for large arrays."""
    if src.nbytes >= (1 << 20):
        try:
            from ..native import runtime
            runtime().copy_into(dst.reshape(-1).view(np.uint8), src.reshape(-1).view(np.uint8), COPY_THREADS)
            return
        except (ImportError, AttributeError):
            pass
    np.copyto(dst, src)


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
            mm = _open_reserved(os.path.join(SHM_DIR, name), nbytes)
            s = Slot(self, name, nbytes, mm, len(self._all))
            self._all.append(s)
            return s

    def put(self, arr: np.ndarray) -> Slot:
        """Copy `arr` into a free slot (a multi-threaded native copy, GIL released)."""
        arr = np.ascontiguousarray(arr)
        s = self.acquire(arr.nbytes)
        _copy(s.view(arr.dtype, arr.shape), arr)
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


class LinkPool:
    """Sender side of a same-host stage -> stage link (module docstring)."""

    def __init__(self, prefix: Optional[str] = None, max_slots: int = 6, register_device: bool = False):
        self.prefix = prefix or f"adapt-link-{os.getpid()}-{uuid.uuid4().hex[:8]}"
        self.max_slots = max_slots
        self.register_device = register_device
        self._lock = threading.Lock()
        self._by_size: Dict[int, List[Slot]] = {}
        self._all: List[Slot] = []
        self._registered: List[int] = []

    def _create(self, nbytes: int) -> Slot:
        name = f"{self.prefix}-{len(self._all)}"
        mm = _open_reserved(os.path.join(SHM_DIR, name), LINK_HDR + nbytes)
        s = Slot(self, name, nbytes, mm, len(self._all), offset=LINK_HDR)
        self._all.append(s)
        if self.register_device:          # the device -> host copy is then an async DMA into the slot
            import torch
            addr = np.frombuffer(mm, dtype=np.uint8).ctypes.data
            try:
                rc = torch.cuda.cudart().cudaHostRegister(int(addr), LINK_HDR + nbytes, 0)
                if (int(rc[0]) if isinstance(rc, tuple) else int(rc)) == 0:
                    self._registered.append(int(addr))
            except Exception:  # noqa: BLE001 - a pageable copy still works, just slower
                pass
        return s

    def acquire(self, nbytes: int, stop: Optional[threading.Event] = None) -> Slot:
        """A slot of `nbytes` whose flag is clear (the receiver is done with it),
        flagged as in flight; waits while all `max_slots` slots of that size are."""
        while True:
            with self._lock:
                same = self._by_size.setdefault(nbytes, [])
                for s in same:
                    if s.mm[0] == 0:
                        s.mm[0] = 1
                        return s
                if len(same) < self.max_slots:
                    try:
                        s = self._create(nbytes)
                    except ShmFull:
                        if not same:
                            raise                 # no slot of this size at all: the caller goes inline
                        s = None                  # wait for one of the existing slots instead
                    if s is not None:
                        same.append(s)
                        s.mm[0] = 1
                        return s
            if stop is not None and stop.is_set():
                raise RuntimeError("link stopped while waiting for a free slot")
            time.sleep(0.0002)

    def put(self, arr: np.ndarray, stop: Optional[threading.Event] = None, bf16: bool = False) -> "ShmRef":
        arr = np.ascontiguousarray(arr)
        s = self.acquire(arr.nbytes, stop)
        np.copyto(s.view(arr.dtype, arr.shape), arr)
        return ShmRef(s, arr.dtype, arr.shape, bf16=bf16)

    def close(self) -> None:
        with self._lock:
            for addr in self._registered:
                try:
                    import torch
                    torch.cuda.cudart().cudaHostUnregister(addr)
                except Exception:  # noqa: BLE001
                    pass
            self._registered.clear()
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
            self._by_size.clear()


IPC_HANDLE = 64        # sizeof(hipIpcMemHandle_t)
# device link segment: hand-off header, then pid (u64) | device pointer (u64) | IPC handle
DEV_HDR = LINK_HDR + 16 + IPC_HANDLE


class _DevSlot:
    """Sender side of one device link slot: `copy_` is the device -> slot copy."""
    __slots__ = ("slot", "ptr", "nbytes")

    def __init__(self, slot: Slot, ptr: int, nbytes: int):
        self.slot, self.ptr, self.nbytes = slot, ptr, nbytes

    def copy_(self, src, non_blocking: bool = True) -> None:
        import torch
        from ..ops._lib import kernels, stream_handle
        if not src.is_contiguous() or src.numel() * src.element_size() > self.nbytes:
            raise ValueError("device link slot: source must be contiguous and fit the slot")
        kernels().memcpy_async(self.ptr, int(src.data_ptr()), src.numel() * src.element_size(),
                               stream_handle(torch.cuda.current_stream(src.device)))


class DeviceLinkPool(LinkPool):
    """LinkPool whose slots are device allocations (module docstring)."""

    def __init__(self, device, prefix: Optional[str] = None, max_slots: int = 6):
        super().__init__(prefix=prefix, max_slots=max_slots)
        import torch
        self.device = torch.device(device)
        self._dev: Dict[str, int] = {}

    def _create(self, nbytes: int) -> Slot:
        import torch
        from ..ops._lib import kernels
        K = kernels()
        name = f"{self.prefix}-{len(self._all)}"
        with torch.cuda.device(self.device):
            ptr = K.dev_alloc(max(nbytes, 1))
            handle = K.ipc_handle(ptr)
        try:
            mm = _open_reserved(os.path.join(SHM_DIR, name), DEV_HDR)
        except ShmFull:
            with torch.cuda.device(self.device):
                K.dev_free(ptr)
            raise
        mm[LINK_HDR:LINK_HDR + 16] = os.getpid().to_bytes(8, "little") + int(ptr).to_bytes(8, "little")
        # exporter's device ordinal + 1 in the hand-off header (bytes 8..15; byte 0 is the flag):
        # a receiver on another GPU enables peer access to it before opening the handle
        mm[8:16] = (int(self.device.index or 0) + 1).to_bytes(8, "little")
        if len(handle) != IPC_HANDLE:
            raise RuntimeError(f"device link: IPC handle of {len(handle)} bytes, expected {IPC_HANDLE}")
        mm[LINK_HDR + 16:DEV_HDR] = handle
        s = Slot(self, name, nbytes, mm, len(self._all), offset=0)
        self._all.append(s)
        self._dev[name] = ptr
        return s

    def acquire_dev(self, nbytes: int, stop: Optional[threading.Event] = None) -> _DevSlot:
        s = self.acquire(nbytes, stop)
        return _DevSlot(s, self._dev[s.name], s.nbytes)

    def close(self, handoff_timeout_s: float = 0.0) -> None:
        """Callers synchronise the device first (no copy may still target a slot).

        Freeing an IPC-exported allocation while an importer may still copy out
        of it is undefined (the CUDA IPC contract, which HIP follows).  A torn
        down epoch's pool is therefore not closed at once: the worker retires it
        (`Node.retire_link_pool`) and closes it one epoch later, when every
        importer has long finished or died.  `handoff_timeout_s` additionally
        waits (bounded) for flagged slots: the receiver of a slot clears the
        flag once its copy has retired."""
        import torch
        from ..ops._lib import kernels
        deadline = time.time() + handoff_timeout_s
        with self._lock:
            slots = list(self._all)
        for sl in slots:
            while time.time() < deadline:
                try:
                    if sl.mm[0] == 0:
                        break
                except ValueError:                  # already unmapped
                    break
                time.sleep(0.001)
        with self._lock:
            for ptr in self._dev.values():
                try:
                    with torch.cuda.device(self.device):
                        kernels().dev_free(ptr)
                except Exception:  # noqa: BLE001 - teardown: the process may be exiting
                    pass
            self._dev.clear()
        super().close()


class DevArray:
    """Receiver side of a device link tensor: `ptr` is the slot's device address in
    this process (the IPC mapping is opened once per slot and cached)."""
    __slots__ = ("name", "offset", "dtype", "shape")

    def __init__(self, name: str, offset: int, dtype, shape: Tuple[int, ...]):
        self.name, self.offset, self.dtype, self.shape = name, int(offset), np.dtype(dtype), tuple(shape)

    @property
    def nbytes(self) -> int:
        return int(np.prod(self.shape)) * self.dtype.itemsize

    @property
    def ptr(self) -> int:
        return dev_ptr(self.name) + self.offset


class DevRef:
    """Sender side: a tensor in a device link slot; on the wire the "dev" descriptor."""

    def __init__(self, slot: _DevSlot, dtype, shape: Tuple[int, ...], bf16: bool = False):
        self.slot, self.dtype, self.shape = slot, np.dtype(dtype), tuple(int(v) for v in shape)
        self.bf16 = bf16

    def container(self) -> bytes:
        from .. import codec as C
        return C.wrap(self.slot.slot.name.encode() + b"\0" + (0).to_bytes(8, "little"), "dev",
                      self.dtype, self.shape, bf16=self.bf16)


def dev_ptr(name: str) -> int:
    """Device address of device link slot `name` in this process: the sender's own
    pointer when the sender is this process, else its IPC mapping (opened once)."""
    a = attach(name)
    with _att_lock:
        if a.dptr is None:
            pid = int.from_bytes(bytes(a.mm[LINK_HDR:LINK_HDR + 8]), "little")
            if pid == os.getpid():
                a.dptr = int.from_bytes(bytes(a.mm[LINK_HDR + 8:LINK_HDR + 16]), "little")
            else:
                from ..ops._lib import kernels
                peer = int.from_bytes(bytes(a.mm[8:16]), "little") - 1
                a.dptr = kernels().ipc_open(bytes(a.mm[LINK_HDR + 16:DEV_HDR]), peer)
                a.ipc = True
        return a.dptr


def is_link(name: str) -> bool:
    return name.startswith("adapt-link-")


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
        self.dptr: Optional[int] = None      # device link slot: its device address in this process
        self.ipc = False                     # ... opened from an IPC handle (closed at detach)


class ShmRef:
    """A request tensor that lives in a pool slot: on the wire it is the "shm"
    codec container (segment name + offset), not the bytes."""

    def __init__(self, slot: Slot, dtype, shape: Tuple[int, ...], bf16: bool = False):
        self.slot, self.dtype, self.shape = slot, np.dtype(dtype), tuple(int(v) for v in shape)
        self.bf16 = bf16

    @property
    def array(self) -> np.ndarray:
        return self.slot.view(self.dtype, self.shape)

    def container(self) -> bytes:
        from .. import codec as C
        return C.wrap(self.slot.name.encode() + b"\0" + int(self.slot.offset).to_bytes(8, "little"), "shm",
                      self.dtype, self.shape, bf16=self.bf16)


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
            # under the lock: a second concurrent register of the same pages would
            # fail and leave the first registration untracked (never unregistered)
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


def release(name: str) -> None:
    """Receiver side of a link: the copy out of slot `name` has completed.  A
    segment this process no longer maps (its epoch was torn down and detached)
    is left alone: re-mapping it would leak the mapping, and the sender's pool
    may already have unlinked the file."""
    with _att_lock:
        a = _attached.get(name)
        if a is not None and a.arr is not None:
            a.arr[0] = 0


def detach(names) -> None:
    """Unmap the given attached segments (a finished epoch's link slots)."""
    with _att_lock:
        for n in names:
            a = _attached.pop(n, None)
            if a is None:
                continue
            if a.ipc and a.dptr is not None:
                try:
                    from ..ops._lib import kernels
                    kernels().ipc_close(a.dptr)
                except Exception:  # noqa: BLE001
                    pass
                a.dptr = None
            if a.registered:
                try:
                    import torch
                    torch.cuda.cudart().cudaHostUnregister(int(a.arr.ctypes.data))
                except Exception:  # noqa: BLE001
                    pass
            a.arr = None
            try:
                a.mm.close()
            except (BufferError, ValueError):
                pass                       # a view is still alive: the mapping goes with it


def detach_all() -> None:
    """Unmap every attached segment, closing IPC mappings of device slots too."""
    with _att_lock:
        names = list(_attached)
    detach(names)
