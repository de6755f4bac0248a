"""TEST-ONLY stand-in for the native RCCL communicator (`_comm.Comm`, csrc/comm/rccl_p2p.cpp) between two
processes that share ONE GPU.

Why it exists: `DEFER(transport="rccl")` runs the stage data plane through `EpochGroup(backend="nccl")` ->
`PairLinks` -> `CollectiveStageRuntime._data_loop` (its non-staged, device-ordered path), but RCCL refuses
two ranks on one device, and the test box has one GPU.  Without a stand-in that branch -- the reference's
core hop, device to device (`/root/reference/src/dispatcher.py:204-220`, `src/node.py:163-179`) -- would
only ever execute on the driver's 8-GPU node.  This module gives it the same interface as the native
communicator, with the data moved through device memory exported by IPC handle:

* each rank of a link exports a ring of `depth` slots (device memory, `ADAPT_LOOPBACK_SLOT_MB` each) for
  the messages it sends; the peer opens it by IPC handle (`transport/shm.py` does the same for device
  links);
* a message is one grouped `p2p` call: a send enqueues, on the link stream, a wait for its slot to be free,
  device copies of every tensor into the slot and a counter store; a receive enqueues a wait for that
  counter, the copies out and a "consumed" counter store (`csrc/kernels/loopback.hip`); the counters, a
  shared abort word and per-rank status words live in a page-locked /dev/shm control block both
  processes map;
* `abort()` raises the shared abort word, which ends every spinning wait of both ranks (ncclCommAbort's
  role); a wait that ends by abort or by its time bound marks the communicator failed, so `Work` raises.

It is selected ONLY when a test sets ``ADAPT_TEST_LOOPBACK_COMM=1`` in the worker processes'
environment (parallel/rccl.py `RcclComm`); it is never a default and never a fallback for a missing RCCL.
"""
from __future__ import annotations

import mmap
import os
import threading
import time
import uuid

import numpy as np
import torch

ENV_FLAG = "ADAPT_TEST_LOOPBACK_COMM"
CTL_BYTES = 4096
# control block words (bytes): per direction d (0: rank 0 -> 1, 1: rank 1 -> 0) posted / consumed u64
_POSTED = (0, 16)
_CONSUMED = (8, 24)
_ABORT = 64                      # int32
_STATUS = (128, 192)             # int32 per rank: 0 ok, 2 a wait timed out, 3 a wait saw the abort word


def selected() -> bool:
    return os.environ.get(ENV_FLAG) == "1"


def _kernels():
    from ..ops._lib import kernels
    return kernels()


class LoopbackComm:
    """The `_comm.Comm` surface RcclComm uses: wait_ready / init_ms / start_watch / poll / failed / aborted /
    error_text / bytes_sent / bytes_recv / p2p / abort."""

    def __init__(self, store, key: str, nranks: int, rank: int, device_index: int, depth: int = 3,
                 wait_timeout_s: float = 900.0):
        if nranks != 2 or rank not in (0, 1):
            raise ValueError("the loopback communicator links exactly two ranks")
        self.store, self.key, self.rank = store, key, rank
        self.device = torch.device("cuda", device_index)
        self.depth = depth
        self.cap = int(os.environ.get("ADAPT_LOOPBACK_SLOT_MB", "64")) << 20
        self.wait_ms = wait_timeout_s * 1e3
        self.init_ms = 0.0
        self._t0 = time.perf_counter()
        self._aborted = False
        self._fail_text = ""
        self._sent = self._recvd = 0              # messages
        self.bytes_sent = self.bytes_recv = 0
        self._lock = threading.Lock()
        K = _kernels()
        with torch.cuda.device(self.device):
            self._ring = K.dev_alloc(self.depth * self.cap)        # this rank's outgoing slots
            handle = K.ipc_handle(self._ring)
        self._peer_ring = None
        self._ctl_name = None
        self._mm = None
        self._ctl_host = self._ctl_dev = 0
        store.set(f"{key}/lb_ring{rank}", handle)
        store.set(f"{key}/lb_owner{rank}", f"{os.getpid()}:{self._ring}".encode())
        if rank == 0:                                              # rank 0 owns the control block
            self._ctl_name = f"adapt-lb-{uuid.uuid4().hex[:16]}"
            self._map_ctl(create=True)
            store.set(f"{key}/lb_ctl", self._ctl_name.encode())

    # -- setup
    def _map_ctl(self, create: bool) -> None:
        path = os.path.join("/dev/shm", self._ctl_name)
        fd = os.open(path, os.O_RDWR | (os.O_CREAT | os.O_EXCL if create else 0), 0o600)
        try:
            if create:
                os.ftruncate(fd, CTL_BYTES)
            self._mm = mmap.mmap(fd, CTL_BYTES)
        finally:
            os.close(fd)
        self._arr = np.frombuffer(self._mm, dtype=np.uint8)
        self._ctl_host = int(self._arr.ctypes.data)
        with torch.cuda.device(self.device):
            self._ctl_dev = _kernels().host_register(self._ctl_host, CTL_BYTES)

    def start_watch(self, watch_us: int, abort_on_error: bool) -> None:
        pass                                                       # errors surface through `failed`

    def wait_ready(self, timeout_s: float) -> None:
        import datetime
        if self._peer_ring is not None:
            return
        peer = 1 - self.rank
        self.store.wait([f"{self.key}/lb_ring{peer}", f"{self.key}/lb_owner{peer}"],
                        datetime.timedelta(seconds=timeout_s))
        if self.rank == 1:
            self.store.wait([f"{self.key}/lb_ctl"], datetime.timedelta(seconds=timeout_s))
            self._ctl_name = bytes(self.store.get(f"{self.key}/lb_ctl")).decode()
            self._map_ctl(create=False)
        pid, ptr = bytes(self.store.get(f"{self.key}/lb_owner{peer}")).decode().split(":")
        if int(pid) == os.getpid():                   # both ranks in one process: no IPC mapping of our own
            self._peer_ring = int(ptr)
        else:
            with torch.cuda.device(self.device):
                self._peer_ring = _kernels().ipc_open(bytes(self.store.get(f"{self.key}/lb_ring{peer}")), -1)
        self.init_ms = (time.perf_counter() - self._t0) * 1e3

    # -- state
    def _word(self, off: int, dtype) -> int:
        return int(np.frombuffer(self._mm, dtype=dtype, count=1, offset=off)[0])

    def poll(self) -> int:
        return 1 if self.failed else 0

    @property
    def failed(self) -> bool:
        if self._fail_text:
            return True
        if self._mm is None:
            return False
        if self._word(_ABORT, np.int32):
            self._fail_text = "aborted (loopback abort word)"
            return True
        st = self._word(_STATUS[self.rank], np.int32)
        if st:
            self._fail_text = "loopback wait timed out" if st == 2 else "loopback wait ended by an abort"
            return True
        return False

    @property
    def aborted(self) -> bool:
        return self._aborted or (self._mm is not None and self._word(_ABORT, np.int32) != 0)

    @property
    def error_text(self) -> str:
        return self._fail_text

    # -- data
    def p2p(self, ops, stream: int, timeout_s: float) -> None:
        """One grouped message: all ("s", ptr, nbytes, peer) ops form one message to the peer, all ("r", ...)
        ops one message from it (PairLinks groups one direction per call)."""
        if self._peer_ring is None:
            self.wait_ready(timeout_s)
        if self.aborted:
            raise RuntimeError(f"{self.key}: communicator aborted")
        K = _kernels()
        sends = [(p, n) for k, p, n, _ in ops if k == "s"]
        recvs = [(p, n) for k, p, n, _ in ops if k == "r"]
        d_out, d_in = self.rank, 1 - self.rank
        stat = self._ctl_dev + _STATUS[self.rank]
        abort = self._ctl_dev + _ABORT
        with self._lock:
            if sends:
                total = sum(n for _, n in sends)
                if total > self.cap:
                    raise RuntimeError(f"{self.key}: a {total}-byte message exceeds the {self.cap}-byte loopback "
                                       f"slot (ADAPT_LOOPBACK_SLOT_MB)")
                self._sent += 1
                seq = self._sent
                slot = self._ring + (seq % self.depth) * self.cap
                K.lb_wait(self._ctl_dev + _CONSUMED[d_out], max(0, seq - self.depth), abort, stat, self.wait_ms,
                          stream)
                off = 0
                for p, n in sends:
                    K.memcpy_async(slot + off, p, n, stream)
                    off += n
                K.lb_signal(self._ctl_dev + _POSTED[d_out], seq, stream)
                self.bytes_sent += total
            if recvs:
                self._recvd += 1
                seq = self._recvd
                slot = self._peer_ring + (seq % self.depth) * self.cap
                K.lb_wait(self._ctl_dev + _POSTED[d_in], seq, abort, stat, self.wait_ms, stream)
                off = 0
                for p, n in recvs:
                    K.memcpy_async(p, slot + off, n, stream)
                    off += n
                K.lb_signal(self._ctl_dev + _CONSUMED[d_in], seq, stream)
                self.bytes_recv += off

    def broadcast(self, *a, **k):
        raise NotImplementedError("the loopback communicator carries point-to-point stage links only")

    def allreduce_max_f32(self, *a, **k):
        raise NotImplementedError("the loopback communicator carries point-to-point stage links only")

    # -- teardown
    def abort(self) -> float:
        """Raise the shared abort word (every pending wait of both ranks ends); returns ms.  The rings are
        not freed: the peer may still be copying out of them (the IPC contract); a test-only leak of
        3 slots per link and epoch.  Rank 0 unlinks the control block's name (mappings stay valid)."""
        t0 = time.perf_counter()
        self._aborted = True
        if self._mm is not None:
            np.frombuffer(self._mm, dtype=np.int32, count=1, offset=_ABORT)[0] = 1
        if self.rank == 0 and self._ctl_name:
            try:
                os.unlink(os.path.join("/dev/shm", self._ctl_name))
            except OSError:
                pass
        return (time.perf_counter() - t0) * 1e3
