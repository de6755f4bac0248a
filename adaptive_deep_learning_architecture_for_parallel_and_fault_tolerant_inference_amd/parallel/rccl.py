"""Python face of the native RCCL p2p layer (`csrc/comm/rccl_p2p.cpp`, module `_comm`).

The reference forwards activations stage to stage over TCP
(`src/dispatcher.py:204-220`, `src/node.py:163-179`) and has no failure
semantics beyond socket errors and a task watchdog keyed on start time
(`src/dispatcher.py:186-194,302-304`).  Here:

* `RcclComm` is one RCCL communicator, initialised *non-blocking*
  (``ncclCommInitRankConfig`` with ``blocking=0``) from a unique id exchanged
  over a `torch.distributed` store, with an async-error watch thread and an
  ``ncclCommAbort`` callable from any thread;
* `PairLinks` gives a pipeline stage one 2-rank communicator per adjacent
  stage pair, each on its own HIP stream, so the send of micro-batch t-1,
  the receive of t+1 and the compute of t run on three hardware queues;
* `Work` is an event recorded on the link stream behind the grouped
  send/recv: ``wait()`` orders the caller's current stream after it (no host
  block), ``wait_host()`` polls it abortably;
* ``abort()`` is bounded: ``ncclCommAbort`` runs on a native helper thread
  and is waited for at most ``abort_deadline_s`` (3 s).  Past it the
  communicator reports ``abort_stuck``; its owner then publishes
  UNRECOVERABLE and exits non-zero (`StuckAbort`, node.py) so the
  dispatcher re-plans without it and a supervisor may start a fresh process.

Point-to-point matching is FIFO per communicator (RCCL has no tags): every
caller posts its sends and receives in tick order, which the pipeline
schedules do by construction.
"""
from __future__ import annotations

import os
import threading
import time
from typing import Iterable, List, Optional, Sequence

import torch

_mod = None
_lock = threading.Lock()


class LinkError(RuntimeError):
    """A communicator reported an asynchronous error or was aborted."""


class StuckAbort(LinkError):
    """ncclCommAbort did not return within the abort deadline: the process must be given up."""


ABORT_DEADLINE_S = float(os.environ.get("ADAPT_ABORT_DEADLINE_S", "3.0"))


def native():
    """The `_comm` extension; raises if it was not built (never a silent fallback)."""
    global _mod
    with _lock:
        if _mod is None:
            from .. import _comm  # noqa: PLC0415 - built in-tree by _build.build_comm
            hint = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
            _comm.load(hint)
            _mod = _comm
    return _mod


def available() -> bool:
    try:
        native()
        return True
    except Exception:  # noqa: BLE001
        return False


def _exchange_uid(store, key: str, rank: int, root: int = 0, timeout_s: float = 60.0) -> bytes:
    if rank == root:
        uid = native().unique_id()
        store.set(key, uid)
        return uid
    store.wait([key], _td(timeout_s))
    return bytes(store.get(key))


def _td(s: float):
    import datetime
    return datetime.timedelta(seconds=s)


class Work:
    """Completion handle of one grouped enqueue on a link stream."""

    __slots__ = ("event", "comm", "stream")

    def __init__(self, event: torch.cuda.Event, comm: "RcclComm", stream: torch.cuda.Stream):
        self.event, self.comm, self.stream = event, comm, stream

    def wait(self) -> None:
        """Device-side: the caller's current stream waits for the transfer."""
        torch.cuda.current_stream(self.stream.device).wait_event(self.event)

    def is_completed(self) -> bool:
        if self.comm.failed:
            raise LinkError(f"{self.comm.name}: {self.comm.error_text}")
        return self.event.query()

    def wait_host(self, abort_flag: Optional[threading.Event] = None, timeout_s: Optional[float] = None,
                  poll_s: float = 5e-5) -> None:
        t0 = time.monotonic()
        while not self.is_completed():
            if abort_flag is not None and abort_flag.is_set():
                raise LinkError(f"{self.comm.name}: aborted")
            if self.comm.aborted:
                raise LinkError(f"{self.comm.name}: communicator aborted")
            if timeout_s is not None and time.monotonic() - t0 > timeout_s:
                raise LinkError(f"{self.comm.name}: transfer not complete after {timeout_s} s")
            time.sleep(poll_s)


class RcclComm:
    """One non-blocking RCCL communicator with an async-error watch."""

    def __init__(self, store, key: str, nranks: int, rank: int, device, wait: bool = True,
                 timeout_s: float = 60.0, watch_us: int = 1000, abort_on_error: bool = True,
                 stream: Optional[torch.cuda.Stream] = None, abort_deadline_s: Optional[float] = None):
        self.device = torch.device(device)
        self.name = key
        self.nranks, self.rank = nranks, rank
        self.timeout_s = timeout_s
        from . import loopback_comm
        self.loopback = loopback_comm.selected()
        self.t0 = time.perf_counter()
        if self.loopback:
            # TEST-ONLY: two ranks on one GPU (parallel/loopback_comm.py), never a default or a fallback
            self._c = loopback_comm.LoopbackComm(store, key, nranks, rank, self.device.index or 0)
        else:
            uid = _exchange_uid(store, f"{key}/uid", rank, timeout_s=timeout_s)
            self.t0 = time.perf_counter()
            self._c = native().Comm(uid, nranks, rank, self.device.index or 0, False, key[-63:])
            if hasattr(self._c, "set_abort_deadline"):       # (test doubles of `_comm.Comm` may lack it)
                self._c.set_abort_deadline(ABORT_DEADLINE_S if abort_deadline_s is None else abort_deadline_s)
        if watch_us > 0:
            self._c.start_watch(watch_us, abort_on_error)
        self.stream = stream if stream is not None else torch.cuda.Stream(device=self.device)
        if wait:
            self.wait_ready(timeout_s)

    # -- state
    def wait_ready(self, timeout_s: Optional[float] = None) -> float:
        """Poll the non-blocking init to completion; returns init ms."""
        self._c.wait_ready(self.timeout_s if timeout_s is None else timeout_s)
        return self._c.init_ms

    def poll(self) -> int:
        return self._c.poll()

    @property
    def failed(self) -> bool:
        return self._c.failed

    @property
    def aborted(self) -> bool:
        return self._c.aborted

    @property
    def abort_stuck(self) -> bool:
        """ncclCommAbort (or a caller inside RCCL) did not return within the
        abort deadline: this process cannot vouch for its RCCL state any more."""
        return bool(getattr(self._c, "abort_stuck", False))

    @property
    def error_text(self) -> str:
        return self._c.error_text

    @property
    def bytes_sent(self) -> int:
        return self._c.bytes_sent

    @property
    def bytes_recv(self) -> int:
        return self._c.bytes_recv

    # -- data
    def p2p(self, sends: Sequence = (), recvs: Sequence = (), after: Optional[torch.cuda.Event] = None,
            stream: Optional[torch.cuda.Stream] = None) -> Work:
        """One grouped enqueue: ``sends``/``recvs`` are (tensor, peer) pairs.
        ``after``: the link stream first waits for this event (e.g. the compute
        that produced the send buffers)."""
        s = stream or self.stream
        if after is not None:
            s.wait_event(after)
        ops = []
        for t, peer in sends:
            _check_dev(t, self.device)
            ops.append(("s", t.data_ptr(), t.numel() * t.element_size(), int(peer)))
        for t, peer in recvs:
            _check_dev(t, self.device)
            ops.append(("r", t.data_ptr(), t.numel() * t.element_size(), int(peer)))
        try:
            self._c.p2p(ops, s.cuda_stream, self.timeout_s)
        except Exception as e:  # noqa: BLE001
            raise LinkError(f"{self.name}: {e}") from e
        ev = torch.cuda.Event()
        ev.record(s)
        # the caching allocator must not recycle these buffers before the link stream is done
        for t, _ in list(sends) + list(recvs):
            t.record_stream(s)
        return Work(ev, self, s)

    def broadcast(self, t: torch.Tensor, root: int) -> Work:
        _check_dev(t, self.device)
        self._c.broadcast(t.data_ptr(), t.numel() * t.element_size(), root, self.stream.cuda_stream, self.timeout_s)
        ev = torch.cuda.Event()
        ev.record(self.stream)
        return Work(ev, self, self.stream)

    def allreduce_max(self, t: torch.Tensor) -> Work:
        if t.dtype != torch.float32:
            raise TypeError("allreduce_max takes fp32")
        _check_dev(t, self.device)
        self._c.allreduce_max_f32(t.data_ptr(), t.numel(), self.stream.cuda_stream, self.timeout_s)
        ev = torch.cuda.Event()
        ev.record(self.stream)
        return Work(ev, self, self.stream)

    # -- teardown
    def abort(self) -> float:
        """ncclCommAbort (any thread), bounded by the abort deadline; returns
        its latency in ms (check `abort_stuck` afterwards)."""
        return self._c.abort()

    def destroy(self, timeout_s: float = 10.0) -> bool:
        """Tear down once the link stream has drained; returns whether it did.
        The drain is polled, never a blocking stream sync: a peer that died with
        a send or receive still pending on this stream would keep that sync from
        returning, and the abort that releases it would never run.  So the wait
        ends early when the communicator failed or was aborted, and at
        `timeout_s` at the latest.  ncclCommAbort rather than ncclCommFinalize +
        ncclCommDestroy: nothing is left to flush, and abort never waits on the
        peer (a finalize on RCCL 2.26 was seen to block for good after an
        earlier failed group in the process)."""
        ev = torch.cuda.Event()
        ev.record(self.stream)
        t0 = time.monotonic()
        drained = True
        while not ev.query():
            if self.failed or self.aborted or time.monotonic() - t0 > timeout_s:
                drained = False
                break
            time.sleep(1e-4)
        self._c.abort()
        return drained


def _check_dev(t: torch.Tensor, dev: torch.device) -> None:
    if t.device != dev:
        raise ValueError(f"tensor on {t.device}, communicator on {dev}")
    if not t.is_contiguous():
        raise ValueError("p2p needs contiguous tensors")


class PairLinks:
    """A stage's RCCL links to its pipeline neighbours.

    One 2-rank communicator per adjacent pair (global ranks ``a < b``: ``a`` is
    comm rank 0), keyed ``{prefix}/link{a}-{b}`` in the store; each has its own
    HIP stream.  Both inits are started before either is polled, so the order
    in which neighbours arrive cannot deadlock (non-blocking init)."""

    def __init__(self, store, prefix: str, rank: int, prev: Optional[int], next: Optional[int], device,
                 timeout_s: float = 60.0, watch_us: int = 1000):
        self.rank, self.prev, self.next = rank, prev, next
        self.device = torch.device(device)
        self.abort_flag = threading.Event()
        self.inp: Optional[RcclComm] = None
        self.out: Optional[RcclComm] = None
        t0 = time.perf_counter()
        try:
            # the out-link first: this rank publishes that pair's unique id, so the
            # next stage never waits on our own upstream rendezvous
            if next is not None:
                self.out = RcclComm(store, f"{prefix}/link{rank}-{next}", 2, 0, device, wait=False,
                                    timeout_s=timeout_s, watch_us=watch_us)
            if prev is not None:
                self.inp = RcclComm(store, f"{prefix}/link{prev}-{rank}", 2, 1, device, wait=False,
                                    timeout_s=timeout_s, watch_us=watch_us)
            for c in (self.inp, self.out):
                if c is not None:
                    c.wait_ready(timeout_s)
        except BaseException:
            # a half-built pair (e.g. the upstream peer never arrived) must not keep its
            # communicator, watch thread and RCCL resources alive until garbage collection
            self.abort()
            raise
        self.init_ms = (time.perf_counter() - t0) * 1e3

    def comms(self) -> List[RcclComm]:
        return [c for c in (self.inp, self.out) if c is not None]

    def isend(self, tensors: Iterable[torch.Tensor], after: Optional[torch.cuda.Event] = None) -> Work:
        return self.out.p2p(sends=[(t, 1) for t in tensors], after=after)

    def irecv(self, tensors: Iterable[torch.Tensor], after: Optional[torch.cuda.Event] = None) -> Work:
        return self.inp.p2p(recvs=[(t, 0) for t in tensors], after=after)

    def failed(self) -> Optional[str]:
        for c in self.comms():
            if c.failed or c.aborted:
                return f"{c.name}: {c.error_text or 'aborted'}"
        return None

    def abort(self) -> None:
        self.abort_flag.set()
        for c in self.comms():
            c.abort()

    def abort_stuck(self) -> bool:
        return any(c.abort_stuck for c in self.comms())

    def destroy(self, timeout_s: float = 10.0) -> bool:
        """Bounded teardown of both links (see `RcclComm.destroy`); False when a
        link had to be aborted with work still pending."""
        ok = True
        for c in self.comms():
            ok = c.destroy(timeout_s) and ok
        return ok
