"""Per-epoch communicator for the stage workers of one pipeline.

RCCL communicators are static and block on a dead peer (SURVEY §5.8,
§7.4 item 4).  Every pipeline *epoch* therefore gets a fresh backend
process-group object built directly on a `PrefixStore` (no global default
group), so a failed epoch can be aborted (`ncclCommAbort` under
`ProcessGroupNCCL.abort()`) and replaced in-process while the worker keeps
its resident weights, HIP context and captured graphs:

* the dispatcher hosts the rendezvous `TCPStore`; the prefix
  ``adapt/epoch{e}/`` isolates epochs,
* ``nccl`` (= RCCL over xGMI) for GPU stages goes through the *native* comm
  layer (`parallel/rccl.py` over `csrc/comm/rccl_p2p.cpp`): one non-blocking
  2-rank communicator per adjacent stage pair, each on its own HIP stream, an
  ``ncclCommGetAsyncError`` watch thread per communicator, and
  ``ncclCommAbort`` on abort.  ``gloo`` serves CPU stages and the host-staged
  rehearsal of GPU stages;
* every wait is *abortable*: RCCL work is waited on with stream dependencies
  plus host polling of HIP events (which also checks the async-error state),
  gloo work with `is_completed()` polling, both checking an abort flag;
* a wedged but *alive* peer is found by the dispatcher's progress watch (each
  worker's heartbeat carries its completed-micro-batch counter), not here; the
  send-age *stall watch* below is only a last-resort bound (``stall_s``).  The
  backend op timeout is set far out (``op_timeout_s``): an idle pipeline
  legitimately keeps receives posted for as long as no request comes.
"""
from __future__ import annotations

import datetime
import threading
import time
from typing import Optional

import torch
import torch.distributed as dist

from .rccl import ABORT_DEADLINE_S


class Aborted(RuntimeError):
    """The epoch was aborted (peer failure or reconfiguration)."""


class LinkStalled(RuntimeError):
    """A send was not taken by its peer within the stall bound, or the link's
    communicator reported an asynchronous error."""


def make_store_server(host: str = "0.0.0.0", port: int = 0) -> dist.TCPStore:
    return dist.TCPStore(host, port, None, True, timeout=datetime.timedelta(seconds=30), wait_for_workers=False)


class EpochGroup:
    def __init__(self, backend: str, store_host: str, store_port: int, epoch: int, rank: int, world: int,
                 device: Optional[torch.device] = None, timeout_s: float = 30.0, ctl: bool = False,
                 stall_s: float = 5.0, op_timeout_s: float = 7 * 86400.0):
        self.backend = backend
        self.rank, self.world, self.epoch = rank, world, epoch
        self.device = device
        self.abort_flag = threading.Event()
        self._pg_stuck = False
        self.stall_s = stall_s
        self._sends: list = []                   # (work, posted_at) not yet seen complete
        self.links = None
        self.pg = None
        store = dist.TCPStore(store_host, store_port, None, False, timeout=datetime.timedelta(seconds=timeout_s))
        self.store = dist.PrefixStore(f"adapt/epoch{epoch}/", store)
        to = datetime.timedelta(seconds=op_timeout_s)
        if backend == "nccl":
            from .rccl import PairLinks
            if device is not None:
                torch.cuda.set_device(device)
            self.links = PairLinks(self.store, "rccl", rank, rank - 1 if rank > 0 else None,
                                   rank + 1 if rank < world - 1 else None, device, timeout_s=timeout_s)
        elif backend == "gloo":
            self.pg = dist.ProcessGroupGloo(self.store, rank, world, to)
        else:
            raise ValueError(f"unknown backend {backend}")
        # host control group (compressed links: per-message byte counts travel here,
        # so a receiver can size its data receive without a device round trip)
        self.ctl = None
        if ctl:
            self.ctl = dist.ProcessGroupGloo(dist.PrefixStore("ctl/", self.store), rank, world, to)

    # ------------------------------------------------------------- p2p
    def _after(self):
        """Event on the caller's stream: the link stream starts behind it (the
        compute that filled a send buffer / last read a receive buffer)."""
        ev = torch.cuda.Event()
        ev.record()
        return ev

    def isend(self, t: torch.Tensor, dst: int, tag: int = 0):
        return self.isend_many([t], dst, tag)[0]

    def isend_many(self, ts, dst: int, tag: int = 0) -> list:
        """Send several tensors to `dst`.  RCCL: one grouped enqueue (order-matched
        with the peer's `irecv_many`; tags are not used).  gloo: one send each."""
        if self.links is not None:
            if dst != self.links.next:
                raise ValueError(f"rank {self.rank} has no link to {dst}")
            w = self.links.isend(list(ts), after=self._after())
            self._sends.append((w, time.monotonic()))
            return [w]
        return [self.pg.send([t], dst, tag + k) for k, t in enumerate(ts)]

    def irecv(self, t: torch.Tensor, src: int, tag: int = 0):
        return self.irecv_many([t], src, tag)[0]

    def irecv_many(self, ts, src: int, tag: int = 0) -> list:
        if self.links is not None:
            if src != self.links.prev:
                raise ValueError(f"rank {self.rank} has no link from {src}")
            return [self.links.irecv(list(ts), after=self._after())]
        return [self.pg.recv([t], src, tag + k) for k, t in enumerate(ts)]

    def check_stall(self) -> None:
        """Raise `LinkStalled` if a link's communicator reported an async error,
        or a posted send has waited longer than `stall_s`."""
        if self.links is not None:
            bad = self.links.failed()
            if bad and not self.abort_flag.is_set():
                raise LinkStalled(f"epoch {self.epoch}: {bad}")
        if not self._sends:
            return
        now = time.monotonic()
        keep = []
        for w, t0 in self._sends:
            try:
                done = w.is_completed()
            except Exception as e:  # noqa: BLE001 - a failed work is a broken link
                raise LinkStalled(f"epoch {self.epoch}: send failed: {e}") from e
            if done:
                continue
            if now - t0 > self.stall_s:
                raise LinkStalled(f"epoch {self.epoch}: a send waited {now - t0:.1f} s for its peer")
            keep.append((w, t0))
        self._sends = keep

    def wait(self, work, poll_s: float = 0.0002) -> None:
        """Abortable wait.  NCCL: make the current stream depend on the work
        (host returns immediately; host-side progress is bounded elsewhere by
        `wait_event`).  gloo: poll completion on the host."""
        if work is None:
            return
        if self.backend == "nccl":
            work.wait()
            return
        self.wait_host(work, poll_s)

    def wait_all(self, works) -> None:
        for w in works or []:
            self.wait(w)

    def wait_host(self, work, poll_s: float = 0.0002) -> None:
        """Abortable wait on a host (gloo) work item: gloo p2p work only progresses
        inside wait(), so it runs on a helper thread that an abort can abandon."""
        if work is None:
            return
        if self.links is not None and hasattr(work, "wait_host"):
            try:
                work.wait_host(self.abort_flag)
            except Exception as e:  # noqa: BLE001
                if self.abort_flag.is_set():
                    raise Aborted(f"epoch {self.epoch} aborted") from e
                raise LinkStalled(f"epoch {self.epoch}: {e}") from e
            return
        done = threading.Event()
        err: list = []

        def waiter():
            try:
                work.wait()
            except Exception as e:  # noqa: BLE001
                err.append(e)
            done.set()

        threading.Thread(target=waiter, daemon=True).start()
        while not done.wait(poll_s * 50):
            if self.abort_flag.is_set():
                raise Aborted(f"epoch {self.epoch} aborted")
            self.check_stall()
        if err:
            raise err[0]

    def wait_event(self, ev, poll_s: float = 0.0001, timeout_s: Optional[float] = None) -> None:
        """Host-poll a CUDA/HIP event, abortable; watches posted sends for stalls."""
        if ev is None:
            return
        t0 = time.monotonic()
        n = 0
        while not ev.query():
            if self.abort_flag.is_set():
                raise Aborted(f"epoch {self.epoch} aborted")
            n += 1
            if self.links is not None and n % 20 == 0:     # native async-error state: two atomic loads
                self.check_stall()
            if n % 1000 == 0:                    # ~0.1 s
                self.check_stall()
                if timeout_s is not None and time.monotonic() - t0 > timeout_s:
                    raise LinkStalled(f"epoch {self.epoch}: device wait exceeded {timeout_s} s")
            time.sleep(poll_s)

    def ctl_isend(self, t: torch.Tensor, dst: int, tag: int = 0):
        return self.ctl.send([t], dst, tag)

    def ctl_irecv(self, t: torch.Tensor, src: int, tag: int = 0):
        return self.ctl.recv([t], src, tag)

    def abort(self) -> None:
        self.abort_flag.set()
        if self.links is not None:
            try:
                self.links.abort()
            except Exception:  # noqa: BLE001
                pass
        for pg in (self.pg, self.ctl):
            if pg is None:
                continue
            # bounded like the native links: ProcessGroupNCCL.abort() is an ncclCommAbort underneath
            th = threading.Thread(target=_abort_quietly, args=(pg,), daemon=True, name=f"epoch{self.epoch}-pgabort")
            th.start()
            th.join(ABORT_DEADLINE_S)
            if th.is_alive():
                self._pg_stuck = True

    def abort_stuck(self) -> bool:
        """An abort of this epoch's communicators did not return within the deadline."""
        if self._pg_stuck:
            return True
        return self.links is not None and hasattr(self.links, "abort_stuck") and self.links.abort_stuck()


def _abort_quietly(pg) -> None:
    try:
        pg.abort()
    except Exception:  # noqa: BLE001 - best effort; the group is discarded either way
        pass
