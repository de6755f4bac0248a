"""Per-epoch communicator for the stage workers of one pipeline.

RCCL communicators are static and block on a dead peer (SURVEY §5.8,
§7.4 item 4).  Every pipeline *epoch* therefore gets a fresh backend
process-group object built directly on a `PrefixStore` (no global default
group), so a failed epoch can be aborted (`ncclCommAbort` under
`ProcessGroupNCCL.abort()`) and replaced in-process while the worker keeps
its resident weights, HIP context and captured graphs:

* the dispatcher hosts the rendezvous `TCPStore`; the prefix
  ``adapt/epoch{e}/`` isolates epochs,
* ``nccl`` (= RCCL over xGMI) for GPU stages, ``gloo`` for CPU stages / tests,
* every wait is *abortable*: NCCL work is waited on with stream
  dependencies plus host polling of CUDA events, gloo work with
  `is_completed()` polling, both checking an abort flag;
* a *stall watch* stands in for ``ncclCommGetAsyncError``: a send the peer
  has not taken within ``stall_s`` (receivers post their receives a buffer set
  ahead, so a healthy send completes within a few stage times) raises
  `LinkStalled` from the next wait, which fails the epoch -> LINK_ERROR ->
  re-plan.  The backend's own op timeout is set far out (``op_timeout_s``): an
  idle pipeline legitimately keeps receives posted for as long as no request
  comes, and the NCCL watchdog must not tear the worker down for that.
"""
from __future__ import annotations

import datetime
import threading
import time
from typing import Optional

import torch
import torch.distributed as dist


class Aborted(RuntimeError):
    """The epoch was aborted (peer failure or reconfiguration)."""


class LinkStalled(RuntimeError):
    """A send was not taken by its peer within the stall bound."""


def make_store_server(host: str = "0.0.0.0", port: int = 0) -> dist.TCPStore:
    return dist.TCPStore(host, port, None, True, timeout=datetime.timedelta(seconds=30), wait_for_workers=False)


class EpochGroup:
    def __init__(self, backend: str, store_host: str, store_port: int, epoch: int, rank: int, world: int,
                 device: Optional[torch.device] = None, timeout_s: float = 30.0, ctl: bool = False,
                 stall_s: float = 10.0, op_timeout_s: float = 7 * 86400.0):
        self.backend = backend
        self.rank, self.world, self.epoch = rank, world, epoch
        self.device = device
        self.abort_flag = threading.Event()
        self.stall_s = stall_s
        self._sends: list = []                   # (work, posted_at) not yet seen complete
        store = dist.TCPStore(store_host, store_port, None, False, timeout=datetime.timedelta(seconds=timeout_s))
        self.store = dist.PrefixStore(f"adapt/epoch{epoch}/", store)
        to = datetime.timedelta(seconds=op_timeout_s)
        if backend == "nccl":
            if device is not None:
                torch.cuda.set_device(device)
            opts = dist.ProcessGroupNCCL.Options()
            opts._timeout = to
            self.pg = dist.ProcessGroupNCCL(self.store, rank, world, opts)
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
    def isend(self, t: torch.Tensor, dst: int, tag: int = 0):
        w = self.pg.send([t], dst, tag)
        if self.backend == "nccl":               # gloo send work only completes inside wait()
            self._sends.append((w, time.monotonic()))
        return w

    def check_stall(self) -> None:
        """Raise `LinkStalled` if a posted send has waited longer than `stall_s`."""
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

    def irecv(self, t: torch.Tensor, src: int, tag: int = 0):
        return self.pg.recv([t], src, tag)

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

    def wait_host(self, work, poll_s: float = 0.0002) -> None:
        """Abortable wait on a host (gloo) work item: gloo p2p work only progresses
        inside wait(), so it runs on a helper thread that an abort can abandon."""
        if work is None:
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
        for pg in (self.pg, self.ctl):
            if pg is None:
                continue
            try:
                pg.abort()
            except Exception:  # noqa: BLE001 - best effort; the group is discarded either way
                pass
