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
  `is_completed()` polling, both checking an abort flag.
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


def make_store_server(host: str = "0.0.0.0", port: int = 0) -> dist.TCPStore:
    return dist.TCPStore(host, port, None, True, timeout=datetime.timedelta(seconds=30), wait_for_workers=False)


class EpochGroup:
    def __init__(self, backend: str, store_host: str, store_port: int, epoch: int, rank: int, world: int,
                 device: Optional[torch.device] = None, timeout_s: float = 30.0, ctl: bool = False):
        self.backend = backend
        self.rank, self.world, self.epoch = rank, world, epoch
        self.device = device
        self.abort_flag = threading.Event()
        store = dist.TCPStore(store_host, store_port, None, False, timeout=datetime.timedelta(seconds=timeout_s))
        self.store = dist.PrefixStore(f"adapt/epoch{epoch}/", store)
        to = datetime.timedelta(seconds=timeout_s)
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
        return self.pg.send([t], dst, tag)

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
        if err:
            raise err[0]

    def wait_event(self, ev, poll_s: float = 0.0001) -> None:
        """Host-poll a CUDA/HIP event, abortable."""
        if ev is None:
            return
        while not ev.query():
            if self.abort_flag.is_set():
                raise Aborted(f"epoch {self.epoch} aborted")
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
