"""Pipeline stage over RCCL point-to-point (xGMI) — the data plane.

Replaces the reference's TCP activation chain: dispatcher -> node :6000
(`src/dispatcher.py:99-107,204-220`), worker `model.predict` -> node/dispatcher
:6003 (`src/node.py:163-179`), with zfp+lz4 on every hop
(`src/dispatcher.py:92-98`).

One process per MI355X holds one slice.  Per micro-batch tick a stage:

1. waits for the receive of its frontier inputs (posted one tick earlier
   into the *other* buffer set, so it overlapped the previous compute),
2. waits for the send that last used this set's output buffers,
3. replays the slice's hipGraph on the compute stream,
4. posts `isend` of its outputs to the next stage and `irecv` of the
   micro-batch after next into this set's input buffers.

With the ``nccl`` backend (= RCCL on ROCm) device tensors go straight onto
the wire: each stage pair gets its own communicator and HIP stream, and
torch orders the RCCL stream after the compute stream, so send(t-1),
recv(t+1) and compute(t) overlap on different hardware queues.

``host_staged=True`` stages device tensors through host memory and uses a
CPU backend (gloo).  It exists for CPU-only tests and for rehearsing the
multi-stage schedule with several ranks on one GPU (RCCL refuses two ranks
on one device); it is never the production path.

Frontier tensors are sent in slice-output order; a multi-tensor frontier
(e.g. ``part_at=['conv3_block1_1_conv']``) is just several p2p messages.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional

import torch
import torch.distributed as dist


class _HostRecv:
    """irecv into a host mirror; wait() copies it to the device buffer."""

    def __init__(self, work, host: torch.Tensor, dev: torch.Tensor):
        self.work, self.host, self.dev = work, host, dev

    def wait(self):
        self.work.wait()
        if self.dev is not self.host:
            # blocking copy: the next irecv may land in this host mirror right after
            self.dev.copy_(self.host, non_blocking=False)


class StageLink:
    """Double-buffered p2p plumbing around a compute callable.

    ``compute(set_idx)`` must consume ``in_bufs[set_idx]`` and fill
    ``out_bufs[set_idx]`` on the current stream.
    """

    def __init__(self, compute: Callable[[int], None], in_bufs: List[List[torch.Tensor]],
                 out_bufs: List[List[torch.Tensor]], prev_rank: Optional[int], next_rank: Optional[int],
                 group=None, host_staged: bool = False):
        self.compute = compute
        self.in_bufs = in_bufs
        self.out_bufs = out_bufs
        self.prev = prev_rank
        self.next = next_rank
        self.group = group
        self.host_staged = host_staged
        self.nsets = max(len(in_bufs), len(out_bufs))
        self.recv_work: List[Optional[list]] = [None] * self.nsets
        self.send_work: List[Optional[list]] = [None] * self.nsets
        self.tick = 0
        if host_staged:
            def mirror(t):
                return t if t.device.type == "cpu" else torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
            self.in_host = [[mirror(t) for t in s] for s in in_bufs]
            self.out_host = [[mirror(t) for t in s] for s in out_bufs]

    def _irecv(self, j: int):
        if not self.host_staged:
            return [dist.irecv(t, src=self.prev, group=self.group) for t in self.in_bufs[j]]
        return [_HostRecv(dist.irecv(h, src=self.prev, group=self.group), h, d)
                for h, d in zip(self.in_host[j], self.in_bufs[j])]

    def _isend(self, j: int):
        if not self.host_staged:
            return [dist.isend(t, dst=self.next, group=self.group) for t in self.out_bufs[j]]
        works = []
        for h, d in zip(self.out_host[j], self.out_bufs[j]):
            if h is not d:
                h.copy_(d)               # synchronous D2H: the compute that filled d is done
            works.append(dist.isend(h, dst=self.next, group=self.group))
        return works

    @staticmethod
    def _wait(works):
        if works:
            for w in works:
                w.wait()

    def prime(self, total_ticks: Optional[int] = None) -> None:
        """Post the first receives.  With `total_ticks` known, no receive is ever
        posted for a micro-batch that will not be sent (so teardown finds no
        dangling p2p ops)."""
        self.total_ticks = total_ticks
        if self.prev is not None:
            for j in range(self.nsets):
                if total_ticks is None or j < total_ticks:
                    self.recv_work[j] = self._irecv(j)

    def step(self) -> int:
        """Process one micro-batch; returns the buffer set used."""
        j = self.tick % self.nsets
        if self.prev is not None:
            self._wait(self.recv_work[j])
            self.recv_work[j] = None
        self._wait(self.send_work[j])
        self.send_work[j] = None
        self.compute(j)
        if self.next is not None:
            self.send_work[j] = self._isend(j)
        total = getattr(self, "total_ticks", None)
        if self.prev is not None and (total is None or self.tick + self.nsets < total):
            self.recv_work[j] = self._irecv(j)
        self.tick += 1
        return j

    def drain(self) -> None:
        for j in range(self.nsets):
            self._wait(self.send_work[j])
            self.send_work[j] = None


def stage_ranks(stage: int, stages: int, replica: int) -> Dict[str, Optional[int]]:
    base = replica * stages
    return {
        "rank": base + stage,
        "prev": base + stage - 1 if stage > 0 else None,
        "next": base + stage + 1 if stage < stages - 1 else None,
    }
