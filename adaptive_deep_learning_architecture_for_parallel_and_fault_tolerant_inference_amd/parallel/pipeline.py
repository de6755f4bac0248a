"""Pipeline stage over RCCL point-to-point (xGMI) — the data plane.

Replaces the reference's TCP activation chain: dispatcher -> node :6000
(`src/dispatcher.py:99-107,204-220`), worker `model.predict` -> node/dispatcher
:6003 (`src/node.py:163-179`), with zfp+lz4 on every hop
(`src/dispatcher.py:92-98`).

One process per MI355X holds one slice.  Per micro-batch tick a stage:

1. waits for the receive of its frontier inputs (issued one tick earlier into
   the *other* buffer set, so it overlapped the previous compute),
2. waits for the send that last used this set's output buffers,
3. replays the slice's hipGraph on the compute stream,
4. posts `isend` of its outputs to the next stage and `irecv` of the
   micro-batch after next into this set's input buffers.

`torch.distributed` with the ``nccl`` backend is RCCL on ROCm; each stage pair
gets its own communicator/stream, so send(t-1), recv(t+1) and compute(t) run
concurrently on different HIP queues.  The same class runs with ``gloo`` on
CPU tensors for the CPU plumbing tests (no GPU).

Frontier tensors are sent in slice-output order; a multi-tensor frontier
(e.g. ``part_at=['conv3_block1_1_conv']``) is just several p2p messages.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional

import torch
import torch.distributed as dist


class StageLink:
    """Double-buffered p2p plumbing around a compute callable.

    ``compute(set_idx)`` must consume ``in_bufs[set_idx]`` and fill
    ``out_bufs[set_idx]`` on the current stream.
    """

    def __init__(self, compute: Callable[[int], None], in_bufs: List[List[torch.Tensor]],
                 out_bufs: List[List[torch.Tensor]], prev_rank: Optional[int], next_rank: Optional[int],
                 group=None, result_rank: Optional[int] = None, result_bufs: Optional[List[torch.Tensor]] = None):
        self.compute = compute
        self.in_bufs = in_bufs
        self.out_bufs = out_bufs
        self.prev = prev_rank
        self.next = next_rank
        self.group = group
        self.nsets = len(in_bufs) if in_bufs else len(out_bufs)
        self.recv_work: List[Optional[list]] = [None] * self.nsets
        self.send_work: List[Optional[list]] = [None] * self.nsets
        self.tick = 0
        self.result_rank = result_rank
        self.result_bufs = result_bufs

    def _irecv(self, j: int):
        return [dist.irecv(t, src=self.prev, group=self.group) for t in self.in_bufs[j]]

    def _isend(self, j: int):
        return [dist.isend(t, dst=self.next, group=self.group) for t in self.out_bufs[j]]

    @staticmethod
    def _wait(works):
        if works:
            for w in works:
                w.wait()

    def prime(self) -> None:
        """Post the first receives (all sets)."""
        if self.prev is not None:
            for j in range(self.nsets):
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
        if self.prev is not None:
            self.recv_work[j] = self._irecv(j)
        self.tick += 1
        return j

    def drain(self) -> None:
        for j in range(self.nsets):
            self._wait(self.send_work[j])
            self.send_work[j] = None

    def cancel_pending_recvs(self) -> None:
        self.recv_work = [None] * self.nsets


def stage_ranks(stage: int, stages: int, replica: int) -> Dict[str, Optional[int]]:
    base = replica * stages
    return {
        "rank": base + stage,
        "prev": base + stage - 1 if stage > 0 else None,
        "next": base + stage + 1 if stage < stages - 1 else None,
    }
