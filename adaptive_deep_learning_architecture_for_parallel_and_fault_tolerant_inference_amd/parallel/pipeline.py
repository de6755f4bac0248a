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

With RCCL (``links``: a `parallel.rccl.PairLinks` over the native comm layer)
device tensors go straight onto the wire: each stage pair gets its own
non-blocking communicator and HIP stream, every grouped send/recv starts
behind an event of the compute stream, and the compute stream waits on the
transfer's event, so send(t-1), recv(t+1) and compute(t) overlap on different
hardware queues without the host ever blocking.

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
                 group=None, host_staged: bool = False, links=None):
        self.compute = compute
        self.links = links
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

    @staticmethod
    def _now():
        ev = torch.cuda.Event()
        ev.record()
        return ev

    def _irecv(self, j: int):
        if self.links is not None:       # one grouped receive of the whole frontier
            return [self.links.irecv(self.in_bufs[j], after=self._now())]
        if not self.host_staged:
            return [dist.irecv(t, src=self.prev, group=self.group) for t in self.in_bufs[j]]
        return [_HostRecv(dist.irecv(h, src=self.prev, group=self.group), h, d)
                for h, d in zip(self.in_host[j], self.in_bufs[j])]

    def _isend(self, j: int):
        if self.links is not None:
            return [self.links.isend(self.out_bufs[j], after=self._now())]
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


class CompressedStageLink(StageLink):
    """StageLink whose frontier tensors travel compressed (BASELINE config 3:
    "8-stage pipeline with lz4 activation compression"; the reference
    compresses every hop, `src/dispatcher.py:92-98`, `src/node.py:178`).

    Per frontier tensor and buffer set a `codec.wire.WireCodec` turns the
    stage output into one device byte buffer.  A point-to-point receive must
    know its length, so each tick sends two messages:

    * the byte counts, int64[n_out], on a host (gloo) control group, tag 7;
    * the wire buffers on the data group (RCCL over xGMI, or gloo).

    Schedule of a stage at tick t (set j = t % nsets):

    1. receive t's byte counts, post the data receives, decode into the
       slice's input set j on the compute stream (device-side scan + decode);
    2. compute(j);
    3. enqueue the encode of t's outputs on the codec's side stream behind an
       event of the compute stream;
    4. post the messages of tick t-1: its encode ran beside compute(t).

    The receiver learns a length one tick later than an uncompressed link
    would; with two buffer sets the compute stream still has the next
    micro-batch queued while the host waits.
    """

    SIZE_TAG = 7

    def __init__(self, compute: Callable[[int], None], in_bufs: List[List[torch.Tensor]],
                 out_bufs: List[List[torch.Tensor]], prev_rank: Optional[int], next_rank: Optional[int],
                 codec: str = "lz4", group=None, ctl_group=None, host_staged: bool = False, links=None):
        StageLink.__init__(self, compute, in_bufs, out_bufs, prev_rank, next_rank, group=group, host_staged=False,
                           links=links)
        from ..codec.wire import WireCodec
        self.host_staged = host_staged
        self.ctl = ctl_group
        self.codec = codec
        ref = (out_bufs or in_bufs)[0][0]
        self.gpu = ref.device.type == "cuda"
        self.side = torch.cuda.Stream(device=ref.device) if self.gpu else None
        self.enc = [[WireCodec(codec, t, self.side) for t in s] for s in out_bufs] if next_rank is not None else []
        self.dec = [[WireCodec(codec, t) for t in s] for s in in_bufs] if prev_rank is not None else []
        n_out = len(out_bufs[0]) if out_bufs and out_bufs[0] else 1
        n_in = len(in_bufs[0]) if in_bufs and in_bufs[0] else 1
        self.size_out = [torch.zeros(n_out, dtype=torch.int64) for _ in range(self.nsets)]
        self.size_in = [torch.zeros(n_in, dtype=torch.int64) for _ in range(self.nsets)]
        self.size_recv: List[Optional[object]] = [None] * self.nsets
        self.size_send: List[Optional[object]] = [None] * self.nsets
        self.enc_done: List[Optional[torch.cuda.Event]] = [None] * self.nsets
        self.pending: List[int] = []
        self.raw_bytes = 0
        self.wire_bytes = 0
        self.staged = host_staged and self.gpu
        if self.staged:
            self.host_out = [[torch.empty(e.wire.numel(), dtype=torch.uint8, pin_memory=True) for e in s]
                             for s in self.enc]
            self.host_in = [[torch.empty(d.wire.numel(), dtype=torch.uint8, pin_memory=True) for d in s]
                            for s in self.dec]

    @property
    def ratio(self) -> Optional[float]:
        return self.raw_bytes / self.wire_bytes if self.wire_bytes else None

    def _post_size_recv(self, j: int) -> None:
        self.size_recv[j] = dist.irecv(self.size_in[j], src=self.prev, group=self.ctl, tag=self.SIZE_TAG)

    def prime(self, total_ticks: Optional[int] = None) -> None:
        self.total_ticks = total_ticks
        if self.prev is not None:
            for j in range(self.nsets):
                if total_ticks is None or j < total_ticks:
                    self._post_size_recv(j)

    def _recv(self, j: int) -> None:
        self.size_recv[j].wait()
        self.size_recv[j] = None
        sizes = [int(v) for v in self.size_in[j].tolist()]
        works = []
        if self.links is not None:
            works.append(self.links.irecv([d.wire[:nb] for d, nb in zip(self.dec[j], sizes)], after=self._now()))
        for k, (d, nb) in enumerate(zip(self.dec[j], sizes) if self.links is None else []):
            if self.staged:
                h = self.host_in[j][k]
                dist.recv(h[:nb], src=self.prev, group=self.group)
                d.wire[:nb].copy_(h[:nb], non_blocking=False)
            else:
                works.append(dist.irecv(d.wire[:nb], src=self.prev, group=self.group))
        for w in works:
            w.wait()                 # RCCL: the compute stream waits for the receive; gloo: host wait
        for d, nb, buf in zip(self.dec[j], sizes, self.in_bufs[j]):
            d.decode(nb, buf)
        total = getattr(self, "total_ticks", None)
        if total is None or self.tick + self.nsets < total:
            self._post_size_recv(j)

    def _send(self, j: int) -> None:
        sizes = [e.nbytes() for e in self.enc[j]]          # waits for set j's encode only
        if self.size_send[j] is not None:
            self.size_send[j].wait()
        self.size_out[j].copy_(torch.tensor(sizes, dtype=torch.int64))
        self.size_send[j] = dist.isend(self.size_out[j], dst=self.next, group=self.ctl, tag=self.SIZE_TAG)
        works = []
        if self.links is not None:
            for e, nb in zip(self.enc[j], sizes):
                self.raw_bytes += e.n
                self.wire_bytes += nb
            ev = torch.cuda.Event()
            ev.record(self.side)                            # behind set j's encode
            works.append(self.links.isend([e.wire[:nb] for e, nb in zip(self.enc[j], sizes)], after=ev))
        for k, (e, nb) in enumerate(zip(self.enc[j], sizes) if self.links is None else []):
            self.raw_bytes += e.n
            self.wire_bytes += nb
            if self.staged:
                h = self.host_out[j][k]
                h[:nb].copy_(e.wire[:nb])                   # the encode is complete (nbytes waited)
                works.append(dist.isend(h[:nb], dst=self.next, group=self.group))
            elif self.gpu:
                with torch.cuda.stream(self.side):          # RCCL orders the send after the encode
                    works.append(dist.isend(e.wire[:nb], dst=self.next, group=self.group))
            else:
                works.append(dist.isend(e.wire[:nb], dst=self.next, group=self.group))
        self.send_work[j] = works

    def _release(self, j: int) -> None:
        """Set j's wire buffers are about to be re-encoded: their send must be done."""
        works = self.send_work[j]
        if not works:
            return
        if self.gpu and not self.staged:
            with torch.cuda.stream(self.side):
                for w in works:
                    w.wait()
        else:
            for w in works:
                w.wait()
        self.send_work[j] = None

    def step(self) -> int:
        j = self.tick % self.nsets
        if self.prev is not None:
            self._recv(j)
        if self.gpu and self.enc_done[j] is not None:
            # compute(j) overwrites the outputs that set j's last encode reads
            torch.cuda.current_stream().wait_event(self.enc_done[j])
        self.compute(j)
        if self.next is not None:
            self._release(j)
            if self.gpu:
                ev = torch.cuda.Event()
                ev.record()
                for e, t in zip(self.enc[j], self.out_bufs[j]):
                    self.enc_done[j] = e.encode(t, after=ev)
            else:
                for e, t in zip(self.enc[j], self.out_bufs[j]):
                    e.encode(t)
            for p in self.pending:
                self._send(p)
            self.pending = [j]
        self.tick += 1
        return j

    def flush(self) -> None:
        """Post the deferred messages now (a host-side sync point follows, e.g. a
        barrier: the peer must not wait for a tick this rank will not run)."""
        for p in self.pending:
            self._send(p)
        self.pending = []

    def drain(self) -> None:
        self.flush()
        for j in range(self.nsets):
            self._release(j)
            if self.size_send[j] is not None:
                self.size_send[j].wait()
                self.size_send[j] = None
        for row in self.dec:
            for d in row:
                d.check()


def stage_ranks(stage: int, stages: int, replica: int) -> Dict[str, Optional[int]]:
    base = replica * stages
    return {
        "rank": base + stage,
        "prev": base + stage - 1 if stage > 0 else None,
        "next": base + stage + 1 if stage < stages - 1 else None,
    }
