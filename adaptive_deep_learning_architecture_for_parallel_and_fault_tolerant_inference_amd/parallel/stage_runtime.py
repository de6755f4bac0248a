"""Node data plane with collective links: RCCL p2p over xGMI between GPU
stages (``nccl``), or gloo between CPU stages.

The reference forwards every activation over TCP, compressed, through the
dispatcher hub (`src/node.py:163-179`, `src/dispatcher.py:121-151,204-220`).
Here only stage 0 (inputs) and the last stage (results) talk TCP to the
dispatcher; stage i -> i+1 is a point-to-point send of device-resident
tensors on the epoch's communicator (parallel/epoch_group.py):

    meta   int64[4] = (req_id, count, epoch, 1)      # rides with the data
    frontier tensors in slice-output order, in the job's precision (the
    executor's buffers: fp32 by default, as the reference; bf16 when the
    job asks for it; always fp32 on CPU stages)

Double-buffered per stage (`nsets` buffer sets): the receive of micro-batch
t+1 and the send of t-1 run on the communicator's HIP stream while t
computes on the compute stream; host run-ahead is bounded by polling one
event per buffer set, and every wait is abortable so a reconfiguration can
tear the epoch down even while a peer is dead.
"""
from __future__ import annotations

import os
import queue
import sys
import threading
import time
import traceback
from typing import Dict, List, Optional

import numpy as np
import torch

from ..graph.manifest import SliceManifest
from ..transport.messages import Message
from .epoch_group import Aborted, EpochGroup


class CollectiveStageRuntime:
    def __init__(self, node, cfg: Dict, manifest: SliceManifest, weights: Dict[str, np.ndarray]):
        self.node = node
        self.cfg = cfg
        self.epoch = int(cfg["epoch"])
        self.stage = int(cfg["stage"])
        self.stages = int(cfg["stages"])
        self.batch = int(cfg["batch"])
        self.codec = cfg.get("codec", "lz4")                 # TCP edges (dispatcher <-> first / last stage)
        self.link_codec = cfg.get("link_codec", "none")      # stage-to-stage collective links
        self.manifest = manifest
        self.nsets = int(cfg.get("nsets", 2))
        g = manifest.graph()
        self.compute = node.stage_compute(cfg, g, weights)
        self.gpu = self.compute.gpu
        self.dev = self.compute.device
        self.group: Optional[EpochGroup] = None     # rendezvous happens on the data thread (after ACK)
        self.prev = self.stage - 1 if self.stage > 0 else None
        self.next = self.stage + 1 if self.stage < self.stages - 1 else None
        self.inq: "queue.Queue" = queue.Queue(maxsize=int(cfg.get("queue", 4)))
        self.outq: "queue.Queue" = queue.Queue(maxsize=int(cfg.get("queue", 4)))
        self.stop = threading.Event()
        self.error: Optional[str] = None
        self.processed = 0
        self.upstream = None
        self.downstream = None
        self.threads: List[threading.Thread] = []
        self._alloc()

    # ------------------------------------------------------------ buffers
    def _alloc(self) -> None:
        c = self.compute
        if self.gpu:
            self.in_bufs = [[c.ex.input_buf(n, j) for n in c.inputs] for j in range(self.nsets)]
            self.out_bufs = [[c.ex.output_buf(n, j) for n in c.outputs] for j in range(self.nsets)]
        else:
            g = self.manifest.graph()
            self.in_bufs = [[torch.zeros((self.batch,) + tuple(g.layers[n].out_shape)) for n in c.inputs]
                            for _ in range(self.nsets)]
            self.out_bufs = [[torch.zeros((self.batch,) + tuple(g.layers[n].out_shape)) for n in c.outputs]
                             for _ in range(self.nsets)]
        mdev = self.dev if self.gpu else torch.device("cpu")
        self.meta_in = [torch.zeros(4, dtype=torch.int64, device=mdev) for _ in range(self.nsets)]
        self.meta_out = [torch.zeros(4, dtype=torch.int64, device=mdev) for _ in range(self.nsets)]
        self.events = [None] * self.nsets
        self.cur_meta = [torch.zeros(4, dtype=torch.int64) for _ in range(self.nsets)]   # host copy per set
        self.enc = self.dec = None
        if self.link_codec != "none":
            from ..codec.wire import WireCodec
            self.side = torch.cuda.Stream(device=self.dev) if self.gpu else None
            if self.next is not None:
                self.enc = [[WireCodec(self.link_codec, t, self.side) for t in st] for st in self.out_bufs]
            if self.prev is not None:
                self.dec = [[WireCodec(self.link_codec, t) for t in st] for st in self.in_bufs]
            # host meta: request id, count, epoch, 1, then the byte count of each wire buffer
            self.hmeta_in = [torch.zeros(4 + len(self.in_bufs[0]), dtype=torch.int64) for _ in range(self.nsets)]
            self.hmeta_out = [torch.zeros(4 + len(self.out_bufs[0]), dtype=torch.int64) for _ in range(self.nsets)]

    # ----------------------------------------------------------- lifecycle
    def attach_upstream(self, sock) -> None:
        """Stage 0 only: TCP connection from the dispatcher."""
        self.upstream = sock
        t = threading.Thread(target=self._tcp_recv_loop, daemon=True, name=f"cstage{self.stage}-tcprecv")
        t.start()
        self.threads.append(t)

    def start(self) -> None:
        t = threading.Thread(target=self._data_loop, daemon=True, name=f"cstage{self.stage}-data-e{self.epoch}")
        t.start()
        self.threads.append(t)
        if self.next is None:
            t = threading.Thread(target=self._tcp_send_loop, daemon=True, name=f"cstage{self.stage}-tcpsend")
            t.start()
            self.threads.append(t)

    def _fail(self, where: str, e: BaseException) -> None:
        report = not self.stop.is_set() and not isinstance(e, Aborted)
        if report:
            self.error = f"{where}: {type(e).__name__}: {e}"
        self.abort()
        if report:
            # same contract as the TCP runtime (node.py): a broken link is
            # published at once so the dispatcher re-plans without the lease TTL
            self.node.report_failure(self, "STAGE_ERROR" if where == "compute" else "LINK_ERROR")

    def quiesced(self) -> bool:
        """No thread of this epoch is still running (safe to reuse its compute)."""
        me = threading.current_thread()
        return not any(t.is_alive() for t in self.threads if t is not me)

    def abort(self) -> None:
        if self.stop.is_set():
            return
        self.stop.set()
        if self.group is not None:
            self.group.abort()
            if self.group.abort_stuck():
                self.node.give_up(self, f"epoch {self.epoch}: communicator abort exceeded its deadline")
        for s in (self.upstream, self.downstream):
            if s is not None:
                try:
                    import socket
                    s.shutdown(socket.SHUT_RDWR)
                except OSError:
                    pass
                try:
                    s.close()
                except OSError:
                    pass
        # bounded join: the loops poll `stop` every <=0.1 s, so a stopped runtime
        # has no thread left inside a device call when the process tears down
        me = threading.current_thread()
        for t in self.threads:
            if t is not me:
                t.join(timeout=2.0)

    # ------------------------------------------------------- TCP edges
    def _tcp_recv_loop(self) -> None:
        from ..transport.messages import recv_message
        try:
            while not self.stop.is_set():
                m = recv_message(self.upstream, self.node.state.chunk_size)
                if m is None:
                    if not self.stop.is_set():
                        raise ConnectionError("dispatcher closed the input link")
                    break
                if m.epoch != self.epoch:
                    continue
                while not self.stop.is_set():
                    try:
                        self.inq.put(m, timeout=0.1)
                        break
                    except queue.Full:
                        continue
        except Exception as e:  # noqa: BLE001
            self._fail("tcp-recv", e)

    def _tcp_send_loop(self) -> None:
        from ..transport.messages import connect, send_message
        import json
        try:
            host, port = self.cfg["result_addr"]
            hello = json.dumps({"epoch": self.epoch, "from_stage": self.stage}).encode()
            self.downstream = connect(host, int(port), hello=hello)
            while not self.stop.is_set():
                try:
                    m = self.outq.get(timeout=0.1)
                except queue.Empty:
                    continue
                send_message(self.downstream, m, self.codec, self.node.state.chunk_size)
        except Exception as e:  # noqa: BLE001
            self._fail("tcp-send", e)

    # -------------------------------------------------------- data loop
    def _next_request(self, j: int) -> bool:
        """Stage 0: fill buffer set j from the dispatcher's next message."""
        from ..runtime.stage import to_torch
        while True:
            if self.stop.is_set():
                raise Aborted("stopped")
            try:
                m: Message = self.inq.get(timeout=0.05)
                break
            except queue.Empty:
                continue
        for name, buf, a, b in zip(self.compute.inputs, self.in_bufs[j], m.tensors, m.bf16):
            t = to_torch(a, b, buf.device)
            if t.dtype != buf.dtype:
                t = t.to(buf.dtype)
            if t.shape[-1] != buf.shape[-1]:
                t = torch.nn.functional.pad(t, (0, buf.shape[-1] - t.shape[-1]))
            buf.zero_() if t.shape[0] < buf.shape[0] else None
            buf[: t.shape[0]].copy_(t)
        self.cur_meta[j] = torch.tensor([m.req_id, m.count, self.epoch, 1], dtype=torch.int64)
        self.meta_in[j].copy_(self.cur_meta[j])
        return True

    def _compute(self, j: int) -> None:
        if self.gpu:
            self.compute.ex.forward(j)
        else:
            # the native CPU path (runtime/cpu_executor.py) works on numpy views of the host buffers
            feed = {n: t.numpy() for n, t in zip(self.compute.inputs, self.in_bufs[j])}
            y = self.compute.ex.run(feed, outputs=self.compute.outputs)
            for t, n in zip(self.out_bufs[j], self.compute.outputs):
                t.copy_(torch.from_numpy(np.ascontiguousarray(y[n])))
        self.meta_out[j].copy_(self.meta_in[j])

    def _emit_result(self, j: int) -> None:
        from ..runtime.stage import to_numpy
        meta = self.meta_out[j].cpu().tolist()
        rid, count = int(meta[0]), int(meta[1])
        outs, flags = [], []
        for t in self.out_bufs[j]:
            a, f = to_numpy(t[:count])
            outs.append(a)
            flags.append(f)
        m = Message(self.stage + 2, rid, self.epoch, count, outs, flags)
        while not self.stop.is_set():
            try:
                self.outq.put(m, timeout=0.1)
                return
            except queue.Full:
                continue

    def _handshake(self, G: EpochGroup) -> None:
        """Connect this epoch's p2p links at formation: RCCL builds a pair's
        communicator on its first send/recv, so without this the first
        micro-batch after every re-plan would pay the communicator setup."""
        dev = self.dev if self.gpu else torch.device("cpu")
        out, inp = torch.ones(1, device=dev), torch.zeros(1, device=dev)
        works = []
        if self.next is not None:
            works.append(G.isend(out, self.next, 99))
        if self.prev is not None:
            works.append(G.irecv(inp, self.prev, 99))
        for w in works:
            G.wait(w)
        if self.gpu:
            ev = torch.cuda.Event()
            ev.record()
            G.wait_event(ev, timeout_s=float(self.cfg["collective"].get("timeout", 30)))

    def _data_loop(self) -> None:
        cc = self.cfg["collective"]
        t0 = time.perf_counter()
        try:
            self.group = EpochGroup(cc["backend"], cc["store_host"], int(cc["store_port"]), self.epoch, self.stage,
                                    self.stages, self.dev if self.gpu else None, float(cc.get("timeout", 30)),
                                    ctl=self.link_codec != "none", stall_s=float(cc.get("stall_s", 5.0)))
            t1 = time.perf_counter()
            self._handshake(self.group)
        except Exception as e:  # noqa: BLE001 - rendezvous failed (a member died): epoch is dead
            self._fail("rendezvous", e)
            return
        self.setup_ms = {"group": round((t1 - t0) * 1e3, 1), "handshake": round((time.perf_counter() - t1) * 1e3, 1)}
        if os.environ.get("ADAPT_EPOCH_TIMING") == "1":
            print(f"cstage{self.stage} epoch {self.epoch}: formed {getattr(self, 'form_ms', {})}, links "
                  f"{self.setup_ms} ms", file=sys.stderr, flush=True)
        if self.stop.is_set():
            self.group.abort()
            return
        G = self.group
        if self.link_codec != "none":
            try:
                self._codec_loop(G)
            except Exception as e:  # noqa: BLE001
                if not isinstance(e, Aborted):
                    traceback.print_exc()
                self._fail("data", e)
            return
        recv_w: List[Optional[list]] = [None] * self.nsets
        send_w: List[Optional[list]] = [None] * self.nsets
        # gloo between GPU stages (the rehearsal of the RCCL path on one device):
        # device tensors are staged through pinned host mirrors, one bulk copy each
        staged = self.gpu and G.backend != "nccl"
        if staged:
            def pinned(t):
                return torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
            h_in = [[pinned(t) for t in [self.meta_in[j]] + self.in_bufs[j]] for j in range(self.nsets)]
            h_out = [[pinned(t) for t in [self.meta_out[j]] + self.out_bufs[j]] for j in range(self.nsets)]

        def post_recv(j):
            # one grouped RCCL receive (meta + frontier) per tick; gloo: one recv per tensor,
            # tags 16*j + k (a set's tags never collide with the next set's)
            dst = h_in[j] if staged else [self.meta_in[j]] + self.in_bufs[j]
            return G.irecv_many(dst, self.prev, 16 * j)

        def land(j):
            if staged:                                   # pinned -> device (the next irecv reuses the mirror)
                for h, d in zip(h_in[j], [self.meta_in[j]] + self.in_bufs[j]):
                    d.copy_(h, non_blocking=False)

        def post_send(j):
            src = [self.meta_out[j]] + self.out_bufs[j]
            if staged:
                G.wait_event(self.events[j])             # abortable: the compute that filled set j is done
                for h, d in zip(h_out[j], src):
                    h.copy_(d)
                src = h_out[j]
            return G.isend_many(src, self.next, 16 * j)

        tick = 0
        t_tick = time.perf_counter()
        try:
            if self.prev is not None:
                for j in range(self.nsets):
                    recv_w[j] = post_recv(j)
            while not self.stop.is_set():
                j = tick % self.nsets
                if self.gpu:
                    G.wait_event(self.events[j])           # bounds host run-ahead to nsets ticks
                if self.prev is None:
                    self._next_request(j)
                else:
                    for w in recv_w[j]:
                        G.wait(w)
                    recv_w[j] = None
                    land(j)
                for w in send_w[j] or []:
                    G.wait(w)
                send_w[j] = None
                slept = self.node.fault_point(self.stop)
                t_c = time.perf_counter() - slept     # an injected delay counts as compute
                self._compute(j)
                if self.gpu:
                    ev = torch.cuda.Event()
                    ev.record()
                    self.events[j] = ev
                if self.next is not None:
                    send_w[j] = post_send(j)
                else:
                    if self.gpu:
                        G.wait_event(self.events[j])     # abortable: never block in a D2H sync
                    self._emit_result(j)
                if self.prev is not None:
                    recv_w[j] = post_recv(j)
                self.processed += 1
                # CPU: the compute itself; GPU: one loop period (host run-ahead is bounded by the events)
                now = time.perf_counter()
                self.node.note_progress(self.epoch, busy_s=(now - t_c) if not self.gpu else now - t_tick)
                t_tick = now
                tick += 1
        except Exception as e:  # noqa: BLE001
            if not isinstance(e, Aborted):
                traceback.print_exc()
            self._fail("data", e)

    # ------------------------------------------------ compressed links
    def _codec_loop(self, G: EpochGroup) -> None:
        """Data loop of a compressed collective link (DEFER ``link_codec``; the
        reference compresses every hop, `src/node.py:178`).  Per frontier tensor a
        `codec.wire.WireCodec` turns the stage output into one wire buffer; the
        request meta and the byte counts travel on the epoch's host control
        group, the wire buffers on the data group (RCCL over xGMI, or gloo).
        Encodes run on a side stream and a sender thread posts them, so the
        compute of the next micro-batch is queued while this one's encode and
        send are in flight."""
        staged = self.gpu and G.backend != "nccl"           # gloo between GPU stages: host-staged wire
        if staged:
            h_out = [[torch.empty(e.wire.numel(), dtype=torch.uint8, pin_memory=True) for e in st]
                     for st in (self.enc or [])]
            h_in = [[torch.empty(d.wire.numel(), dtype=torch.uint8, pin_memory=True) for d in st]
                    for st in (self.dec or [])]
        released = [threading.Event() for _ in range(self.nsets)]
        for e in released:
            e.set()
        sendq: "queue.Queue" = queue.Queue()

        def sender():
            try:
                while not self.stop.is_set():
                    try:
                        j = sendq.get(timeout=0.05)
                    except queue.Empty:
                        continue
                    hm = self.hmeta_out[j]
                    sizes = [e.nbytes() for e in self.enc[j]]     # waits for set j's encode only
                    for k, nb in enumerate(sizes):
                        hm[4 + k] = nb
                    wm = G.ctl_isend(hm, self.next, 2 * j)
                    works = []
                    for k, (e, nb) in enumerate(zip(self.enc[j], sizes)):
                        if staged:
                            h_out[j][k][:nb].copy_(e.wire[:nb])
                            works.append(G.isend(h_out[j][k][:nb], self.next, 2 * j + 1))
                        elif self.gpu:
                            with torch.cuda.stream(self.side):  # RCCL orders the send after the encode
                                works.append(G.isend(e.wire[:nb], self.next, 2 * j + 1))
                        else:
                            works.append(G.isend(e.wire[:nb], self.next, 2 * j + 1))
                    G.wait_host(wm)
                    for w in works:
                        if self.gpu and not staged:
                            with torch.cuda.stream(self.side):  # the next encode into this wire waits for it
                                w.wait()
                        else:
                            G.wait_host(w)
                    released[j].set()
            except Exception as e:  # noqa: BLE001
                if not isinstance(e, Aborted):
                    traceback.print_exc()
                self._fail("send", e)

        if self.next is not None:
            t = threading.Thread(target=sender, daemon=True, name=f"cstage{self.stage}-send-e{self.epoch}")
            t.start()
            self.threads.append(t)
        meta_w: List[Optional[object]] = [None] * self.nsets
        if self.prev is not None:
            for j in range(self.nsets):
                meta_w[j] = G.ctl_irecv(self.hmeta_in[j], self.prev, 2 * j)
        tick = 0
        while not self.stop.is_set():
            j = tick % self.nsets
            if self.prev is None:
                self._next_request(j)
            else:
                G.wait_host(meta_w[j])
                hm = self.hmeta_in[j]
                sizes = [int(v) for v in hm[4:].tolist()]
                works = []
                for k, (d, nb) in enumerate(zip(self.dec[j], sizes)):
                    if staged:
                        G.wait_host(G.irecv(h_in[j][k][:nb], self.prev, 2 * j + 1))
                        d.wire[:nb].copy_(h_in[j][k][:nb])
                    else:
                        works.append(G.irecv(d.wire[:nb], self.prev, 2 * j + 1))
                for w in works:
                    G.wait(w)
                for d, nb, buf in zip(self.dec[j], sizes, self.in_bufs[j]):
                    d.decode(nb, buf)
                self.cur_meta[j] = hm[:4].clone()             # before the next meta may land in hm
                self.meta_in[j].copy_(self.cur_meta[j])
                meta_w[j] = G.ctl_irecv(self.hmeta_in[j], self.prev, 2 * j)
            while not released[j].wait(0.05):                 # set j's previous send has left
                if self.stop.is_set():
                    raise Aborted("stopped")
            if self.gpu and self.enc is not None and self.enc[j]:
                torch.cuda.current_stream(self.dev).wait_event(self.enc[j][-1].done)
            slept = self.node.fault_point(self.stop)
            t_c = time.perf_counter() - slept     # an injected delay counts as compute
            self._compute(j)
            if self.gpu:
                ev = torch.cuda.Event()
                ev.record()
                self.events[j] = ev
            if self.next is not None:
                self.hmeta_out[j][:4].copy_(self.cur_meta[j])
                for e, tns in zip(self.enc[j], self.out_bufs[j]):
                    e.encode(tns, after=self.events[j])
                released[j].clear()
                sendq.put(j)
            else:
                if self.gpu:
                    G.wait_event(self.events[j])
                self._emit_result(j)
            self.processed += 1
            self.node.note_progress(self.epoch, busy_s=time.perf_counter() - t_c if not self.gpu else None)
            tick += 1
