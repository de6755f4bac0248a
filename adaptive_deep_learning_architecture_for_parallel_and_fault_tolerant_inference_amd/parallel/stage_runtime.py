"""Node data plane with collective links: RCCL p2p over xGMI between GPU
stages (``nccl``), or gloo between CPU stages.

The reference forwards every activation over TCP, compressed, through the
dispatcher hub (`src/node.py:163-179`, `src/dispatcher.py:121-151,204-220`).
Here only stage 0 (inputs) and the last stage (results) talk TCP to the
dispatcher; stage i -> i+1 is a point-to-point send of device-resident
tensors on the epoch's communicator (parallel/epoch_group.py):

    meta   int64[4] = (req_id, count, epoch, 1)      # rides with the data
    frontier tensors in slice-output order (bf16 on GPU, fp32 on CPU)

Double-buffered per stage (`nsets` buffer sets): the receive of micro-batch
t+1 and the send of t-1 run on the communicator's HIP stream while t
computes on the compute stream; host run-ahead is bounded by polling one
event per buffer set, and every wait is abortable so a reconfiguration can
tear the epoch down even while a peer is dead.
"""
from __future__ import annotations

import queue
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
        from ..runtime.stage import StageCompute
        self.node = node
        self.cfg = cfg
        self.epoch = int(cfg["epoch"])
        self.stage = int(cfg["stage"])
        self.stages = int(cfg["stages"])
        self.batch = int(cfg["batch"])
        self.codec = cfg.get("codec", "lz4")
        self.manifest = manifest
        self.nsets = int(cfg.get("nsets", 2))
        g = manifest.graph()
        self.compute = StageCompute(g, weights, self.batch, node.device, graph_capture=cfg.get("graph", True),
                                    num_sets=self.nsets)
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
        if not self.stop.is_set() and not isinstance(e, Aborted):
            self.error = f"{where}: {type(e).__name__}: {e}"
        self.abort()

    def abort(self) -> None:
        if self.stop.is_set():
            return
        self.stop.set()
        if self.group is not None:
            self.group.abort()
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

    # ------------------------------------------------------- TCP edges
    def _tcp_recv_loop(self) -> None:
        from ..transport.messages import recv_message
        try:
            while not self.stop.is_set():
                m = recv_message(self.upstream, self.node.state.chunk_size)
                if m is None:
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
        self.meta_in[j].copy_(torch.tensor([m.req_id, m.count, self.epoch, 1], dtype=torch.int64))
        return True

    def _compute(self, j: int) -> None:
        if self.gpu:
            self.compute.ex.forward(j)
        else:
            feed = dict(zip(self.compute.inputs, self.in_bufs[j]))
            y = self.compute.ex.run(feed, outputs=self.compute.outputs)
            for t, n in zip(self.out_bufs[j], self.compute.outputs):
                t.copy_(y[n])
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

    def _data_loop(self) -> None:
        cc = self.cfg["collective"]
        try:
            self.group = EpochGroup(cc["backend"], cc["store_host"], int(cc["store_port"]), self.epoch, self.stage,
                                    self.stages, self.dev if self.gpu else None, float(cc.get("timeout", 30)))
        except Exception as e:  # noqa: BLE001 - rendezvous failed (a member died): epoch is dead
            self._fail("rendezvous", e)
            return
        if self.stop.is_set():
            self.group.abort()
            return
        G = self.group
        recv_w: List[Optional[list]] = [None] * self.nsets
        send_w: List[Optional[list]] = [None] * self.nsets

        def post_recv(j):
            return [G.irecv(self.meta_in[j], self.prev, 2 * j)] + \
                   [G.irecv(t, self.prev, 2 * j + 1) for t in self.in_bufs[j]]

        def post_send(j):
            return [G.isend(self.meta_out[j], self.next, 2 * j)] + \
                   [G.isend(t, self.next, 2 * j + 1) for t in self.out_bufs[j]]

        tick = 0
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
                for w in send_w[j] or []:
                    G.wait(w)
                send_w[j] = None
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
                tick += 1
        except Exception as e:  # noqa: BLE001
            if not isinstance(e, Aborted):
                traceback.print_exc()
            self._fail("data", e)
