"""Worker node: one process per MI355X (public API of `src/node.py`).

Reference worker (`src/node.py:24-211`): a config server receives the Keras
JSON + index + weights and ACKs (`:65-98`), a data server reads activations
(`:137-161`), a client loop runs ``model.predict`` and forwards the result
(`:163-179`); the process registers nowhere although the dispatcher waits on
etcd for it.  Here:

* **membership**: a leased ``/workers/{id}`` record (host, ports, device,
  state, epoch) with a keepalive heartbeat; death => lease expiry => the
  dispatcher repartitions;
* **config server** (``config_port``, 6001): framed JSON command, then for
  ``configure`` the slice (manifest + ASCII index + weights, the reference
  order) and an ACK ``0x06`` (NAK ``0x15`` + reason frame on failure);
* **data plane** per *epoch*: ``StageRuntime`` receives micro-batches from its
  upstream (dispatcher for stage 0, previous stage otherwise), runs the slice
  (our HIP runtime on the GPU, the fp32 oracle on CPU) and forwards to its
  downstream (next stage, or the dispatcher's result port for the last
  stage).  Receive, compute and send run on three threads with bounded
  queues so transfers overlap compute.  A new ``configure`` aborts the old
  epoch's links (sockets closed => blocked peers unblock) and starts the new
  one — this is how survivors re-form a pipeline after a failure;
* **links**: TCP framed messages (any host, CPU or GPU; codec per link), or
  RCCL point-to-point over xGMI between GPU stages (parallel/stage_runtime.py).

CLI:  python -m <pkg>.node --dispatcher 127.0.0.1 --membership-port 2379 \
          --data-port 6000 --config-port 6001 --device cuda:0
"""
from __future__ import annotations

import argparse
import json
import os
import queue
import socket
import sys
import threading
import time
import traceback
import uuid
from typing import Dict, Optional, Tuple

import numpy as np

from .graph.manifest import ACK, NAK, SliceManifest, arrays_to_dict, recv_slice
from .node_state import NodeState, StateEnum, socket_recv, socket_send
from .transport.messages import Message, connect, listen, recv_message, send_message

DATA_PORT = 6000     # receive input data      (src/node.py:20)
CONFIG_PORT = 6001   # receive model config    (src/node.py:21)
RESULT_PORT = 6003   # send results            (src/node.py:22)
CTRL_CHUNK = 1 << 16


def get_local_ip() -> str:
    """UDP-connect trick with 127.0.0.1 fallback (`src/node.py:197-208`)."""
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    try:
        s.connect(("1.1.1.1", 1))
        ip = s.getsockname()[0]
    except OSError:
        ip = "127.0.0.1"
    finally:
        s.close()
    return ip


# exit status of a worker process that gave up after a stuck RCCL abort (EX_TEMPFAIL:
# a supervisor may start a fresh process)
EXIT_UNRECOVERABLE = 75


class _Pending:
    """A pipelined GPU micro-batch in the send queue: `msg`'s host tensors are
    ready once `ev` has completed; `links` are its input's link slots."""
    __slots__ = ("ev", "msg", "links", "t_submit")

    def __init__(self, ev, msg, links):
        self.ev, self.msg, self.links = ev, msg, links
        self.t_submit = time.perf_counter()


class StageRuntime:
    """One epoch's data plane on this node."""

    def __init__(self, node: "Node", cfg: Dict, manifest: SliceManifest, weights: Dict[str, np.ndarray]):
        from .runtime.stage import StageCompute
        self.node = node
        self.cfg = cfg
        self.epoch = int(cfg["epoch"])
        self.stage = int(cfg["stage"])
        self.codec = cfg.get("codec", "lz4")
        self.manifest = manifest
        g = manifest.graph()
        plot_dir = os.environ.get("ADAPT_PLOT_DIR")
        if plot_dir:                          # the reference's per-worker plot_model (src/node.py:49)
            from .utils.plot import plot_model, slice_plot_name
            plot_model(g, slice_plot_name(plot_dir, node.node_id, self.epoch))
        # "shm": the next stage shares this host's /dev/shm, so frontier tensors go
        # device -> page-locked link slot and only descriptors cross the socket
        # (transport/shm.py LinkPool); "dev": both stages are GPU workers on the host,
        # so the slots are device memory exported by IPC handle (DeviceLinkPool) and
        # the hop is a device-to-device copy; the TCP codec applies to neither
        self.link = cfg.get("link", "tcp")
        if self.link == "dev" and not str(node.device).startswith("cuda"):
            self.link = "shm"
        # GPU stages with a GPU codec compress frontier tensors on a side HIP stream
        # while the next micro-batch computes (two buffer sets ping-pong)
        self.gpu_codec = (self.codec in ("zvc", "lz4") and str(node.device).startswith("cuda")
                          and self.link == "tcp")
        self.compute = node.stage_compute(cfg, g, weights)
        self._linkpool = None
        if self.link == "dev":
            from .transport import shm
            self._linkpool = shm.DeviceLinkPool(node.device, prefix=f"adapt-link-{os.getpid()}-e{self.epoch}-"
                                                                    f"s{self.stage}-{uuid.uuid4().hex[:6]}")
        elif self.link == "shm":
            from .transport import shm
            self._linkpool = shm.LinkPool(prefix=f"adapt-link-{os.getpid()}-e{self.epoch}-s{self.stage}-"
                                                 f"{uuid.uuid4().hex[:6]}",
                                          register_device=bool(getattr(self.compute, "gpu", False)))
        self._attached_links: set = set()     # upstream link segments this epoch mapped
        if self.gpu_codec:
            self._init_gpu_codec()
        self.inq: "queue.Queue" = queue.Queue(maxsize=int(cfg.get("queue", 4)))
        self.outq: "queue.Queue" = queue.Queue(maxsize=int(cfg.get("queue", 4)))
        self.stop = threading.Event()
        self.upstream: Optional[socket.socket] = None
        self.downstream: Optional[socket.socket] = None
        self.processed = 0
        self._busy_s = 0.0                       # host compute time of the last synchronous micro-batch
        self._last_done = 0.0
        self.threads = []
        self.error: Optional[str] = None
        # held while a micro-batch runs on `compute`: abort() waits on it, so a
        # cached StageCompute is never driven by two epochs' threads at once
        self._busy = threading.Lock()

    def quiesced(self) -> bool:
        return True          # abort() waits for the running micro-batch (`_busy`)

    # downstream = next stage's data port, or the dispatcher result port
    def _connect_downstream(self) -> socket.socket:
        nxt = self.cfg.get("next")
        hello = json.dumps({"epoch": self.epoch, "from_stage": self.stage,
                            "replica": self.cfg.get("replica", 0)}).encode()
        host, port = (nxt["host"], nxt["port"]) if nxt else tuple(self.cfg["result_addr"])
        deadline = time.time() + float(self.cfg.get("connect_timeout", 10.0))
        while True:
            try:
                return connect(host, int(port), hello=hello)
            except OSError:
                if time.time() > deadline or self.stop.is_set():
                    raise
                time.sleep(0.05)

    def attach_upstream(self, sock: socket.socket) -> None:
        self.upstream = sock
        t = threading.Thread(target=self._recv_loop, daemon=True, name=f"stage{self.stage}-recv-e{self.epoch}")
        t.start()
        self.threads.append(t)

    def start(self) -> None:
        for fn, nm in ((self._compute_loop, "compute"), (self._send_loop, "send")):
            t = threading.Thread(target=fn, daemon=True, name=f"stage{self.stage}-{nm}-e{self.epoch}")
            t.start()
            self.threads.append(t)

    def _fail(self, where: str, e: BaseException) -> None:
        report = not self.stop.is_set()
        if report:
            self.error = f"{where}: {type(e).__name__}: {e}"
        self.abort()
        if report:
            # a broken hop (neighbour SIGKILLed) is published at once, so the
            # dispatcher re-plans without waiting for the dead worker's lease TTL;
            # a failure of this stage's own compute is a STAGE_ERROR (the
            # dispatcher quarantines the worker instead of re-placing onto it)
            self.node.report_failure(self, "LINK_ERROR" if where in ("recv", "send") else "STAGE_ERROR")

    def _recv_loop(self) -> None:
        try:
            while not self.stop.is_set():
                m = recv_message(self.upstream, self.node.state.chunk_size,
                                 keep_encoded=("zvc", "lz4") if self.gpu_codec else ())
                if m is not None and m.links:
                    self._attached_links.update(m.links)
                if m is None:
                    if not self.stop.is_set():
                        # clean EOF inside a live epoch: the upstream process died
                        # (the kernel closed its socket) or its epoch was torn down
                        raise ConnectionError("upstream closed the link")
                    break
                if m.epoch != self.epoch:
                    self._release_links(m.links)
                    continue                     # stale micro-batch from an older epoch
                while not self.stop.is_set():
                    try:
                        self.inq.put(m, timeout=0.1)
                        break
                    except queue.Full:
                        continue
        except Exception as e:  # noqa: BLE001 - any transport error ends the epoch
            self._fail("recv", e)

    @staticmethod
    def _release_links(names) -> None:
        if names:
            from .transport import shm
            for n in names:
                shm.release(n)

    def _link_slot(self, shape, dtype):
        """`StageCompute.submit` out_slots: a page-locked link slot and its descriptor."""
        import numpy as np
        import torch
        from .transport.shm import ShmRef
        bf16 = dtype == torch.bfloat16
        np_dt = np.dtype(np.uint16) if bf16 else np.dtype(str(dtype).replace("torch.", ""))
        n = 1
        for v in shape:
            n *= int(v)
        from .transport.shm import ShmFull
        try:
            if self.link == "dev":
                from .transport.shm import DevRef
                ds = self._linkpool.acquire_dev(n * np_dt.itemsize, self.stop)
                return ds, DevRef(ds, np_dt, shape, bf16=bf16)
            slot = self._linkpool.acquire(n * np_dt.itemsize, self.stop)
        except ShmFull:
            # /dev/shm is full: this tensor travels inline on the TCP hop (page-locked
            # staging buffer, kept alive by the numpy view until the send)
            host = torch.empty(tuple(shape), dtype=dtype, pin_memory=True)
            arr = host.view(torch.int16).numpy().view(np.uint16) if bf16 else host.numpy()
            return host, arr
        host = torch.from_numpy(slot.view(np_dt, shape))
        if bf16:
            host = host.view(torch.bfloat16)
        return host, ShmRef(slot, np_dt, shape, bf16=bf16)

    # ------------------------------------------------ GPU side-stream codec
    def _init_gpu_codec(self) -> None:
        from .codec.gpu_lz4 import GpuLZ4
        from .codec.gpu_zvc import GpuZVC
        ex = self.compute.ex
        self.codecs = []
        for j in range(2):
            per = []
            for o in self.compute.outputs:
                t = ex.output_buf(o, j)
                if self.codec == "zvc" and t.element_size() in (2, 4):
                    per.append(GpuZVC(t.numel(), t.element_size(), self.compute.device))
                else:
                    per.append(GpuLZ4(t.numel() * t.element_size(), self.compute.device))
            self.codecs.append(per)
        # set j (its output buffers and its codecs' device streams) is reusable only
        # after the send thread has copied set j's compressed bytes to the host
        self._set_free = [threading.Event(), threading.Event()]
        for e in self._set_free:
            e.set()
        self._tick = 0
        self.decoders: Dict[Tuple[str, str], object] = {}   # (input, codec) -> device decoder

    def _gpu_decode(self, name: str, buf, dst) -> bool:
        """Decode an encoded input container straight into its device buffer;
        False when the container does not match the buffer (host fallback)."""
        from . import codec as C
        from .codec.gpu_lz4 import GpuLZ4
        from .codec.gpu_zvc import GpuZVC
        cname, _dt, shape, payload = C.payload_of(buf)
        n = 1
        for v in shape:
            n *= int(v)
        if n != dst.numel():
            return False
        key = (name, cname)
        dec = self.decoders.get(key)
        if dec is None:
            if cname == "zvc":
                dec = GpuZVC(dst.numel(), dst.element_size(), self.compute.device)
            else:
                dec = GpuLZ4(dst.numel() * dst.element_size(), self.compute.device)
            self.decoders[key] = dec
        if cname == "zvc" and dst.element_size() != int(self._zvc_esz(payload)):
            return False
        dec.decompress(payload, dst)
        return True

    @staticmethod
    def _zvc_esz(payload) -> int:
        from .native import runtime
        return runtime().zvc_info(payload)[1]

    def _compute_gpu(self, m: Message) -> Message:
        import torch
        from .runtime.stage import to_torch
        j = self._tick % 2
        self._tick += 1
        ex = self.compute.ex
        while not self._set_free[j].wait(0.1):    # set j's previous message has left the GPU
            if self.stop.is_set():
                raise RuntimeError("stage stopped")
        self._set_free[j].clear()
        from .transport.shm import DevArray
        for name, a, b in zip(self.compute.inputs, m.tensors, m.bf16):
            dst = ex.input_buf(name, j)
            if isinstance(a, DevArray):
                # the upstream hop was a device link (its slot holds the raw frontier, only
                # zvc/lz4 frames stay encoded): device-to-device into the input buffer.  The
                # caller releases the slot as soon as this returns, so the copy is waited for
                from .ops._lib import kernels, stream_handle
                want = np.dtype(np.uint16) if dst.dtype == torch.bfloat16 else np.dtype(np.float32)
                if (a.dtype != want or tuple(a.shape[1:]) != tuple(dst.shape[1:]) or a.shape[0] > dst.shape[0]):
                    raise ValueError(f"device link tensor {a.shape} {a.dtype} does not match input {name} "
                                     f"{tuple(dst.shape)} {dst.dtype}")
                cur = torch.cuda.current_stream(dst.device)
                kernels().memcpy_async(int(dst.data_ptr()), a.ptr, a.nbytes, stream_handle(cur))
                if a.shape[0] < dst.shape[0]:
                    dst[a.shape[0]:].zero_()
                cur.synchronize()
                continue
            if isinstance(a, (bytes, bytearray, memoryview)):
                if self._gpu_decode(name, a, dst):
                    continue
                from . import codec as C
                a = C.decode(a, copy=False)
            t = to_torch(a, b, dst.device)
            if t.dtype != dst.dtype:
                t = t.to(dst.dtype)
            if t.shape[-1] != dst.shape[-1]:
                t = torch.nn.functional.pad(t, (0, dst.shape[-1] - t.shape[-1]))
            if t.shape[0] < dst.shape[0]:
                dst.zero_()
            dst[: t.shape[0]].copy_(t)
        outs = ex.forward(j)
        ev = torch.cuda.Event()
        ev.record()
        dones = []
        for o, codec in zip(self.compute.outputs, self.codecs[j]):
            dones.append(codec.compress(outs[o], after=ev))
        shapes = [tuple(outs[o].shape) for o in self.compute.outputs]
        dtypes = [outs[o].dtype for o in self.compute.outputs]
        return Message(self.stage + 2, m.req_id, m.epoch, m.count, [("gpu", j, k) for k in range(len(shapes))],
                       [d == torch.bfloat16 for d in dtypes]), shapes, dtypes

    def _finish_gpu_message(self, item) -> Message:
        import numpy as np
        import torch
        from . import codec as C
        m, shapes, dtypes = item
        bufs = []
        for (_, j, k), shp, dt in zip(m.tensors, shapes, dtypes):
            c = self.codecs[j][k]
            # a view of the codec's pinned host buffer: valid until its next
            # use, which comes after this message has been sent (same thread)
            payload = c.stream_view() if hasattr(c, "stream_view") else c.frame_view()
            name = "zvc" if hasattr(c, "stream_view") else "lz4"
            np_dt = np.uint16 if dt == torch.bfloat16 else np.float32
            # the receiver only needs the first `count` images: a partial batch is
            # still sent whole (padding rows are zeros, cheap under either codec)
            bufs.append((C.wrap(b"", name, np_dt, shp, bf16=(dt == torch.bfloat16)), payload))
        self._set_free[m.tensors[0][1]].set()     # all of set j's bytes are on the host now
        return Message(m.partition, m.req_id, m.epoch, m.count, bufs, m.bf16)

    def _compute_loop(self) -> None:
        try:
            while not self.stop.is_set():
                try:
                    m = self.inq.get(timeout=0.1)
                except queue.Empty:
                    continue
                self.node.state.state = StateEnum.BUSY
                slept = self.node.fault_point(self.stop)
                t_c = time.perf_counter() - slept     # an injected delay counts as compute
                with self._busy:
                    if self.stop.is_set():
                        break
                    if self.gpu_codec:
                        out = self._compute_gpu(m)
                        self._release_links(m.links)     # its input copies were synchronous
                    elif self.compute.gpu:
                        # pipelined: H2D, ingest, graph replay and D2H are only enqueued here;
                        # the send thread waits for the event (micro-batch t computes while
                        # t+1 is received and t-1 is sent) and then frees the input link slots
                        ev, res = self.compute.submit(m.tensors, m.bf16, m.count,
                                                      out_slots=self._link_slot if self._linkpool else None)
                        out = _Pending(ev, Message(self.stage + 2, m.req_id, m.epoch, m.count, [r[0] for r in res],
                                                   [r[1] for r in res]), m.links)
                    else:
                        outs, flags = self.compute.run_host(m.tensors, m.bf16, m.count)
                        self._release_links(m.links)
                        if self._linkpool is not None and self.link == "shm":
                            outs = [self._linkpool.put(o, self.stop, bf16=f) for o, f in zip(outs, flags)]
                        out = Message(self.stage + 2, m.req_id, m.epoch, m.count, outs, flags)
                        self._busy_s = time.perf_counter() - t_c
                self.processed += 1
                while not self.stop.is_set():
                    try:
                        self.outq.put(out, timeout=0.1)
                        break
                    except queue.Full:
                        continue
        except Exception as e:  # noqa: BLE001
            traceback.print_exc()
            self._fail("compute", e)

    def _send_loop(self) -> None:
        try:
            self.downstream = self._connect_downstream()
            while not self.stop.is_set():
                try:
                    m = self.outq.get(timeout=0.1)
                except queue.Empty:
                    continue
                busy = None
                if isinstance(m, _Pending):                # pipelined GPU micro-batch: outputs on the host at `ev`
                    # a blocking wait with the GIL released: a 10 kHz query/sleep loop here took
                    # GIL time from the compute and receive threads of this stage
                    m.ev.synchronize()
                    t_done = time.perf_counter()
                    # device busy time of this micro-batch: from its submission (or the previous
                    # completion, if it queued behind that one) to its completion
                    busy = t_done - max(m.t_submit, self._last_done)
                    self._last_done = t_done
                    if self.stop.is_set():
                        return
                    self._release_links(m.links)           # the input copies out of them are done too
                    m = m.msg
                elif isinstance(m, tuple):                 # GPU-encoded frontier (side stream)
                    m = self._finish_gpu_message(m)
                send_message(self.downstream, m, self.codec, self.node.state.chunk_size)
                self.node.note_progress(self.epoch, busy_s=busy if busy is not None else self._busy_s)
        except Exception as e:  # noqa: BLE001
            self._fail("send", e)

    def abort(self) -> None:
        self.stop.set()
        for s in (self.upstream, self.downstream):
            if s is not None:
                try:
                    s.shutdown(socket.SHUT_RDWR)
                except OSError:
                    pass
                try:
                    s.close()
                except OSError:
                    pass
        # the micro-batch in flight (if any) has left `compute`; every loop raises
        # out of its `with self._busy` block before it calls _fail -> abort
        with self._busy:
            pass
        if self._linkpool is not None or self._attached_links:
            # no copy may still be running into or out of a slot that is unmapped below
            if getattr(self.compute, "gpu", False):
                import torch
                torch.cuda.synchronize(self.compute.device)
            if self._linkpool is not None:
                from .transport import shm
                if isinstance(self._linkpool, shm.DeviceLinkPool):
                    # IPC-exported device slots: the next stage may still hold them
                    # open (it tears its epoch down on its own schedule); freed one
                    # epoch later
                    self.node.retire_link_pool(self._linkpool)
                else:
                    self._linkpool.close()
            from .transport import shm
            shm.detach(list(self._attached_links))
            self._attached_links.clear()


class Node:
    def __init__(self, dispatcher_ip: str = "127.0.0.1", membership_port: int = 2379, data_port: int = DATA_PORT,
                 config_port: int = CONFIG_PORT, device: Optional[str] = None, node_id: Optional[str] = None,
                 chunk_size: int = 512 * 1000, host: str = "0.0.0.0", advertise_host: Optional[str] = None,
                 heartbeat_ttl: float = 1.0, register: bool = True, exit_on_unrecoverable: bool = False) -> None:
        self.weights_ready_event = threading.Event()        # reference attribute (src/node.py:27)
        # process mode (main()): a stuck RCCL abort ends the process with EXIT_UNRECOVERABLE;
        # library mode only publishes UNRECOVERABLE and stops the node
        self.exit_on_unrecoverable = exit_on_unrecoverable
        self.unrecoverable: Optional[str] = None
        if device is None:
            import torch
            device = "cuda:0" if torch.cuda.is_available() else "cpu"
        self.device = device
        if str(device).startswith("cuda"):
            from .transport import shm
            shm.REGISTER_DEVICE = True       # same-host ingest slots are page-locked for DMA
        self.host = host
        self.advertise_host = advertise_host or ("127.0.0.1" if dispatcher_ip in ("127.0.0.1", "localhost")
                                                 else get_local_ip())
        self.data_sock = listen(host, data_port)
        self.config_sock = listen(host, config_port)
        self.data_port = self.data_sock.getsockname()[1]
        self.config_port = self.config_sock.getsockname()[1]
        self.node_id = node_id or f"{self.advertise_host}:{self.config_port}"
        self.state = NodeState(chunk_size, dispatcher_ip, membership_port, node_id=self.node_id)
        self.dispatcher_ip = dispatcher_ip
        self.membership_port = membership_port
        self.heartbeat_ttl = heartbeat_ttl
        self.register = register
        self.registration = None
        self.runtime: Optional[StageRuntime] = None
        self._rt_lock = threading.Lock()
        self._pending_upstream: Dict[int, list] = {}
        self._slice_cache: Dict[str, Tuple[SliceManifest, Dict[str, np.ndarray]]] = {}
        # resident whole models (graph, weights) by model key: a re-plan to new cuts
        # is local slicing, with no weight push
        self._models: Dict[str, Tuple[object, Dict[str, np.ndarray]]] = {}
        # built stage computes (packed weights + buffers + captured hipGraphs) by
        # slice key and runtime shape; `prepare` fills it ahead of a failure
        self._computes: Dict[tuple, object] = {}
        self._computes_lock = threading.Lock()
        self._building: Dict[tuple, threading.Event] = {}
        self._pub_lock = threading.Lock()
        self._sessions = 0
        self._stop = threading.Event()
        self.threads = []
        # completed micro-batches (all epochs), carried by every heartbeat so the
        # dispatcher can tell a wedged-but-alive stage from a slow one
        self._progress = 0                               # micro-batches completed in `_prog_epoch`
        self._prog_epoch = 0
        self._stage_s = 0.0                              # EWMA of this worker's busy time per micro-batch
        self._hb_handles: set = set()
        self._hb_lock = threading.Lock()
        self._hang = threading.Event()                   # fault injection: "hang"
        self._delay_s = 0.0                              # fault injection: "delay:<s>"
        self._retired_pools: list = []                   # device link pools of the last torn-down epoch

    # ---------------------------------------------------------- lifecycle
    def record(self) -> Dict:
        from .transport import shm
        rec = {"id": self.node_id, "host": self.advertise_host, "data_port": self.data_port,
               "config_port": self.config_port, "device": self.device, "pid": os.getpid(),
               "state": self.state.state.name, "epoch": self.state.epoch, "shm_domain": shm.domain()}
        try:
            import torch
            if self.device.startswith("cuda"):
                rec["gpu"] = torch.cuda.get_device_name(torch.device(self.device))
        except Exception:  # noqa: BLE001 - telemetry is best effort
            pass
        return rec

    def run(self, block: bool = True) -> None:
        for fn, nm in ((self._config_server, "config"), (self._data_server, "data")):
            t = threading.Thread(target=fn, daemon=True, name=f"node-{nm}")
            t.start()
            self.threads.append(t)
        if self.register:
            from .membership.client import MembershipClient, Registration
            deadline = time.time() + 30
            while True:
                try:
                    client = MembershipClient(self.dispatcher_ip, self.membership_port)
                    self.registration = Registration(client, self.node_id, self.record(), ttl=self.heartbeat_ttl)
                    break
                except (OSError, ConnectionError):
                    if time.time() > deadline:
                        raise
                    time.sleep(0.2)
            t = threading.Thread(target=self._telemetry_loop, daemon=True, name="node-telemetry")
            t.start()
            self.threads.append(t)
        if block:
            try:
                while not self._stop.wait(1.0):
                    pass
            except KeyboardInterrupt:
                pass
            finally:
                self.stop()

    def _telemetry_loop(self, period: float = 2.0) -> None:
        """Publish load + amdsmi readings into the membership record (the
        reference imports psutil / pynvml for this but never uses them,
        `src/node.py:10`, `src/node_state.py:6`)."""
        from .utils.telemetry import gpu_telemetry
        idx = int(self.device.split(":")[1]) if self.device.startswith("cuda:") else None
        while not self._stop.wait(period):
            rt = self.runtime
            rec = {"processed": rt.processed if rt else 0, "error": rt.error if rt else None}
            if idx is not None:
                rec.update(gpu_telemetry(idx))
            try:
                import psutil
                rec["cpu_percent"] = psutil.cpu_percent(interval=None)
            except Exception:  # noqa: BLE001
                pass
            self._publish(**rec)

    # ------------------------------------------------- progress / faults
    def note_progress(self, epoch: int, n: int = 1, busy_s: Optional[float] = None) -> None:
        """A micro-batch of `epoch` finished (`busy_s`: the time this stage spent
        on it): publish the epoch's counter and the per-micro-batch time on the
        heartbeats.  The dispatcher compares the counters of a replica's stages
        with the results it received to find the stage a request is stuck in."""
        with self._hb_lock:
            if epoch != self._prog_epoch:
                if epoch < self._prog_epoch:
                    return                                # a straggler of a retired epoch
                self._prog_epoch, self._progress = epoch, 0
            self._progress += n
            if busy_s is not None and busy_s > 0:
                self._stage_s = busy_s if self._stage_s == 0 else 0.8 * self._stage_s + 0.2 * busy_s
            if self._hb_handles:
                from .native import runtime
                rt = runtime()
                for h in self._hb_handles:
                    rt.hb_sender_progress(h, self._progress, int(self._stage_s * 1e9), self._prog_epoch)

    def inject_fault(self, kind: str) -> None:
        """Fault injection (tests, tools/fault_bench.py): ``"hang"`` wedges this
        worker's compute loops at their next micro-batch while every other
        thread (heartbeat, sessions, config server) keeps running - the
        failure a heartbeat alone cannot see; ``"delay:<s>"`` makes every
        micro-batch take <s> seconds longer (a slow but healthy stage: its
        progress counter and reported stage time include the delay);
        ``"clear"`` releases both."""
        if kind == "hang":
            self._hang.set()
        elif kind.startswith("delay:"):
            self._delay_s = max(0.0, float(kind.split(":", 1)[1]))
        elif kind == "clear":
            self._hang.clear()
            self._delay_s = 0.0
        else:
            raise ValueError(f"unknown fault {kind!r}")

    def fault_point(self, stop: threading.Event) -> float:
        """Called by the compute loops before each micro-batch; returns the
        injected delay it slept (the caller counts it as compute time)."""
        while self._hang.is_set() and not stop.is_set() and not self._stop.is_set():
            time.sleep(0.005)
        d = self._delay_s
        if d > 0:
            stop.wait(d)
        return d

    def retire_link_pool(self, pool) -> None:
        """Keep a torn-down epoch's device link pool alive until the next one is
        retired (or the node stops): importers of its IPC handles finish long
        before that, so freeing it is never a use-after-free on their side."""
        with self._hb_lock:
            old, self._retired_pools = self._retired_pools, [pool]
        for p in old:
            p.close(handoff_timeout_s=0.0)

    def stop(self) -> None:
        self._stop.set()
        if self.registration is not None:
            self.registration.close(revoke=True)
        with self._rt_lock:
            if self.runtime is not None:
                self.runtime.abort()
        with self._hb_lock:
            old, self._retired_pools = self._retired_pools, []
        for p in old:
            p.close(handoff_timeout_s=0.5)
        for s in (self.data_sock, self.config_sock):
            try:
                s.close()
            except OSError:
                pass
        # background builds (prepare) stop between slices: let the one in progress
        # finish so no thread is inside native code when the interpreter exits
        for t in list(self.threads):
            if t.name == "node-prepare" and t is not threading.current_thread():
                t.join(timeout=60)
        # ... and any StageCompute a config handler or stage runtime is building
        # (capturing a hipGraph) right now: no capture may outlive the node, since
        # while one runs PyTorch marks the default CUDA generator as capturing and
        # a CUDA RNG call on any other thread of the process fails
        deadline = time.monotonic() + 60
        while time.monotonic() < deadline:
            with self._computes_lock:
                pending = list(self._building.values())
            if not pending:
                break
            pending[0].wait(max(0.0, deadline - time.monotonic()))

    def _publish(self, **kw) -> None:
        if self.registration is not None:
            try:
                self.registration.put(**kw)
            except (OSError, ConnectionError, RuntimeError):
                pass

    def report_failure(self, rt, state: str) -> None:
        """Publish a failed epoch (LINK_ERROR / STAGE_ERROR) unless a newer epoch
        has replaced it: the check and the put happen under the lock that also
        orders the BUSY put of `_start_epoch`, so a late report can never
        overwrite the record of the epoch that follows."""
        with self._pub_lock:
            if self.runtime is not rt or self.state.epoch != rt.epoch:
                return
            self._publish(state=state, epoch=rt.epoch, error=rt.error)

    def give_up(self, rt, reason: str) -> None:
        """The epoch's communicator could not be aborted within its deadline
        (`RcclComm.abort_stuck`): this process can no longer vouch for its RCCL
        state, so it publishes UNRECOVERABLE (the dispatcher treats that as a
        dead worker and re-plans without it), stops, and in process mode exits
        with EXIT_UNRECOVERABLE so a supervisor can start a *fresh* process in
        its place (never an exec: the GPU is initialised here).  The reference's
        watchdog can only notice a worker that stops answering
        (`/root/reference/src/dispatcher.py:186-194,302-304`)."""
        if self.unrecoverable is not None:
            return
        self.unrecoverable = reason
        print(f"node {self.node_id}: UNRECOVERABLE ({reason}); exiting {EXIT_UNRECOVERABLE}", file=sys.stderr,
              flush=True)
        self._publish(state="UNRECOVERABLE", epoch=getattr(rt, "epoch", self.state.epoch), error=reason)
        if self.exit_on_unrecoverable:
            sys.stdout.flush()
            sys.stderr.flush()
            os._exit(EXIT_UNRECOVERABLE)
        threading.Thread(target=self.stop, daemon=True, name="node-give-up").start()

    # -------------------------------------------------- stage computes
    @staticmethod
    def compute_shape(cfg: Dict, device: str) -> Tuple[int, int, bool, int]:
        """(num_sets, host_ring, graph, streams) the epoch runtime for `cfg` builds
        its StageCompute with: one definition for configure and prepare."""
        graph = bool(cfg.get("graph", True))
        if cfg.get("transport", "tcp") == "tcp":
            # GPU stages double-buffer (pipelined submit / GPU codec); the host ring of
            # output buffers outlives the bounded queues between the stage's threads.
            # streams: the two sets replay on two streams unless the dispatcher saw
            # other workers on this GPU (they already keep it busy)
            gpu = str(device).startswith("cuda")
            return ((2 if gpu else 1), int(cfg.get("queue", 4)) + 4, graph,
                    (int(cfg.get("stage_streams", 2)) if gpu else 1))
        return int(cfg.get("nsets", 2)), 8, graph, 1

    def _compute_key(self, cfg: Dict) -> Optional[tuple]:
        key = cfg.get("cache_key")
        if not key:
            return None
        return (key, int(cfg["batch"]), cfg.get("precision", "fp32"), cfg.get("preprocess", "none")) + \
            self.compute_shape(cfg, self.device)

    def stage_compute(self, cfg: Dict, g, weights: Dict[str, np.ndarray], capture_mode: str = "global"):
        """The StageCompute of a slice: reused from the cache (built by an earlier
        epoch or by `prepare`), else built now and cached."""
        from .runtime.stage import StageCompute
        key = self._compute_key(cfg)
        num_sets, host_ring, graph, streams = self.compute_shape(cfg, self.device)
        while key is not None:
            with self._computes_lock:
                c = self._computes.get(key)
                if c is not None:
                    return c
                ev = self._building.get(key)
                if ev is None:
                    ev = self._building[key] = threading.Event()
                    break
            ev.wait(60)                             # a prepare is building this one right now
        try:
            c = StageCompute(g, weights, int(cfg["batch"]), self.device, graph_capture=graph, num_sets=num_sets,
                             host_ring=host_ring, capture_mode=capture_mode, streams=streams,
                             precision=cfg.get("precision", "fp32"), preprocess=cfg.get("preprocess", "none"))
        finally:
            if key is not None:
                with self._computes_lock:
                    self._building.pop(key).set()
        if key is not None:
            with self._computes_lock:
                self._computes[key] = c
        return c

    def _evict_compute(self, cfg: Dict) -> None:
        key = self._compute_key(cfg)
        if key is not None:
            with self._computes_lock:
                self._computes.pop(key, None)

    def _local_slice(self, cfg: Dict):
        """Slice a resident model locally: (manifest, weights) for cfg's stage."""
        from .graph.slicer import partition, subgraph
        g, w = self._models[cfg["model_key"]]
        sl = partition(g, list(cfg["part_at"]))[int(cfg["stage"])]
        m = SliceManifest(g.name, sl.index + 1, sl.name, subgraph(g, sl).to_json(),
                          [{"name": t} for t in sl.inputs], [{"name": t} for t in sl.outputs], [], sl.start, sl.end)
        return m, w

    def _prepare(self, cfgs) -> None:
        """Build (and capture) the StageComputes of likely next epochs in the
        background, so that a re-plan after a failure is a pointer swap.  Capture
        runs in thread-local mode: the serving threads keep launching meanwhile."""
        for cfg in cfgs:
            if self._stop.is_set():
                return
            key = self._compute_key(cfg)
            if key is None or key in self._computes:
                continue
            try:
                if cfg.get("model_key") in self._models:
                    m, w = self._local_slice(cfg)
                elif cfg["cache_key"] in self._slice_cache:
                    m, w = self._slice_cache[cfg["cache_key"]]
                else:
                    continue
                self.stage_compute(cfg, m.graph(), w, capture_mode="thread_local")
            except Exception:  # noqa: BLE001 - a prepare is an optimisation only
                traceback.print_exc()

    # ------------------------------------------- reference-named helpers
    @staticmethod
    def _comp(arr: np.ndarray) -> bytes:
        """`src/node.py:122-123`: zfp (reversible) then LZ4 frame, native codecs."""
        from . import codec
        return codec.comp(arr)

    @staticmethod
    def _decomp(byts) -> np.ndarray:
        """`src/node.py:124-125`."""
        from . import codec
        return codec.decomp(byts)

    def _recv_weights(self, sock: socket.socket, chunk_size: Optional[int] = None) -> list:
        """`src/node.py:101-119`: u64be array count, then one framed compressed
        array each (written by `DEFER._send_weights`); Keras `get_weights()` order."""
        head = b""
        while len(head) < 8:
            part = sock.recv(8 - len(head))
            if not part:
                raise ConnectionError("connection closed before the weight count")
            head += part
        count = int.from_bytes(head, "big")
        out = []
        for _ in range(count):
            frame = socket_recv(sock, chunk_size or self.state.chunk_size)
            if not frame:
                raise ConnectionError("connection closed inside the weight list")
            out.append(self._decomp(frame))
        return out

    # ------------------------------------------------------- config plane
    def _config_server(self) -> None:
        while not self._stop.is_set():
            try:
                conn, _ = self.config_sock.accept()
            except OSError:
                break
            threading.Thread(target=self._handle_config, args=(conn,), daemon=True, name="node-config").start()

    def _handle_config(self, conn: socket.socket) -> None:
        try:
            raw = socket_recv(conn, CTRL_CHUNK)
            if not raw:
                return
            cmd = json.loads(raw)
            op = cmd.get("cmd")
            if op == "configure" and cmd.get("model_key") in self._models:
                m, w = self._local_slice(cmd)          # resident model: local slicing, no push
                self.weights_ready_event.set()
                self._start_epoch(cmd, m, w)
                conn.sendall(ACK)
            elif op == "configure" and cmd.get("model_key"):
                conn.sendall(NAK)
                socket_send(b"model not resident", conn, CTRL_CHUNK)
            elif op == "load_model":
                m, arrays = recv_slice(conn, self.state.chunk_size)
                self._models[cmd["key"]] = (m.graph(), arrays_to_dict(m, arrays))
                conn.sendall(ACK)
            elif op == "prepare":
                conn.sendall(ACK)
                t = threading.Thread(target=self._prepare, args=(cmd.get("configs", []),), daemon=True,
                                     name="node-prepare")
                t.start()
                self.threads.append(t)
            elif op == "inject":
                try:
                    self.inject_fault(str(cmd.get("fault")))
                    conn.sendall(ACK)
                except ValueError as e:
                    conn.sendall(NAK)
                    socket_send(str(e).encode(), conn, CTRL_CHUNK)
            elif op == "session":
                # liveness channel: the dispatcher holds this connection open and
                # sees EOF the moment this process dies (no lease TTL to wait for)
                conn.sendall(ACK)
                self._sessions += 1
                hb = None
                if cmd.get("hb_port"):
                    # GIL-free UDP heartbeat to the dispatcher (csrc/runtime/heartbeat.cpp): it
                    # stops the instant this process is killed, long before the socket closes
                    from .native import runtime
                    try:
                        hb = runtime().hb_sender_start(conn.getpeername()[0], int(cmd["hb_port"]), self.node_id,
                                                       int(cmd.get("hb_period_us", 5000)))
                        with self._hb_lock:
                            runtime().hb_sender_progress(hb, self._progress, int(self._stage_s * 1e9),
                                                         self._prog_epoch)
                            self._hb_handles.add(hb)
                    except RuntimeError:
                        hb = None
                conn.settimeout(0.5)
                try:
                    while not self._stop.is_set():
                        try:
                            if not conn.recv(64):
                                break
                        except socket.timeout:
                            continue
                        except OSError:
                            break
                finally:
                    if hb is not None:
                        from .native import runtime
                        with self._hb_lock:
                            self._hb_handles.discard(hb)
                        runtime().hb_sender_stop(hb)
            elif op == "configure":
                if cmd.get("cached"):
                    key = cmd["cache_key"]
                    if key not in self._slice_cache:
                        conn.sendall(NAK)
                        socket_send(b"slice not cached", conn, CTRL_CHUNK)
                        return
                    m, w = self._slice_cache[key]
                else:
                    m, arrays = recv_slice(conn, self.state.chunk_size)
                    w = arrays_to_dict(m, arrays)
                    if cmd.get("cache_key"):
                        self._slice_cache[cmd["cache_key"]] = (m, w)
                self.state.weights = w
                self.weights_ready_event.set()
                self._start_epoch(cmd, m, w)
                conn.sendall(ACK)
            elif op == "stop_epoch":
                with self._rt_lock:
                    if self.runtime is not None:
                        self.runtime.abort()
                        self.runtime = None
                self.state.state = StateEnum.IDLE
                self._publish(state="IDLE")
                conn.sendall(ACK)
            elif op == "status":
                rt = self.runtime
                st = {"epoch": self.state.epoch, "state": self.state.state.name,
                      "processed": rt.processed if rt else 0, "error": rt.error if rt else None}
                try:
                    conn.sendall(ACK)
                    socket_send(json.dumps(st).encode(), conn, CTRL_CHUNK)
                except (OSError, RuntimeError):
                    return                  # the prober gave up (bounded liveness probe, shutdown): nothing to report
            elif op == "shutdown":
                conn.sendall(ACK)
                threading.Thread(target=self.stop, daemon=True).start()
            else:
                conn.sendall(NAK)
                socket_send(f"unknown cmd {op}".encode(), conn, CTRL_CHUNK)
        except Exception as e:  # noqa: BLE001 - report failure to the dispatcher
            traceback.print_exc()
            self.state.state = StateEnum.PARSE_ERROR
            try:
                conn.sendall(NAK)
                socket_send(f"{type(e).__name__}: {e}".encode(), conn, CTRL_CHUNK)
            except OSError:
                pass
        finally:
            try:
                conn.close()
            except OSError:
                pass

    def _start_epoch(self, cfg: Dict, m: SliceManifest, w: Dict[str, np.ndarray]) -> None:
        t0 = time.perf_counter()
        with self._rt_lock:
            old = self.runtime
            if old is not None:
                old.abort()
                if not old.quiesced():            # a thread still inside the old compute: do not reuse it
                    self._evict_compute(old.cfg)
            t1 = time.perf_counter()
            if cfg.get("transport", "tcp") == "tcp":
                rt = StageRuntime(self, cfg, m, w)
            else:                                   # RCCL (xGMI) / gloo stage-to-stage links
                from .parallel.stage_runtime import CollectiveStageRuntime
                rt = CollectiveStageRuntime(self, cfg, m, w)
            # epoch formation cost on this worker (old epoch's abort, new runtime incl. its compute: a cache
            # hit when `prepare` built the slice); the collective runtime adds its link rendezvous on the data
            # thread (stage_runtime.py setup_ms)
            rt.form_ms = {"abort_old": round((t1 - t0) * 1e3, 1), "build": round((time.perf_counter() - t1) * 1e3, 1)}
            self.runtime = rt
            self.state.epoch = rt.epoch
            self.state.partition_index = m.part_index
            self.state.model = rt.compute
            self.state.next_node = (cfg.get("next") or {}).get("host", "dispatcher")
            rt.start()
            for s in self._pending_upstream.pop(rt.epoch, []):
                rt.attach_upstream(s)
            for e in [e for e in self._pending_upstream if e < rt.epoch]:
                for s in self._pending_upstream.pop(e):
                    s.close()
        self.state.state = StateEnum.BUSY
        with self._pub_lock:
            self._publish(state="BUSY", epoch=rt.epoch, partition=m.part_index, error=None)

    # --------------------------------------------------------- data plane
    def _data_server(self) -> None:
        while not self._stop.is_set():
            try:
                conn, _ = self.data_sock.accept()
            except OSError:
                break
            conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            try:
                hello = json.loads(socket_recv(conn, CTRL_CHUNK) or b"{}")
            except (RuntimeError, ValueError, OSError):
                conn.close()
                continue
            ep = int(hello.get("epoch", -1))
            with self._rt_lock:
                rt = self.runtime
                if rt is not None and rt.epoch == ep:
                    rt.attach_upstream(conn)
                elif rt is None or ep > rt.epoch:
                    self._pending_upstream.setdefault(ep, []).append(conn)   # config not here yet
                else:
                    conn.close()


def _follow_parent(ppid: int) -> None:
    """Die with the launcher: PR_SET_PDEATHSIG (SIGTERM when the parent exits), a check that it has
    not already gone, and a watcher thread for launchers that are not the direct parent."""
    import ctypes
    import signal as _signal
    try:
        ctypes.CDLL(None, use_errno=True).prctl(1, int(_signal.SIGTERM), 0, 0, 0)   # PR_SET_PDEATHSIG = 1
    except (OSError, AttributeError):
        pass

    def gone() -> bool:
        try:
            os.kill(ppid, 0)
            return False
        except ProcessLookupError:
            return True
        except PermissionError:
            return False

    if gone():
        os._exit(0)

    def watch():
        while not gone():
            time.sleep(0.5)
        os._exit(0)
    threading.Thread(target=watch, daemon=True, name="parent-watch").start()


def main(argv=None):
    # epoch communicators are aborted by this runtime (re-plan, stall watch): the
    # NCCL watchdog must not kill the worker over receives an idle pipeline keeps posted
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "0")
    # before the first HIP call: compute, capture, link, RCCL, codec and copy streams
    # must not share the default 4 hardware queues (utils/hwqueues.py)
    from .utils.hwqueues import ensure_hw_queues
    ensure_hw_queues()
    ap = argparse.ArgumentParser(description="ADAPT worker node (one per GPU)")
    ap.add_argument("--dispatcher", default="127.0.0.1", help="dispatcher / membership host")
    ap.add_argument("--membership-port", type=int, default=2379)
    ap.add_argument("--data-port", type=int, default=DATA_PORT)
    ap.add_argument("--config-port", type=int, default=CONFIG_PORT)
    ap.add_argument("--device", default=None, help="cuda:N or cpu (default: cuda:0 if present)")
    ap.add_argument("--id", default=None)
    ap.add_argument("--ttl", type=float, default=1.0, help="membership lease TTL (s)")
    ap.add_argument("--chunk-size", type=int, default=512 * 1000)
    ap.add_argument("--parent-pid", type=int, default=0,
                    help="exit when this process (the launcher) is gone: a launcher killed at its time limit "
                         "must not leave GPU workers behind")
    a = ap.parse_args(argv)
    if a.parent_pid:
        _follow_parent(a.parent_pid)
    node = Node(a.dispatcher, a.membership_port, a.data_port, a.config_port, a.device, a.id, a.chunk_size,
                heartbeat_ttl=a.ttl, exit_on_unrecoverable=True)
    print(f"node {node.node_id} device={node.device} data={node.data_port} config={node.config_port}", flush=True)
    node.run(block=True)
    # Communicator threads of aborted epochs may still sit in backend waits on
    # peers that will never answer; leave without running interpreter
    # finalization over them.
    sys.stdout.flush()
    sys.stderr.flush()
    os._exit(0)


if __name__ == "__main__":
    main()
