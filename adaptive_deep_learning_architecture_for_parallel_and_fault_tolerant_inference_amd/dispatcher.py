"""DEFER dispatcher: partition, place, stream, collect, and recover.

Public API of the reference (`src/dispatcher.py:20-317`):
``DEFER(computeNodes).run_defer(model, partition_layers, input_stream,
output_stream)`` blocks until shutdown, reading inputs from a `queue.Queue`
and putting predictions on another.  The reference body is spliced and
references five undefined methods and five undefined attributes (SURVEY
§2.6); this is a complete implementation of the intended gen-2 design:

* `_worker_monitor` — watches ``/workers/`` in the membership store (our
  etcd stand-in, started in-process unless an external one is given);
* `_partition` — cuts the model with `dag_util` semantics into
  ``part1..partN`` (multi-tensor frontiers allowed), or with the balanced
  planner when the worker count changes;
* `_get_available_workers` / `_acquire_and_configure_worker` — choose live
  workers and push each its slice (manifest + index + weights, ACK 0x06) for
  the current *epoch*;
* `_startDistEdgeInference` — assigns request ids, keeps every in-flight
  input (`inflight_tasks`), bounded by `concurrency_sem`, and streams it to
  stage 0;
* `_intermediate_result_server` — accepts the last stages' connections,
  de-duplicates results by request id, emits them in completion order (or
  request order with ``ordered=True``) and releases credits;
* `_task_watchdog` — a request older than `task_timeout` means its pipeline
  is stuck: re-form it and replay;
* repartition on worker leave (lease expiry / DELETE event) and, with
  ``elastic=True``, on join: bump the epoch, re-plan cuts for the live set,
  reconfigure survivors, replay every unfinished request from its retained
  input.  Recovery-to-steady time is recorded per event in `recoveries`.

The data plane between stages is the workers' business (TCP links, or RCCL
p2p over xGMI between GPU stages); the dispatcher only feeds stage 0 and
collects from the last stage.
"""
from __future__ import annotations

import json
import queue
import socket
import threading
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .graph.manifest import ACK, SliceManifest, build_manifest, send_slice
from .graph.planner import plan_cuts
from .graph.slicer import Slice, partition, validate_slices
from .membership.client import MembershipClient, live_workers
from .membership.server import MembershipServer
from .membership.store import KVStore
from .models.model import Model
from .node_state import socket_recv, socket_send
from .transport.messages import Message, connect, listen, recv_message, send_message
from .utils.telemetry import METRICS, TRACER

DATA_PORT = 6000     # send input data                 (src/dispatcher.py:15)
CONFIG_PORT = 6001   # send model config + weights     (src/dispatcher.py:16)
RESULT_PORT = 6003   # receive results                 (src/dispatcher.py:17)
CTRL_CHUNK = 1 << 16


@dataclass
class Pipeline:
    epoch: int
    part_at: List[str]
    workers: List[str]               # worker id per stage
    records: List[dict]
    stage0: Optional[socket.socket] = None
    lock: threading.Lock = field(default_factory=threading.Lock)


class DEFER:
    def __init__(self, computeNodes: Optional[Sequence[str]] = None, *, membership: Optional[Tuple[str, int]] = None,
                 membership_port: int = 2379, result_port: int = RESULT_PORT, chunk_size: int = 512 * 1000,
                 batch: int = 1, codec: str = "lz4", weight_codec: str = "zfp+lz4", max_inflight: int = 8,
                 task_timeout: float = 30.0, worker_wait: float = 5.0, elastic: bool = False,
                 ordered: bool = False, device_graph: bool = True, min_workers: int = 1,
                 transport: str = "tcp", link_codec: str = "none") -> None:
        """link_codec: compression of the collective stage-to-stage links ("none",
        "lz4", "zvc"; codec/wire.py, on a side stream); `codec` applies to TCP hops.
        transport: stage-to-stage links — "tcp" (framed, codec; any host),
        "rccl" (RCCL p2p over xGMI between GPU workers), "gloo" (CPU workers)."""
        if transport not in ("tcp", "rccl", "gloo"):
            raise ValueError(f"unknown transport {transport!r}")
        self.transport = transport
        self.link_codec = link_codec
        self._store_server = None
        self._store_port = 0
        if transport != "tcp":
            from .parallel.epoch_group import make_store_server
            self._store_server = make_store_server()       # rendezvous for per-epoch communicators
            self._store_port = self._store_server.port
        self.computeNodes = list(computeNodes or [])
        self.dispatchIP = self.get_local_ip()
        self.chunk_size = chunk_size
        self.batch = batch
        self.codec = codec
        self.weight_codec = weight_codec
        self.task_timeout = task_timeout
        self.worker_wait = worker_wait
        self.elastic = elastic
        self.ordered = ordered
        self.device_graph = device_graph
        self.min_workers = min_workers
        # a worker whose config port does not answer within this many seconds is left
        # out of the next epoch even while its membership lease is still alive
        self.probe_timeout = 0.5
        # gen-2 attributes the reference uses but never initialises
        self.worker_lock = threading.Lock()
        self.inflight_lock = threading.Lock()
        self.inflight_tasks: Dict[int, dict] = {}
        self.concurrency_sem = threading.BoundedSemaphore(max_inflight)
        self._shutdown_event = threading.Event()
        self.models_to_dispatch: List[Tuple[SliceManifest, list]] = []
        # membership: external service, or an in-process store + TCP front-end
        self._own_membership = membership is None
        if membership is None:
            self.store = KVStore()
            self.membership_server = MembershipServer(self.store, port=membership_port)
            self.membership_addr = ("127.0.0.1", self.membership_server.port)
        else:
            self.store = None
            self.membership_server = None
            self.membership_addr = tuple(membership)
        self.client = MembershipClient(*self.membership_addr)
        self.result_sock = listen("0.0.0.0", result_port)
        self.result_port = self.result_sock.getsockname()[1]
        self.workers: Dict[str, dict] = {}
        self.pipeline: Optional[Pipeline] = None
        self._epoch = 0
        self._reconf_lock = threading.Lock()
        self._reconf_needed = threading.Event()
        self._next_req = 0
        self._completed = 0
        self.completion_times: List[float] = []
        self.recoveries: List[dict] = []
        self.events: List[Tuple[float, str]] = []
        self._model: Optional[Model] = None
        self._user_cuts: List[str] = []
        self._order_buf: Dict[int, np.ndarray] = {}
        self._next_emit = 0
        self._output: Optional[queue.Queue] = None
        self._result_conns: set = set()

    # ------------------------------------------------------------ helpers
    @staticmethod
    def get_local_ip() -> str:
        s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        try:
            s.connect(("1.1.1.1", 1))
            ip = s.getsockname()[0]
        except OSError:
            ip = "127.0.0.1"
        finally:
            s.close()
        return ip

    def _log(self, msg: str) -> None:
        self.events.append((time.time(), msg))

    @property
    def membership_port(self) -> int:
        return self.membership_addr[1]

    # ---------------------------------------------------------- partition
    def _partition(self, model: Model, layer_parts: Sequence[str]) -> List[Tuple[SliceManifest, list]]:
        """Cut into part1..partN (`src/dispatcher.py:39-53`) -> [(manifest, arrays)]."""
        g = model.graph
        slices = partition(g, list(layer_parts))
        validate_slices(g, slices)
        return [build_manifest(g, s, model.weights) for s in slices]

    # --------------------------------------------------------- membership
    def _worker_monitor(self) -> None:
        """Watch /workers/ and keep `self.workers` current; losing a worker of
        the active pipeline (or gaining one when elastic) triggers repartition."""
        def on_event(ev):
            wid = ev.kv.key[len("/workers/"):]
            with self.worker_lock:
                if ev.type == "PUT":
                    try:
                        rec = json.loads(ev.kv.value)
                    except ValueError:
                        return
                    new = wid not in self.workers
                    self.workers[wid] = rec
                else:
                    new = False
                    self.workers.pop(wid, None)
            p = self.pipeline
            if ev.type == "DELETE" and p is not None and wid in p.workers:
                self._log(f"worker {wid} left (lease expired or revoked)")
                self._reconf_needed.set()
            elif (ev.type == "PUT" and p is not None and wid in p.workers and rec.get("state") == "LINK_ERROR"
                  and rec.get("epoch") == p.epoch):
                self._log(f"worker {wid} reports a broken hop: {rec.get('error')}")
                self._reconf_needed.set()
            elif ev.type == "PUT" and new and self.elastic and p is not None:
                self._log(f"worker {wid} joined")
                self._reconf_needed.set()

        with self.worker_lock:
            self.workers = live_workers(self.client)
        if self.store is not None:
            w = self.store.watch("/workers/")
            while not self._shutdown_event.is_set():
                ev = w.get(timeout=0.1)
                if ev is not None:
                    on_event(ev)
            w.cancel()
        else:
            rw = self.client.watch("/workers/", on_event)
            self._shutdown_event.wait()
            rw.cancel()

    def _get_available_workers(self) -> List[str]:
        with self.worker_lock:
            ws = dict(self.workers)
        if self.computeNodes:
            allowed = set(self.computeNodes)
            ws = {k: v for k, v in ws.items() if k in allowed or v.get("host") in allowed or "0.0.0.0" in allowed}
        # workers that failed to load a slice (StateEnum.PARSE_ERROR) are not offered again
        ws = {k: v for k, v in ws.items() if v.get("state") != "PARSE_ERROR"}
        # deterministic order (host, device) keeps stage placement - and each worker's
        # cached slices - stable across epochs; consecutive GPUs of a host become
        # consecutive stages (neighbouring xGMI peers)
        return sorted(ws, key=lambda k: (ws[k].get("host", ""), ws[k].get("device", ""), k))

    # ---------------------------------------------------------- configure
    def _send_full_configuration(self, rec: dict, manifest: SliceManifest, arrays: list, cfg: dict) -> None:
        """Config push + ACK (`src/dispatcher.py:223-264`)."""
        s = socket.create_connection((rec["host"], int(rec["config_port"])), timeout=5)
        try:
            s.settimeout(120)
            socket_send(json.dumps(cfg).encode(), s, CTRL_CHUNK)
            if not cfg.get("cached"):
                send_slice(s, manifest, arrays, self.chunk_size, self.weight_codec)
            ack = s.recv(1)
            if ack != ACK:
                reason = socket_recv(s, CTRL_CHUNK) if ack else b"connection closed"
                raise RuntimeError(f"worker {rec.get('id')} rejected configuration: {reason.decode(errors='replace')}")
        finally:
            s.close()

    def _acquire_and_configure_worker(self, partition_index: int, wid: str, cfg: dict) -> Optional[str]:
        """Configure worker `wid` with slice `partition_index` (1-based); returns its id or None."""
        with self.worker_lock:
            rec = self.workers.get(wid)
        if rec is None:
            return None
        m, arrays = self.models_to_dispatch[partition_index - 1]
        key = f"{self._model.name}|{','.join(self._cur_cuts)}|{partition_index}|b{self.batch}"
        cfg = dict(cfg)
        cfg["cache_key"] = key
        # a worker keeps every slice it was ever sent resident, so a repartition
        # back to known cuts is a pointer swap instead of a weight push
        cfg["cached"] = key in self._sent_slices.get(wid, set())
        try:
            self._send_full_configuration(rec, m, arrays, cfg)
        except RuntimeError as e:
            if not (cfg["cached"] and "not cached" in str(e)):
                raise
            cfg["cached"] = False
            self._send_full_configuration(rec, m, arrays, cfg)
        self._sent_slices.setdefault(wid, set()).add(key)
        return wid

    def _form_pipeline(self) -> bool:
        """(Re)build the pipeline for the current live worker set; new epoch."""
        with self._reconf_lock:
            t0 = time.time()
            live = self._probe_live(self._get_available_workers())
            if not live:
                self._log(f"no workers available ({len(live)})")
                return False
            g = self._model.graph
            want = len(self._user_cuts) + 1
            k = min(want, len(live)) if not self.elastic else len(live)
            if k == want:
                cuts = list(self._user_cuts)
            else:
                cuts, _ = plan_cuts(g, k, batch=self.batch)
            self._cur_cuts = cuts
            self.models_to_dispatch = self._partition(self._model, cuts)
            members = live[:k]
            self._epoch += 1
            epoch = self._epoch
            old = self.pipeline
            self.pipeline = None
            if old is not None and old.stage0 is not None:
                try:
                    old.stage0.close()
                except OSError:
                    pass
            with self.worker_lock:
                recs = [dict(self.workers[w]) for w in members]
            # configure last stage first so downstream listeners exist early
            for st in reversed(range(k)):
                rec = recs[st]
                nxt = None
                if st < k - 1:
                    nxt = {"host": recs[st + 1]["host"], "port": int(recs[st + 1]["data_port"])}
                cfg = {"cmd": "configure", "epoch": epoch, "stage": st, "stages": k, "batch": self.batch,
                       "next": nxt, "result_addr": [self._result_host(rec), self.result_port],
                       "codec": self.codec, "graph": self.device_graph, "transport": self.transport}
                if self.transport != "tcp":
                    cfg["link_codec"] = self.link_codec
                    cfg["collective"] = {"backend": "nccl" if self.transport == "rccl" else "gloo",
                                         "store_host": self._result_host(rec), "store_port": self._store_port,
                                         "timeout": 30}
                if self._acquire_and_configure_worker(st + 1, members[st], cfg) is None:
                    self._log(f"worker {members[st]} vanished during configuration")
                    return False
            # live workers left out of this epoch drop their old data plane
            for wid in live[k:]:
                self._send_ctrl(wid, {"cmd": "stop_epoch"})
            hello = json.dumps({"epoch": epoch, "from_stage": -1}).encode()
            s0 = connect(recs[0]["host"], int(recs[0]["data_port"]), hello=hello)
            self.pipeline = Pipeline(epoch, cuts, members, recs, s0)
            self._log(f"epoch {epoch}: {k} stages on {members} cuts={cuts} ({(time.time() - t0) * 1e3:.0f} ms)")
            return True

    def _send_ctrl(self, wid: str, cmd: dict) -> bool:
        with self.worker_lock:
            rec = self.workers.get(wid)
        if rec is None:
            return False
        try:
            s = socket.create_connection((rec["host"], int(rec["config_port"])), timeout=2)
            try:
                socket_send(json.dumps(cmd).encode(), s, CTRL_CHUNK)
                return s.recv(1) == ACK
            finally:
                s.close()
        except OSError:
            return False

    def _probe_live(self, wids: Sequence[str]) -> List[str]:
        """Keep the workers whose config server answers a ``status`` command.

        A SIGKILLed worker keeps its membership record until the lease expires
        (TTL), so a re-plan triggered by a socket error would otherwise place a
        stage on it, fail mid-push and start over.  The probes run in parallel:
        a dead local process refuses the connect at once, an unreachable host
        costs at most `probe_timeout`."""
        if len(wids) == 0:
            return []
        ok: Dict[str, bool] = {}

        def probe(wid: str) -> None:
            with self.worker_lock:
                rec = self.workers.get(wid)
            if rec is None:
                ok[wid] = False
                return
            try:
                with socket.create_connection((rec["host"], int(rec["config_port"])), timeout=self.probe_timeout) as s:
                    s.settimeout(self.probe_timeout)
                    socket_send(json.dumps({"cmd": "status"}).encode(), s, CTRL_CHUNK)
                    ok[wid] = s.recv(1) == ACK
            except OSError:
                ok[wid] = False

        ts = [threading.Thread(target=probe, args=(w,), daemon=True) for w in wids]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        dead = [w for w in wids if not ok.get(w)]
        if dead:
            self._log(f"unresponsive (lease still alive): {dead}")
        return [w for w in wids if ok.get(w)]

    def _result_host(self, rec: dict) -> str:
        return "127.0.0.1" if rec.get("host") in ("127.0.0.1", "localhost") else self.dispatchIP

    # ------------------------------------------------------- data: input
    def _send_to_stage0(self, rid: int, x: np.ndarray) -> bool:
        p = self.pipeline
        if p is None or p.stage0 is None:
            return False
        m = Message(1, rid, p.epoch, int(x.shape[0]), [x], [False])
        try:
            with p.lock:
                send_message(p.stage0, m, self.codec, self.chunk_size, timeout_ms=10000)
            with self.inflight_lock:
                if rid in self.inflight_tasks:
                    self.inflight_tasks[rid]["epoch"] = p.epoch
            return True
        except (OSError, RuntimeError):
            self._reconf_needed.set()
            return False

    def _startDistEdgeInference(self, input_stream: "queue.Queue") -> None:
        """Input pump (`src/dispatcher.py:99-107`): request ids, credits, retention."""
        while not self._shutdown_event.is_set():
            try:
                x = input_stream.get(timeout=0.1)
            except queue.Empty:
                continue
            if x is None:
                continue
            x = np.asarray(x, np.float32)
            if x.ndim == 3:
                x = x[None]
            for i in range(0, x.shape[0], self.batch):
                chunk = np.ascontiguousarray(x[i:i + self.batch])
                while not self._shutdown_event.is_set():
                    if self.concurrency_sem.acquire(timeout=0.1):
                        break
                if self._shutdown_event.is_set():
                    return
                self._wait_and_forward(1, chunk)

    def _wait_and_forward(self, partition_index: int, data: np.ndarray) -> Optional[int]:
        """`src/dispatcher.py:176-201`: register the task in the in-flight registry
        (retained input = the replay source of the watchdog) and forward it.  The
        dispatcher feeds partition 1 only; later partitions are fed stage to
        stage by the workers (TCP or RCCL), not relayed through this hub."""
        if partition_index != 1:
            raise ValueError("the dispatcher forwards to partition 1; stages feed each other")
        rid = self._next_req
        self._next_req += 1
        with self.inflight_lock:
            self.inflight_tasks[rid] = {"partition": partition_index, "data": data, "start_time": time.time(),
                                        "epoch": None}
        self._forward_data_to_worker(rid, data)
        return rid

    def _forward_data_to_worker(self, rid: int, data: np.ndarray) -> bool:
        """`src/dispatcher.py:204-220` (one persistent framed connection per epoch
        instead of a new TCP connection per message)."""
        return self._send_to_stage0(rid, data)

    # ------------------------------------------- reference-named helpers
    @staticmethod
    def _comp(arr: np.ndarray) -> bytes:
        """`src/dispatcher.py:92-93`: zfp (reversible) then LZ4 frame, native codecs."""
        from . import codec
        return codec.comp(arr)

    @staticmethod
    def _decomp(byts) -> np.ndarray:
        """`src/dispatcher.py:94-98`."""
        from . import codec
        return codec.decomp(byts)

    def _send_weights(self, weights: Sequence[np.ndarray], sock: socket.socket,
                      chunk_size: Optional[int] = None) -> None:
        """`src/dispatcher.py:76-89`: u64be array count, then one framed `_comp(array)`
        per array in Keras `get_weights()` order (read back by `Node._recv_weights`)."""
        sock.sendall(len(weights).to_bytes(8, "big"))
        for w in weights:
            socket_send(self._comp(np.require(w, None, ["C"])), sock, chunk_size or self.chunk_size)

    def _update_localhost(self, conn, raw_ip: str, worker_cli: dict) -> None:
        """`src/dispatcher.py:164-173`: a peer address outside `computeNodes` maps to
        127.0.0.1 when the deployment is all-local."""
        final_ip = raw_ip
        with self.worker_lock:
            if raw_ip not in self.computeNodes and "127.0.0.1" in self.computeNodes:
                final_ip = "127.0.0.1"
        worker_cli[conn] = final_ip

    def _result_server(self, output_stream: "queue.Queue") -> None:
        """Gen-1 result sink (`src/dispatcher.py:109-119`) = the gen-2 server here."""
        self._intermediate_result_server(output_stream)

    def _dispatchModels(self, models: Optional[Sequence[str]], nodeIPs: Sequence[str]) -> bool:
        """Gen-1 static placement (`src/dispatcher.py:55-73`, dead code there): restrict
        the pipeline to the workers on `nodeIPs` (host or worker id) and configure
        one slice per worker as a new epoch.  `models`: the cut list (layer names),
        or None to keep the current cuts.  Needs the model of a running `run_defer`."""
        if self._model is None:
            raise RuntimeError("_dispatchModels needs the model of a running run_defer")
        if models is not None:
            self._user_cuts = list(models)
        self.computeNodes = list(nodeIPs)
        return self._form_pipeline()

    # ------------------------------------------------------ data: results
    def _intermediate_result_server(self, output_stream: "queue.Queue") -> None:
        self._output = output_stream
        while not self._shutdown_event.is_set():
            try:
                self.result_sock.settimeout(0.2)
                conn, _ = self.result_sock.accept()
            except socket.timeout:
                continue
            except OSError:
                break
            conn.settimeout(None)
            conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            self._result_conns.add(conn)
            threading.Thread(target=self._result_conn, args=(conn, output_stream), daemon=True).start()

    def _result_conn(self, conn: socket.socket, output_stream: "queue.Queue") -> None:
        try:
            hello = socket_recv(conn, CTRL_CHUNK)
            if not hello:
                return
            while not self._shutdown_event.is_set():
                m = recv_message(conn, self.chunk_size)
                if m is None:
                    break
                self._complete(m, output_stream)
        except (OSError, RuntimeError, ValueError):
            pass
        finally:
            self._result_conns.discard(conn)
            conn.close()

    def _complete(self, m: Message, output_stream: "queue.Queue") -> None:
        with self.inflight_lock:
            task = self.inflight_tasks.pop(m.req_id, None)
        if task is None:
            METRICS.inc("results_duplicate_dropped")
            return                                   # duplicate from a replay: drop
        METRICS.observe("request_latency_ms", (time.time() - task["start_time"]) * 1e3)
        METRICS.inc("results")
        TRACER.event("complete", req=m.req_id, epoch=m.epoch, count=m.count)
        pred = m.tensors[0]
        if m.bf16 and m.bf16[0]:
            pred = (pred.astype(np.uint32) << 16).view(np.float32)
        pred = np.array(pred[: m.count])             # own, writable copy for the caller
        self._completed += 1
        self.completion_times.append(time.time())
        if self.ordered:
            with self.inflight_lock:
                self._order_buf[m.req_id] = pred
                while self._next_emit in self._order_buf:
                    output_stream.put(self._order_buf.pop(self._next_emit))
                    self._next_emit += 1
        else:
            output_stream.put(pred)
        self.concurrency_sem.release()

    # ----------------------------------------------------- fault handling
    def _task_watchdog(self) -> None:
        while not self._shutdown_event.wait(0.05):
            now = time.time()
            stale = False
            with self.inflight_lock:
                for t in self.inflight_tasks.values():
                    if now - t["start_time"] > self.task_timeout:
                        stale = True
                        break
            if stale and self.pipeline is not None:
                self._log("watchdog: stale in-flight task")
                self._reconf_needed.set()
            if self._reconf_needed.is_set():
                self._reconf_needed.clear()
                self._recover()

    def _recover(self) -> None:
        t_fail = time.time()
        done_before = self._completed
        ok = False
        deadline = t_fail + max(self.worker_wait, 10.0)
        while not self._shutdown_event.is_set() and time.time() < deadline:
            # let expired leases drain so the live set is accurate
            time.sleep(0.05)
            try:
                ok = self._form_pipeline()
            except Exception as e:  # noqa: BLE001 - a member died during configuration; retry
                self._log(f"reconfigure failed: {type(e).__name__}: {e}")
                ok = False
            if ok:
                break
            time.sleep(0.1)
        if not ok:
            self._log("recovery failed: no usable workers")
            return
        t_ready = time.time()
        with self.inflight_lock:
            replay = sorted(self.inflight_tasks.items())
            for _, t in replay:
                t["start_time"] = time.time()
        for rid, t in replay:
            self._send_to_stage0(rid, t["data"])
        self.recoveries.append({"t_fail": t_fail, "t_ready": t_ready, "replayed": len(replay),
                                "epoch": self._epoch, "reconfig_ms": (t_ready - t_fail) * 1e3,
                                "completed_before": done_before})
        self._log(f"recovered in {(t_ready - t_fail) * 1e3:.0f} ms, replayed {len(replay)} requests")

    # --------------------------------------------------------------- main
    def run_defer(self, model: Model, partition_layers: Sequence[str], input_stream: "queue.Queue",
                  output_stream: "queue.Queue") -> None:
        """Blocks until `shutdown()` (`src/dispatcher.py:273-317`)."""
        if self.membership_server is not None and not self.membership_server._thread.is_alive():
            self.membership_server.start()
        self._model = model
        self._user_cuts = list(partition_layers)
        self._cur_cuts = list(partition_layers)
        self._sent_slices: Dict[str, set] = {}
        # 1. worker monitor
        threading.Thread(target=self._worker_monitor, daemon=True, name="defer-monitor").start()
        # 2. partition (validates the cut list up front)
        self.models_to_dispatch = self._partition(model, partition_layers)
        # 3. wait for workers
        deadline = time.time() + self.worker_wait
        while time.time() < deadline:
            with self.worker_lock:
                self.workers.update(live_workers(self.client))
            if len(self._get_available_workers()) >= max(1, self.min_workers):
                break
            time.sleep(0.1)
        else:
            self._log(f"no workers registered after {self.worker_wait} s")
            self._shutdown_event.set()
            return
        # 4. result server
        threading.Thread(target=self._intermediate_result_server, args=(output_stream,), daemon=True,
                         name="defer-results").start()
        # place the pipeline (retry while members come up)
        if not self._form_pipeline():
            self._shutdown_event.set()
            return
        # 5. watchdog (also runs recoveries)
        threading.Thread(target=self._task_watchdog, daemon=True, name="defer-watchdog").start()
        # 6. input pump
        threading.Thread(target=self._startDistEdgeInference, args=(input_stream,), daemon=True,
                         name="defer-input").start()
        # 7. stay alive
        try:
            while not self._shutdown_event.is_set():
                self._shutdown_event.wait(0.5)
        except KeyboardInterrupt:
            pass
        finally:
            self._shutdown_event.set()

    def shutdown(self, stop_workers: bool = False) -> None:
        if stop_workers:
            for rec in list(self.workers.values()):
                try:
                    s = socket.create_connection((rec["host"], int(rec["config_port"])), timeout=2)
                    socket_send(json.dumps({"cmd": "shutdown"}).encode(), s, CTRL_CHUNK)
                    s.recv(1)
                    s.close()
                except OSError:
                    pass
        self._shutdown_event.set()
        for c in [self.result_sock] + list(self._result_conns):
            try:
                c.shutdown(socket.SHUT_RDWR)
            except OSError:
                pass
            try:
                c.close()
            except OSError:
                pass
        p = self.pipeline
        if p is not None and p.stage0 is not None:
            try:
                p.stage0.close()
            except OSError:
                pass
        if self.membership_server is not None:
            self.membership_server.stop()

    # ---------------------------------------------------------- metrics
    def throughput(self, window: float = 1.0, now: Optional[float] = None) -> float:
        now = now or time.time()
        return sum(1 for t in self.completion_times if now - window <= t <= now) * self.batch / window

    def recovery_to_steady_ms(self, t_kill: Optional[float] = None, window: float = 0.5,
                              frac: float = 0.95) -> List[float]:
        """Per recovery: ms from the failure (`t_kill` if the caller knows when it
        injected it, else the detection time) until the windowed throughput first
        returns to >= frac x the post-recovery steady state."""
        out = []
        ts = np.array(self.completion_times)
        for r in self.recoveries:
            post = ts[ts > r["t_ready"]]
            if len(post) < 4:
                continue
            steady_span = post[-1] - post[len(post) // 2]
            if steady_span <= 0:
                continue
            steady = (len(post) - len(post) // 2 - 1) / steady_span
            t = t_kill if t_kill is not None else r["t_fail"]
            t0 = t
            found = None
            while t < post[-1]:
                n = np.count_nonzero((ts > t) & (ts <= t + window))
                if t > r["t_ready"] and n / window >= frac * steady:
                    found = t
                    break
                t += window / 10
            if found is not None:
                out.append((found - t0) * 1e3)
        return out
