"""DEFER PP x DP replicas and the fast failure paths (CPU, in-process workers).

* R = live // k replicas of a k-stage pipeline serve round-robin, exactly once
  (the reference lets any idle worker take any partition,
  `src/dispatcher.py:176-194`);
* a dead worker is detected through its session connection (no lease TTL),
  only its replica is re-formed and the other keeps its epoch;
* a stage whose own compute fails reports STAGE_ERROR and is quarantined;
* `_probe_live` drops a worker whose lease is alive but whose process is not.
"""
import queue
import socket
import threading
import time

import numpy as np
import pytest

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.dispatcher import DEFER
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.model import resnet
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.node import Node


@pytest.fixture(scope="module")
def tiny():
    return resnet("resnet_tiny", input_shape=(32, 32, 3), classes=10, seed=5)


def _nodes(d, n, prefix):
    nodes = [Node(membership_port=d.membership_port, data_port=0, config_port=0, device="cpu", node_id=f"{prefix}{i}",
                  heartbeat_ttl=2.0) for i in range(n)]
    for nd in nodes:
        nd.run(block=False)
    return nodes


def _wait(pred, timeout=30.0):
    t0 = time.time()
    while time.time() - t0 < timeout:
        if pred():
            return True
        time.sleep(0.05)
    return False


def test_pp_dp_replicas_serve_and_reform_one(tiny):
    d = DEFER(membership_port=0, result_port=0, worker_wait=20, ordered=True, batch=1, weight_codec="lz4",
              min_workers=4, max_inflight=2)
    d.membership_server.start()
    nodes = _nodes(d, 4, "r")
    try:
        inq, outq = queue.Queue(), queue.Queue()
        threading.Thread(target=d.run_defer, args=(tiny, ["conv4_block1_out"], inq, outq), daemon=True).start()
        assert _wait(lambda: len(d.replicas) == 2)
        reps = {r: (p.epoch, list(p.workers)) for r, p in d.replicas.items()}
        assert sorted(len(w) for _, w in reps.values()) == [2, 2]
        rng = np.random.default_rng(3)
        xs = [rng.standard_normal((1, 32, 32, 3)).astype(np.float32) for _ in range(24)]
        want = tiny.predict(np.concatenate(xs), device="cpu")
        for x in xs[:12]:
            inq.put(x)
        got = [outq.get(timeout=60) for _ in range(12)]
        # both replicas served: every worker ran micro-batches
        assert all(nd.runtime is not None and nd.runtime.processed > 0 for nd in nodes)
        # kill one worker of replica A: only A is re-formed, B keeps its epoch
        ra = min(reps)
        rb = max(reps)
        victim = reps[ra][1][1]
        vnode = next(nd for nd in nodes if nd.node_id == victim)
        t_kill = time.time()
        vnode.stop()
        assert _wait(lambda: d.replicas.get(ra) is not None and d.replicas[ra].epoch != reps[ra][0])
        assert d.replicas[rb].epoch == reps[rb][0]
        assert victim not in d.replicas[ra].workers
        assert _wait(lambda: len(d.recoveries) > 0)       # recorded after the replay that follows the re-form
        rec = d.recoveries[0]
        assert rec["replica"] == ra
        assert rec["t_fail"] - t_kill < 1.0          # session EOF, not the 2 s lease
        for x in xs[12:]:
            inq.put(x)
        got += [outq.get(timeout=60) for _ in range(12)]
        time.sleep(0.3)
        assert outq.empty()                          # exactly once
        np.testing.assert_allclose(np.concatenate(got), want, rtol=1e-4, atol=1e-5)
    finally:
        d.shutdown(stop_workers=True)
        for nd in nodes:
            nd.stop()


def test_stage_error_is_quarantined(tiny):
    d = DEFER(membership_port=0, result_port=0, worker_wait=20, ordered=True, batch=1, weight_codec="lz4",
              min_workers=3, replicas=1, max_inflight=2)
    d.membership_server.start()
    nodes = _nodes(d, 3, "q")
    bad = nodes[1]
    real = bad.stage_compute

    class Broken:
        def __init__(self, c):
            self.c = c

        def __getattr__(self, k):
            return getattr(self.c, k)

        def run_host(self, *a, **kw):
            raise RuntimeError("injected compute fault")

    armed = threading.Event()

    def faulty(cfg, g, w, **kw):
        c = real(cfg, g, w, **kw)
        return Broken(c) if armed.is_set() else c

    bad.stage_compute = faulty
    try:
        inq, outq = queue.Queue(), queue.Queue()
        threading.Thread(target=d.run_defer, args=(tiny, ["conv3_block1_out", "conv4_block1_out"], inq, outq),
                         daemon=True).start()
        assert _wait(lambda: d.pipeline is not None)
        x = np.random.default_rng(4).standard_normal((1, 32, 32, 3)).astype(np.float32)
        want = tiny.predict(x, device="cpu")
        inq.put(x)
        np.testing.assert_allclose(outq.get(timeout=60), want, rtol=1e-4, atol=1e-5)
        armed.set()
        d._dispatchModels(None, [])                  # re-form: the faulty worker now fails its compute
        for _ in range(3):
            inq.put(x)
        outs = [outq.get(timeout=60) for _ in range(3)]
        for y in outs:
            np.testing.assert_allclose(y, want, rtol=1e-4, atol=1e-5)
        assert bad.node_id in d._quarantine
        assert bad.node_id not in d.pipeline.workers
        assert any("stage error" in e for _, e in d.events)
    finally:
        d.shutdown(stop_workers=True)
        for nd in nodes:
            nd.stop()


def test_probe_live_drops_dead_worker_with_live_lease():
    d = DEFER(membership_port=0, result_port=0)
    live = socket.socket()
    live.bind(("127.0.0.1", 0))
    live.listen(4)
    dead = socket.socket()
    dead.bind(("127.0.0.1", 0))
    dead_port = dead.getsockname()[1]
    dead.close()                                      # nothing listens there any more

    def serve():
        from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.node_state import \
            socket_recv
        while True:
            try:
                c, _ = live.accept()
            except OSError:
                return
            socket_recv(c, 1 << 16)
            c.sendall(b"\x06")
            c.close()

    threading.Thread(target=serve, daemon=True).start()
    d.workers = {"a": {"host": "127.0.0.1", "config_port": live.getsockname()[1]},
                 "b": {"host": "127.0.0.1", "config_port": dead_port}}
    try:
        assert d._probe_live(["a", "b"]) == ["a"]
        assert any("unresponsive" in e for _, e in d.events)
    finally:
        live.close()
        d.shutdown()


def test_uint8_ingest_shm_caffe_preprocess(tiny):
    """uint8 image requests through same-host shared memory, caffe
    `preprocess_input` applied by stage 0 (`test/test.py:20-23`)."""
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops.eltwise import \
        preprocess_ref
    d = DEFER(membership_port=0, result_port=0, worker_wait=20, ordered=True, batch=2, weight_codec="lz4",
              min_workers=2, replicas=1, preprocess="caffe")
    assert d._shm is not None
    d.membership_server.start()
    nodes = _nodes(d, 2, "u")
    try:
        inq, outq = queue.Queue(), queue.Queue()
        threading.Thread(target=d.run_defer, args=(tiny, ["conv3_block1_out"], inq, outq), daemon=True).start()
        rng = np.random.default_rng(5)
        xs = [rng.integers(0, 256, (3, 32, 32, 3), dtype=np.uint8) for _ in range(3)]
        for x in xs:
            inq.put(x)
        got = np.concatenate([outq.get(timeout=60) for _ in range(6)])
        want = tiny.predict(preprocess_ref(np.concatenate(xs), "caffe"), device="cpu")
        np.testing.assert_allclose(got, want, rtol=1e-4, atol=1e-5)
        assert len(d._shm._all) >= 1 and {s.nbytes for s in d._shm._all} <= {3072, 2 * 3072}
    finally:
        d.shutdown(stop_workers=True)
        for nd in nodes:
            nd.stop()


def test_link_error_report_triggers_replan_without_a_death(tiny):
    """A stage that publishes LINK_ERROR for the serving epoch (what a broken hop
    does, node.py `_fail`) makes the dispatcher re-form that replica at once; no
    process dies, so neither the session EOF nor the lease can be the trigger."""
    d = DEFER(membership_port=0, result_port=0, worker_wait=20, ordered=True, batch=1, weight_codec="lz4",
              min_workers=2, replicas=1)
    d.membership_server.start()
    nodes = _nodes(d, 2, "l")
    try:
        inq, outq = queue.Queue(), queue.Queue()
        threading.Thread(target=d.run_defer, args=(tiny, ["conv3_block1_out"], inq, outq), daemon=True).start()
        assert _wait(lambda: d.pipeline is not None)
        e0 = d.pipeline.epoch
        x = np.random.default_rng(6).standard_normal((1, 32, 32, 3)).astype(np.float32)
        inq.put(x)
        outq.get(timeout=60)
        nd = next(n for n in nodes if n.node_id == d.pipeline.workers[1])
        rt = nd.runtime
        rt.error = "recv: injected broken hop"
        t0 = time.time()
        nd.report_failure(rt, "LINK_ERROR")
        assert _wait(lambda: d.pipeline is not None and d.pipeline.epoch > e0, timeout=10)
        assert time.time() - t0 < 1.5                      # well under the 2 s lease TTL of these nodes
        assert any("reports a broken hop" in e for _, e in d.events)
        inq.put(x)
        np.testing.assert_allclose(outq.get(timeout=60), tiny.predict(x, device="cpu"), rtol=1e-4, atol=1e-5)
        # a late report about the retired epoch is ignored
        n_rec = len(d.recoveries)
        nd.report_failure(rt, "LINK_ERROR")
        time.sleep(0.3)
        assert len(d.recoveries) == n_rec
    finally:
        d.shutdown(stop_workers=True)
        for n in nodes:
            n.stop()


def test_unrecoverable_worker_is_dropped_and_replanned(tiny):
    """A stage whose communicator abort exceeded its deadline gives up
    (node.py `give_up`): it publishes UNRECOVERABLE and stops.  The dispatcher
    treats that like a dead process -- the chain is re-formed on the other
    workers at once and the worker is not offered again until a fresh process
    (new pid) registers under its id."""
    d = DEFER(membership_port=0, result_port=0, worker_wait=20, ordered=True, batch=1, weight_codec="lz4",
              min_workers=2, replicas=1)
    d.membership_server.start()
    nodes = _nodes(d, 3, "u")
    try:
        inq, outq = queue.Queue(), queue.Queue()
        threading.Thread(target=d.run_defer, args=(tiny, ["conv3_block1_out"], inq, outq), daemon=True).start()
        assert _wait(lambda: d.pipeline is not None)
        e0 = d.pipeline.epoch
        x = np.random.default_rng(7).standard_normal((1, 32, 32, 3)).astype(np.float32)
        inq.put(x)
        outq.get(timeout=60)
        victim = d.pipeline.workers[1]
        nd = next(n for n in nodes if n.node_id == victim)
        t0 = time.time()
        nd.give_up(nd.runtime, "injected: ncclCommAbort exceeded its deadline")
        assert nd.unrecoverable is not None
        assert _wait(lambda: d.pipeline is not None and d.pipeline.epoch > e0 and victim not in d.pipeline.workers,
                     timeout=10)
        assert time.time() - t0 < 1.5
        assert victim not in d._get_available_workers()
        assert any("unrecoverable" in e for _, e in d.events)
        inq.put(x)
        np.testing.assert_allclose(outq.get(timeout=60), tiny.predict(x, device="cpu"), rtol=1e-4, atol=1e-5)
    finally:
        d.shutdown(stop_workers=True)
        for n in nodes:
            n.stop()


def test_prepare_hints_wait_longer_after_a_reformed_epoch():
    """Background `prepare` (building the likely next plans' slices) competes with the serving threads: after a
    re-formed epoch it waits `recovery_prepare_delay` (the loopback hang run's dip ~1 s after recovery came from
    it), after a first epoch only `prepare_delay`."""
    d = DEFER(membership_port=0, result_port=0, resident=False, prepare=True)

    class _G:
        graph = object()

    waits = []

    class _Ev:
        def wait(self, t):
            waits.append(t)
            return True                               # behave as shut down: stop right after the wait

        def is_set(self):
            return False

    real_model, real_ev = d._model, d._shutdown_event
    d._model, d._model_key, d._resident = _G(), "m", {"a": {"m"}}
    d._shutdown_event = _Ev()
    try:
        d._after_epoch(None, reformed=False)
        d._after_epoch(None, reformed=True)
    finally:
        d._model, d._shutdown_event = real_model, real_ev
        d.shutdown()
    assert waits == [d.prepare_delay, d.recovery_prepare_delay]
    assert d.recovery_prepare_delay > d.prepare_delay
