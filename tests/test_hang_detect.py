"""Hang (no-progress) detection on CPU: a stage whose compute loop wedges while
its process, sessions and heartbeat thread stay alive.

The reference tracks every hop's `start_time` for a watchdog
(`src/dispatcher.py:186-194,302-304`) but never defines the watchdog.  Here
each worker's native heartbeat carries its completed-micro-batch counter; the
dispatcher declares a stage hung when its replica holds work and the counter
has not advanced for max(hang_factor x measured period, the replica's floor),
then re-forms and replays as for a kill.  The floor (DEFER.hang_floor) is
derived from the stages' device kind and the period's jitter unless given.
"""
import os
import queue
import signal
import subprocess
import sys
import threading
import time

import numpy as np
import pytest

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.dispatcher import DEFER
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.model import resnet
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.native import runtime

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = "adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd"


def _spawn_worker(port, wid):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    return subprocess.Popen([sys.executable, "-m", f"{PKG}.node", "--membership-port", str(port), "--data-port", "0",
                             "--config-port", "0", "--device", "cpu", "--id", wid, "--ttl", "1.0"],
                            env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, start_new_session=True)


@pytest.fixture(scope="module")
def tiny():
    return resnet("resnet_tiny", input_shape=(32, 32, 3), classes=10, seed=5)


def test_heartbeat_carries_progress_counter():
    rt = runtime()
    mon = rt.hb_monitor_start(0)
    snd = rt.hb_sender_start("127.0.0.1", rt.hb_monitor_port(mon), "w0", 1000)
    try:
        time.sleep(0.05)
        rt.hb_sender_progress(snd, 7)
        time.sleep(0.02)
        prog = {w: (c, a, st, ep) for w, c, a, st, ep in rt.hb_monitor_progress(mon)}
        assert prog["w0"][0] == 7 and prog["w0"][1] < 0.1 and prog["w0"][2] == 0.0
        rt.hb_sender_progress(snd, 8, 3_000_000, 2)
        time.sleep(0.12)
        prog = {w: (c, a, st, ep) for w, c, a, st, ep in rt.hb_monitor_progress(mon)}
        assert prog["w0"][0] == 8 and prog["w0"][1] >= 0.1          # beats continue, counter stands still
        assert abs(prog["w0"][2] - 3e-3) < 1e-9 and prog["w0"][3] == 2
        ages = dict(rt.hb_monitor_ages(mon))
        assert ages["w0"] < 0.05
    finally:
        rt.hb_sender_stop(snd)
        rt.hb_monitor_stop(mon)


@pytest.mark.parametrize("transport", ["tcp", "gloo"])
def test_hung_stage_detected_and_replayed_exactly_once(tiny, transport):
    # the DEFER defaults: three CPU worker processes share this host with the test runner, and a healthy
    # CPU stage can stall > 200 ms under that contention, so the derived floor of a replica with CPU stages
    # is 0.75 s (DEFER.hang_floor); the GPU twin (tests/test_defer_gpu.py) runs at the all-GPU 0.2 s
    d = DEFER(membership_port=0, result_port=0, worker_wait=20, batch=1, max_inflight=4, weight_codec="lz4",
              min_workers=3, replicas=1, task_timeout=30, transport=transport)
    assert d.hang_min_s is None
    d.membership_server.start()
    procs = [_spawn_worker(d.membership_port, f"h{i}") for i in range(3)]
    stop = threading.Event()
    try:
        inq, outq = queue.Queue(8), queue.Queue()
        threading.Thread(target=d.run_defer, args=(tiny, ["conv3_block1_out", "conv4_block1_out"], inq, outq),
                         daemon=True).start()
        x = np.random.default_rng(3).standard_normal((1, 32, 32, 3)).astype(np.float32)
        want = tiny.predict(x, device="cpu")
        sent = [0]

        def feeder():
            while not stop.is_set():
                try:
                    inq.put(x, timeout=0.05)
                    sent[0] += 1
                except queue.Full:
                    continue

        feed = threading.Thread(target=feeder, daemon=True)
        feed.start()
        res = [outq.get(timeout=120) for _ in range(40)]
        assert len(d.pipeline.workers) == 3, (d.hangs, d.events[-6:])
        victim = d.pipeline.workers[1]
        assert d.hang_threshold(d.pipeline.replica, d.pipeline.epoch) is not None
        assert d.hang_floor(d.pipeline.replica) >= DEFER.HANG_CPU_MIN_S
        assert d.hangs == [], f"healthy CPU stages called hung at the defaults: {d.hangs}"
        t_hang = time.time()
        d.inject_fault(victim, "hang")              # over the worker's control channel
        t_end = time.time() + 60
        while not d.recoveries and time.time() < t_end:
            try:
                res.append(outq.get(timeout=0.05))
            except queue.Empty:
                pass
        assert d.hangs, d.events[-5:]
        h = d.hangs[0]
        detect_ms = (h["t"] - t_hang) * 1e3
        print(f"{transport}: hung stage {h['stage']} ({h['worker']}) detected {detect_ms:.0f} ms after the hang, "
              f"threshold {h['threshold_ms']} ms")
        assert h["worker"] == victim and h["stage"] == 1
        # the threshold is max(20 x stage time, the 0.75 s CPU floor); a loaded CI CPU can stretch the stage time
        assert h["threshold_ms"] >= 1e3 * DEFER.HANG_CPU_MIN_S
        assert detect_ms < h["threshold_ms"] + 150.0
        for _ in range(20):
            res.append(outq.get(timeout=120))
        stop.set()
        feed.join()                          # `sent` is final only once the feeder is out of put()
        d.inject_fault(victim, "clear")      # the wedged stage wakes up: its stale outputs must not leak out
        time.sleep(0.5)
        total = sent[0]                      # what is still queued is consumed too: every input gets its answer
        while len(res) < total:
            res.append(outq.get(timeout=120))
        time.sleep(0.5)
        assert outq.empty()                                  # exactly once
        assert len(res) == total
        for y in res:
            np.testing.assert_allclose(y, want, rtol=1e-4, atol=1e-5)
        assert victim not in d.pipeline.workers and len(d.pipeline.workers) == 2
        assert d.duplicates_dropped >= 0
        print(f"{transport}: {total} requests answered exactly once, duplicates dropped {d.duplicates_dropped}")
    finally:
        stop.set()
        d.shutdown(stop_workers=True)
        for p in procs:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
            p.wait(timeout=10)


def test_slow_upstream_after_idle_is_not_a_hang(tiny):
    """An unbalanced 3-stage cut under low-rate traffic: stage 0 takes 0.3 s per
    micro-batch, stages 1 and 2 a few ms (their hang threshold is the 0.2 s
    floor).  After an idle gap each request spends 0.3 s in stage 0 while the
    downstream stages sit idle; their stall clock must start when the request
    can reach them, not at their own last progress, so no stage is called hung
    (a fast downstream stage was quarantined the moment a request
    that waited longer than its threshold upstream arrived)."""
    d = DEFER(membership_port=0, result_port=0, worker_wait=20, batch=1, max_inflight=4, weight_codec="lz4",
              min_workers=3, replicas=1, task_timeout=30, transport="tcp", hang_min_s=0.2, hang_factor=10)
    d.membership_server.start()
    procs = [_spawn_worker(d.membership_port, f"s{i}") for i in range(3)]
    try:
        inq, outq = queue.Queue(8), queue.Queue()
        threading.Thread(target=d.run_defer, args=(tiny, ["conv3_block1_out", "conv4_block1_out"], inq, outq),
                         daemon=True).start()
        x = np.random.default_rng(4).standard_normal((1, 32, 32, 3)).astype(np.float32)
        t_end = time.time() + 120
        while d.pipeline is None and time.time() < t_end:
            time.sleep(0.05)
        assert d.pipeline is not None and len(d.pipeline.workers) == 3
        d.inject_fault(d.pipeline.workers[0], "delay:0.3")
        for _ in range(6):                               # overlapping requests: the replica period is measured
            inq.put(x)
        for _ in range(6):
            outq.get(timeout=120)
        assert d.hang_threshold(d.pipeline.replica, d.pipeline.epoch) is not None
        time.sleep(1.0)                                  # idle gap
        for _ in range(5):                               # low-rate traffic: one request at a time
            inq.put(x)
            outq.get(timeout=120)
            time.sleep(0.3)
        assert not d.hangs, d.hangs
        assert not d.recoveries and len(d.pipeline.workers) == 3, d.events[-5:]
    finally:
        d.shutdown(stop_workers=True)
        for p in procs:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
            p.wait(timeout=10)


def test_slow_first_microbatches_are_warmup_not_a_hang(tiny):
    """A stage whose first micro-batches of an epoch are slow (one-off work such as a GPU stage capturing
    the hipGraph of its second micro-batch set) is not called hung while it has completed fewer than
    DEFER.HANG_WARMUP micro-batches, even though the replica's period measured from the first result
    would put its threshold at the 0.2 s floor."""
    d = DEFER(membership_port=0, result_port=0, worker_wait=20, batch=1, max_inflight=4, weight_codec="lz4",
              min_workers=2, replicas=1, task_timeout=30, transport="tcp", hang_min_s=0.2, hang_factor=10)
    d.HANG_WARMUP = 8 if DEFER.HANG_WARMUP else 0        # the 4 requests that measure the period stay in warm-up
    d.membership_server.start()
    procs = [_spawn_worker(d.membership_port, f"w{i}") for i in range(2)]
    try:
        inq, outq = queue.Queue(8), queue.Queue()
        threading.Thread(target=d.run_defer, args=(tiny, ["conv3_block1_out"], inq, outq), daemon=True).start()
        x = np.random.default_rng(5).standard_normal((1, 32, 32, 3)).astype(np.float32)
        for _ in range(4):                               # overlapping requests: the period is measured
            inq.put(x)
        for _ in range(4):
            outq.get(timeout=120)
        assert d.hang_threshold(d.pipeline.replica, d.pipeline.epoch) is not None
        d.inject_fault(d.pipeline.workers[1], "delay:0.6")   # stage 1's micro-batches 5 and 6: 0.6 s each
        for _ in range(2):
            inq.put(x)
        for _ in range(2):
            outq.get(timeout=120)
        assert not d.hangs, d.hangs
        assert not d.recoveries and len(d.pipeline.workers) == 2, d.events[-5:]
    finally:
        d.shutdown(stop_workers=True)
        for p in procs:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
            p.wait(timeout=10)


def test_hang_floor_by_device_kind_and_jitter(monkeypatch):
    """No processes: the derived floor is 0.2 s for an all-GPU replica, 0.75 s with any CPU stage, at
    least 8 x the measured period jitter, and exactly hang_min_s when the user passes one."""
    from types import SimpleNamespace
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd import dispatcher as dmod
    d = DEFER(membership_port=0, result_port=0, transport="tcp")
    try:
        d.replicas[0] = SimpleNamespace(records=[{"device": "cuda:0"}, {"device": "cuda:1"}], epoch=3)
        d.replicas[1] = SimpleNamespace(records=[{"device": "cuda:0"}, {"device": "cpu"}], epoch=3)
        assert d.hang_floor(0) == DEFER.HANG_GPU_MIN_S
        assert d.hang_floor(1) == DEFER.HANG_CPU_MIN_S
        # completions of replica 0, epoch 3: steady 10 ms intervals, then alternating 10 / 90 ms
        clock = [100.0]
        monkeypatch.setattr(dmod.time, "time", lambda: clock[0])
        for i in range(40):
            clock[0] += 0.010 if (i < 10 or i % 2) else 0.090
            d._note_done(0, 3, busy=True)
        monkeypatch.undo()
        jit = d._rep_jitter[0][1]
        assert jit > 0.02
        assert abs(d.hang_floor(0, 3) - max(DEFER.HANG_GPU_MIN_S, DEFER.HANG_JITTER_X * jit)) < 1e-12
        assert d.hang_floor(0, 4) == DEFER.HANG_GPU_MIN_S           # another epoch's jitter does not count
        assert d.hang_threshold(0, 3) >= d.hang_floor(0, 3)
        d.hang_min_s = 0.3
        assert d.hang_floor(0, 3) == 0.3 and d.hang_floor(1) == 0.3
    finally:
        d.replicas.clear()                  # stand-ins, not pipelines: nothing for shutdown to stop
        d.shutdown()
