"""The RCCL branch of the stage data plane, end to end on ONE GPU.

`DEFER(transport="rccl")` makes every epoch's stages talk through `EpochGroup(backend="nccl")` ->
`PairLinks` -> `CollectiveStageRuntime._data_loop` (the non-staged, device-ordered path: grouped
meta + frontier enqueues on link streams, waits ordered on the device).  RCCL itself refuses two ranks
on one device, so the worker processes here run with ``ADAPT_TEST_LOOPBACK_COMM=1``: the test-only
stand-in communicator (parallel/loopback_comm.py, csrc/kernels/loopback.hip) that moves each message
through an IPC-exported device ring with device-side waits, and whose abort releases pending waits.
Everything above the communicator -- epochs, per-epoch rendezvous, abort / re-form, replay -- is the
code the 8-GPU node runs.  Reference: the stage-to-stage hop `/root/reference/src/dispatcher.py:204-220`,
`src/node.py:163-179`; the in-flight registry and watchdog `src/dispatcher.py:186-194,302-304`."""
import glob
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

pytestmark = pytest.mark.gpu

PKG = "adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _workers(port, n, tag):
    env = dict(os.environ, ADAPT_TEST_LOOPBACK_COMM="1", ADAPT_LOOPBACK_SLOT_MB="16", ADAPT_EPOCH_TIMING="1",
               PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    return [subprocess.Popen([sys.executable, "-m", f"{PKG}.node", "--membership-port", str(port), "--data-port", "0",
                              "--config-port", "0", "--device", "cuda:0", "--id", f"{tag}{i}", "--ttl", "2.0",
                              "--parent-pid", str(os.getpid())], env=env, start_new_session=True)
            for i in range(n)]


def _stop(d, procs):
    d.shutdown(stop_workers=True)
    for p in procs:
        try:
            os.killpg(p.pid, signal.SIGTERM)
        except ProcessLookupError:
            pass
    for p in procs:
        try:
            p.wait(timeout=30)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait(timeout=10)
    for f in glob.glob("/dev/shm/adapt-lb-*"):
        try:
            os.unlink(f)
        except OSError:
            pass


@pytest.mark.parametrize("fault", ["none", "kill", "hang"])
def test_rccl_branch_over_loopback_links(fault):
    """Three GPU stage processes on cuda:0, transport "rccl": the steady pipeline matches the fp32 oracle;
    with a fault, the middle stage is SIGKILLed or wedged, the epoch's links are aborted (releasing the
    survivors' pending device waits), a new epoch re-forms on the two survivors with a fresh per-epoch
    rendezvous, and every request is answered exactly once."""
    m = resnet("resnet50", seed=0)
    d = DEFER(membership_port=0, result_port=0, worker_wait=120, batch=2, ordered=True, weight_codec="lz4",
              min_workers=3, max_inflight=4, transport="rccl", replicas=1)
    d.membership_server.start()
    procs = _workers(d.membership_port, 3, "lb")
    stop = threading.Event()
    try:
        inq, outq = queue.Queue(4), queue.Queue()
        threading.Thread(target=d.run_defer, args=(m, ["conv3_block1_out", "conv4_block3_out"], inq, outq),
                         daemon=True).start()
        x = np.random.default_rng(11).standard_normal((2, 224, 224, 3)).astype(np.float32)
        want = m.predict(x, device="cpu")
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
        res = [outq.get(timeout=240) for _ in range(20)]
        assert len(d.pipeline.workers) == 3
        if fault != "none":
            # let DEFER's background work finish first: the whole-model push to every worker and the `prepare`
            # hints (each survivor builds the slice it would take after a loss), as in a long-running job; the
            # re-form then pays the per-epoch link rendezvous, not a slice build
            t_end = time.time() + 120
            while any(t.is_alive() for t in d._bg) and time.time() < t_end:
                res.append(outq.get(timeout=240))
            t_end = time.time() + 4.0
            while time.time() < t_end:
                res.append(outq.get(timeout=240))
        assert d.epoch_transport(d.pipeline.records) == "rccl"
        assert glob.glob("/dev/shm/adapt-lb-*"), "the stage links are not the loopback communicator"
        for y in res:
            assert np.abs(y - want).sum(-1).max() < 0.1
        if fault != "none":
            victim = d.pipeline.workers[1]
            t_fault = time.time()
            if fault == "hang":
                d.inject_fault(victim, "hang")
            else:
                os.killpg(procs[int(victim[2:])].pid, signal.SIGKILL)
            t_end = time.time() + 90
            while not d.recoveries and time.time() < t_end:
                try:
                    res.append(outq.get(timeout=0.05))
                except queue.Empty:
                    pass
            assert d.recoveries, d.events[-8:]
            r = d.recoveries[0]
            detect_ms = (r["t_fail"] - t_fault) * 1e3
            ready_ms = (r["t_ready"] - t_fault) * 1e3
            print(f"rccl-branch {fault}: detect {detect_ms:.0f} ms, reconfigure {r['reconfig_ms']:.0f} ms "
                  f"(per-epoch link rendezvous included), ready {ready_ms:.0f} ms after the fault, "
                  f"replayed {r['replayed']}")
            if fault == "hang":
                assert d.hangs and d.hangs[0]["worker"] == victim, d.events[-8:]
            for t_ev, ev in d.events:
                if t_fault - 0.05 <= t_ev <= r["t_ready"] + 0.05:
                    print(f"  +{(t_ev - t_fault) * 1e3:7.1f} ms  {ev}")
            # 3 s of the re-formed pipeline: enough for the recovery window and its steady state
            while time.time() < r["t_ready"] + 3.0 or len(res) < 30:
                res.append(outq.get(timeout=240))
            assert victim not in d.pipeline.workers and len(d.pipeline.workers) == 2
            assert d.epoch_transport(d.pipeline.records) == "rccl"
            wins = d.recovery_windows(t_kill=t_fault)
            if wins:
                print(f"rccl-branch {fault}: recovery-to-steady {wins[0]['end_ms']:.0f} ms "
                      f"(first 0.5 s window at >= 95 % of the new steady state)")
            # where the time between ready and steady goes: completions per 100 ms from the fault on,
            # and the events after ready (re-captures, prepare builds, late reports)
            ts = np.array(d.completion_times)
            bins = [int(np.count_nonzero((ts > t_fault + k * 0.1) & (ts <= t_fault + (k + 1) * 0.1)))
                    for k in range(int((r["t_ready"] + 3.0 - t_fault) / 0.1))]
            print(f"rccl-branch {fault}: completions per 100 ms from the fault: {bins}")
            for t_ev, ev in d.events:
                if r["t_ready"] + 0.05 < t_ev <= r["t_ready"] + 3.0:
                    print(f"  +{(t_ev - t_fault) * 1e3:7.1f} ms  {ev}")
        stop.set()
        feed.join()
        if fault == "hang":
            d.inject_fault(d.hangs[0]["worker"], "clear")     # stale outputs of the woken stage must not leak
        time.sleep(0.5)
        total = sent[0]
        while len(res) < total:
            res.append(outq.get(timeout=240))
        time.sleep(0.5)
        assert outq.empty() and len(res) == total            # exactly once
        for y in res:
            assert np.abs(y - want).sum(-1).max() < 0.1
    finally:
        stop.set()
        _stop(d, procs)
