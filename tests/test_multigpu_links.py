"""The DEFER data plane's same-host links across MI355X devices, with a
same-device twin of each test that runs on the 1-GPU box.

* device links (`links=dev`): the stage -> stage hop is an IPC-exported device
  slot; across GPUs the receiver enables peer access to the exporter's device
  and copies over xGMI (transport/shm.py DeviceLinkPool, `ipc_open(handle, peer)`);
* BASELINE config 5: ResNet-152 bf16 as a 4-stage DEFER pipeline, checked
  against an unsliced forward (probabilities L1, top-1);
* BASELINE config 4 on device links: SIGKILL a middle stage, every request is
  answered exactly once by the re-formed pipeline.

The reference's chain is `src/dispatcher.py:39-53,204-220` / `src/node.py:163-179`.
Workers are separate processes (`python -m <pkg>.node --device cuda:i`).
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
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = "adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd"
pytestmark = pytest.mark.gpu


def _ndev() -> int:
    try:
        return torch.cuda.device_count()
    except Exception:  # noqa: BLE001
        return 0


def _devices(kind: str, n: int):
    """n worker devices: all cuda:0 ("same", the 1-GPU twin) or distinct GPUs ("cross")."""
    if kind == "cross":
        if _ndev() < n:
            pytest.skip(f"needs {n} GPUs, {_ndev()} visible")
        return [f"cuda:{i}" for i in range(n)]
    return ["cuda:0"] * n


def _spawn(port, wid, dev, ttl="2.0"):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="4", HSA_ENABLE_IPC_MODE_LEGACY="0")
    return subprocess.Popen([sys.executable, "-m", f"{PKG}.node", "--membership-port", str(port), "--data-port", "0",
                             "--config-port", "0", "--device", dev, "--id", wid, "--ttl", ttl],
                            env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, start_new_session=True)


def _kill(procs):
    for p in procs:
        try:
            os.killpg(p.pid, signal.SIGKILL)
        except ProcessLookupError:
            pass
    for p in procs:
        try:
            p.wait(timeout=30)
        except subprocess.TimeoutExpired:
            pass


@pytest.mark.parametrize("kind", ["same", "cross"])
def test_device_link_two_workers(kind):
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.dispatcher import DEFER
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.model import resnet
    devs = _devices(kind, 2)
    m = resnet("resnet50", seed=0)
    d = DEFER(membership_port=0, result_port=0, worker_wait=120, batch=4, ordered=True, weight_codec="lz4",
              min_workers=2, links="dev", replicas=1)
    d.membership_server.start()
    procs = [_spawn(d.membership_port, f"l{i}", dv) for i, dv in enumerate(devs)]
    try:
        inq, outq = queue.Queue(), queue.Queue()
        threading.Thread(target=d.run_defer, args=(m, ["conv3_block1_1_conv"], inq, outq), daemon=True).start()
        rng = np.random.default_rng(6)
        xs = [rng.standard_normal((4, 224, 224, 3)).astype(np.float32) for _ in range(8)]
        for x in xs:
            inq.put(x)
        got = np.concatenate([outq.get(timeout=240) for _ in xs])
        want = m.predict(np.concatenate(xs), device="cpu")
        assert np.abs(got - want).sum(-1).max() < 0.1
        assert any("links=dev" in ev for _, ev in d.events), d.events
        assert not d.recoveries, d.events
    finally:
        d.shutdown(stop_workers=True)
        _kill(procs)


@pytest.mark.parametrize("kind", ["same", "cross"])
def test_resnet152_bf16_four_stage_defer_matches_unsliced(kind):
    """BASELINE config 5: ResNet-152 bf16, 4 stages (planner cuts), device links."""
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.dispatcher import DEFER
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.graph.planner import plan_cuts
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.model import resnet
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.runtime.executor import (
        SliceExecutor)
    devs = _devices(kind, 4)
    m = resnet("resnet152", seed=0)
    cuts, _ = plan_cuts(m.graph, 4, batch=8)
    d = DEFER(membership_port=0, result_port=0, worker_wait=240, batch=8, ordered=True, weight_codec="lz4",
              min_workers=4, links="dev", replicas=1, precision="bf16")
    d.membership_server.start()
    procs = [_spawn(d.membership_port, f"r{i}", dv) for i, dv in enumerate(devs)]
    try:
        inq, outq = queue.Queue(), queue.Queue()
        threading.Thread(target=d.run_defer, args=(m, cuts, inq, outq), daemon=True).start()
        rng = np.random.default_rng(9)
        xs = [rng.standard_normal((8, 224, 224, 3)).astype(np.float32) for _ in range(4)]
        for x in xs:
            inq.put(x)
        got = np.concatenate([outq.get(timeout=300) for _ in xs])
        full = SliceExecutor(m.graph, m.weights, batch=8, device="cuda:0", precision="bf16")
        want = np.concatenate([full(torch.from_numpy(x).cuda()).float().cpu().numpy() for x in xs])
        l1 = np.abs(got - want).sum(-1).max()
        top1 = (got.argmax(-1) == want.argmax(-1)).mean()
        print(f"resnet152 4-stage DEFER ({kind}): cuts {cuts}, L1 {l1:.3e}, top-1 agreement {top1:.3f}")
        assert len(d.pipeline.workers) == 4 and d.pipeline.part_at == list(cuts)
        assert l1 < 0.05 and top1 >= 0.97
    finally:
        d.shutdown(stop_workers=True)
        _kill(procs)


@pytest.mark.parametrize("kind", ["same", "cross"])
def test_device_link_sigkill_exactly_once(kind):
    """BASELINE config 4 on device links: SIGKILL the middle of three stages; the
    survivors form a new epoch and every request is answered exactly once."""
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.dispatcher import DEFER
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.model import resnet
    devs = _devices(kind, 3)
    m = resnet("resnet50", seed=0)
    d = DEFER(membership_port=0, result_port=0, worker_wait=120, batch=4, max_inflight=4, weight_codec="lz4",
              min_workers=3, links="dev", replicas=1, task_timeout=60)
    d.membership_server.start()
    procs = {f"k{i}": _spawn(d.membership_port, f"k{i}", dv, ttl="1.0") for i, dv in enumerate(devs)}
    try:
        inq, outq = queue.Queue(), queue.Queue()
        threading.Thread(target=d.run_defer, args=(m, ["conv3_block1_out", "conv4_block1_out"], inq, outq),
                         daemon=True).start()
        x = np.random.default_rng(1).standard_normal((4, 224, 224, 3)).astype(np.float32)
        want = m.predict(x, device="cpu")
        n_req = 24

        def feeder():
            for _ in range(n_req):
                inq.put(x)
                time.sleep(0.02)

        threading.Thread(target=feeder, daemon=True).start()
        res = [outq.get(timeout=300) for _ in range(6)]
        victim = d.pipeline.workers[1]
        os.killpg(procs[victim].pid, signal.SIGKILL)
        while len(res) < n_req:
            res.append(outq.get(timeout=300))
        time.sleep(0.5)
        assert outq.empty()
        for y in res:
            assert np.abs(y - want).sum(-1).max() < 0.1
        assert victim not in d.pipeline.workers and d.recoveries
        print(f"device-link SIGKILL ({kind}): {n_req} answered once, recoveries {len(d.recoveries)}, "
              f"duplicates dropped {d.duplicates_dropped}")
    finally:
        d.shutdown(stop_workers=True)
        _kill(list(procs.values()))
