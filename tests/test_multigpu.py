"""Multi-GPU data plane: RCCL point-to-point over xGMI between stage processes,
one per MI355X (BASELINE configs 2-4; the reference's layer-partitioned chain,
`src/dispatcher.py:39-53`, `src/node.py:163-179`).

Each test is gated on the number of visible GPUs and skips cleanly below it;
the gloo rehearsal at the top runs the same checker with two ranks sharing the
one GPU of a 1-GPU box.  Ranks are separate processes (parallel/launch.py), so
this pytest process never initialises RCCL itself.
"""
import json
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


def needs(n):
    return pytest.mark.skipif(_ndev() < n, reason=f"needs {n} GPUs, {_ndev()} visible")


def _check(*args, timeout=600):
    env = dict(os.environ, PYTHONPATH=ROOT, HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    r = subprocess.run([sys.executable, "-m", f"{PKG}.parallel.check", *args], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    recs = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r, recs


def test_pipeline_check_gloo_rehearsal():
    """The multi-GPU checker itself, two ranks on one GPU (host-staged links)."""
    r, recs = _check("--gpus", "2", "--backend", "gloo", "--part-at", "conv3_block1_1_conv", "--batch", "4")
    assert r.returncode == 0, r.stderr[-3000:]
    assert recs and recs[-1]["ok"] and recs[-1]["part_at"] == ["conv3_block1_1_conv"]


@needs(2)
def test_rccl_two_stage_multi_tensor_cut_matches_unsliced():
    """BASELINE config 2: part_at=['conv3_block1_1_conv'] (a two-tensor frontier)."""
    r, recs = _check("--gpus", "2", "--part-at", "conv3_block1_1_conv")
    assert r.returncode == 0, r.stderr[-3000:]
    assert recs[-1]["ok"] and recs[-1]["stages"] == 2


@needs(2)
def test_rccl_p2p_bandwidth():
    import tempfile
    out = os.path.join(tempfile.mkdtemp(), "p2p_bw.json")
    r, recs = _check("--gpus", "2", "--p2p-bw", "--out", out)
    assert r.returncode == 0, r.stderr[-3000:]
    assert recs and recs[0]["link_bw"] > 1e9


@needs(4)
def test_rccl_four_stage_planner_cuts():
    r, recs = _check("--gpus", "4")
    assert r.returncode == 0, r.stderr[-3000:]
    assert recs[-1]["ok"] and len(recs[-1]["part_at"]) == 3


@needs(8)
def test_rccl_eight_stage_lz4_links():
    """BASELINE config 3: 8 stages, frontier LZ4-compressed on a side stream."""
    r, recs = _check("--gpus", "8", "--codec", "lz4")
    assert r.returncode == 0, r.stderr[-3000:]
    assert recs[-1]["ok"] and recs[-1]["codec"] == "lz4"


def _spawn_gpu_worker(port, wid, dev):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="4", HSA_ENABLE_IPC_MODE_LEGACY="0")
    return subprocess.Popen([sys.executable, "-m", f"{PKG}.node", "--membership-port", str(port), "--data-port", "0",
                             "--config-port", "0", "--device", dev, "--id", wid, "--ttl", "1.0"],
                            env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, start_new_session=True)


def _kill(procs):
    for p in procs:
        try:
            os.killpg(p.pid, signal.SIGKILL)
        except ProcessLookupError:
            pass
        p.wait(timeout=30)


@needs(2)
def test_defer_rccl_two_gpu_workers():
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.dispatcher import DEFER
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.model import resnet
    m = resnet("resnet50", seed=0)
    d = DEFER(membership_port=0, result_port=0, worker_wait=120, batch=4, ordered=True, weight_codec="lz4",
              transport="rccl", min_workers=2, replicas=1)
    d.membership_server.start()
    procs = [_spawn_gpu_worker(d.membership_port, f"x{i}", f"cuda:{i}") for i in range(2)]
    try:
        inq, outq = queue.Queue(), queue.Queue()
        threading.Thread(target=d.run_defer, args=(m, ["conv3_block1_1_conv"], inq, outq), daemon=True).start()
        rng = np.random.default_rng(0)
        xs = [rng.standard_normal((4, 224, 224, 3)).astype(np.float32) for _ in range(3)]
        for x in xs:
            inq.put(x)
        got = np.concatenate([outq.get(timeout=300) for _ in xs])
        want = m.predict(np.concatenate(xs), device="cpu")
        assert np.abs(got - want).sum(-1).max() < 0.1
        assert len(d.pipeline.workers) == 2
    finally:
        d.shutdown(stop_workers=True)
        _kill(procs)


@needs(3)
def test_rccl_sigkill_exactly_once():
    """BASELINE config 4 on RCCL links: SIGKILL the middle stage; the survivors
    form a new epoch (fresh communicator) and every request is answered once."""
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.dispatcher import DEFER
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.model import resnet
    m = resnet("resnet50", seed=0)
    d = DEFER(membership_port=0, result_port=0, worker_wait=120, batch=4, max_inflight=4, weight_codec="lz4",
              transport="rccl", min_workers=3, replicas=1, task_timeout=60)
    d.membership_server.start()
    procs = [_spawn_gpu_worker(d.membership_port, f"k{i}", f"cuda:{i}") for i in range(3)]
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
        os.killpg(procs[int(victim[1:])].pid, signal.SIGKILL)
        while len(res) < n_req:
            res.append(outq.get(timeout=300))
        time.sleep(0.5)
        assert outq.empty()
        for y in res:
            assert np.abs(y - want).sum(-1).max() < 0.1
        assert victim not in d.pipeline.workers and d.recoveries
    finally:
        d.shutdown(stop_workers=True)
        _kill(procs)


@needs(3)
def test_rccl_hung_stage_detected_and_replayed_exactly_once():
    """The RCCL twin of tests/test_hang_detect.py: the middle stage's compute
    loop wedges while its process and heartbeats stay alive.  Its neighbours'
    RCCL kernels would spin until `abort()`; the dispatcher's progress watch
    must find the stage, abort the epoch's communicators, re-form on the two
    survivors (a fresh communicator) and replay every request exactly once
    (`src/dispatcher.py:186-194,302-304`: the reference's watchdog contract)."""
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.dispatcher import DEFER
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.model import resnet
    m = resnet("resnet50", seed=0)
    d = DEFER(membership_port=0, result_port=0, worker_wait=120, batch=4, max_inflight=4, weight_codec="lz4",
              transport="rccl", min_workers=3, replicas=1, task_timeout=60, hang_min_s=0.3, hang_factor=20)
    d.membership_server.start()
    procs = [_spawn_gpu_worker(d.membership_port, f"h{i}", f"cuda:{i}") for i in range(3)]
    stop = threading.Event()
    try:
        inq, outq = queue.Queue(8), queue.Queue()
        threading.Thread(target=d.run_defer, args=(m, ["conv3_block1_out", "conv4_block1_out"], inq, outq),
                         daemon=True).start()
        x = np.random.default_rng(2).standard_normal((4, 224, 224, 3)).astype(np.float32)
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
        res = [outq.get(timeout=300) for _ in range(30)]
        assert d.epoch_transport(d.pipeline.records) == "rccl"
        victim = d.pipeline.workers[1]
        t_hang = time.time()
        d.inject_fault(victim, "hang")
        t_end = time.time() + 60
        while not d.recoveries and time.time() < t_end:
            try:
                res.append(outq.get(timeout=0.05))
            except queue.Empty:
                pass
        assert d.hangs and d.hangs[0]["worker"] == victim, d.events[-6:]
        print(f"rccl: hung stage detected {(d.hangs[0]['t'] - t_hang) * 1e3:.0f} ms after the hang")
        for _ in range(10):
            res.append(outq.get(timeout=300))
        stop.set()
        feed.join()
        d.inject_fault(victim, "clear")
        total = sent[0]                      # queued inputs are consumed too
        while len(res) < total:
            res.append(outq.get(timeout=300))
        time.sleep(0.5)
        assert outq.empty() and len(res) == total
        for y in res:
            assert np.abs(y - want).sum(-1).max() < 0.1
        assert victim not in d.pipeline.workers and len(d.pipeline.workers) == 2
    finally:
        stop.set()
        d.shutdown(stop_workers=True)
        _kill(procs)


@needs(2)
def test_bench_fault_subrun_one_worker_per_gpu():
    """bench.py's config-4 sub-run at its real setting: one DEFER worker per GPU,
    transport auto -> RCCL p2p, middle worker SIGKILLed, exactly once."""
    n = min(_ndev(), 4)
    env = dict(os.environ, PYTHONPATH=ROOT, HSA_ENABLE_IPC_MODE_LEGACY="0")
    out = os.path.join("/tmp", f"fault_sub_{os.getpid()}.json")
    r = subprocess.run([sys.executable, "-m", f"{PKG}.parallel.fault_run", "--workers", str(n), "--devices", "each",
                        "--model", "resnet50", "--image", "224", "--batch", "32", "--duration", "8",
                        "--kill-at", "3", "--json", out], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.load(open(out))
    assert rec["epoch_transport"] == "rccl" and rec["exactly_once"] and rec["ok"], rec
