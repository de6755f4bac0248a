#!/usr/bin/env python3
"""Fault-injection benchmark (BASELINE.json config 4: "8-stage with one worker
killed mid-run"): start a dispatcher and N worker processes, stream requests,
SIGKILL (``--fault kill``) or wedge (``--fault hang``: its compute loop stops,
its process and heartbeats keep running) the worker holding the middle stage
at --kill-at seconds, and report

* detection latency (kill -> lease expiry seen by the dispatcher),
* reconfiguration time (new epoch formed on the survivors),
* recovery-to-steady ms: kill -> first 0.5 s window whose throughput is >= 95%
  of the post-recovery steady state,
* exactly-once check: every request answered once, none lost.

    python tools/fault_bench.py --workers 4 --device cpu --model resnet_tiny
    python tools/fault_bench.py --workers 4 --device cuda:0 --batch 32     # GPU box (workers share the GPU)
"""
import argparse
import json
import os
import queue
import signal
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.dispatcher import DEFER  # noqa: E402
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.graph.planner import plan_cuts  # noqa: E402
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.model import resnet  # noqa: E402

PKG = "adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet_tiny")
    ap.add_argument("--image", type=int, default=64)
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--transport", default="tcp")
    ap.add_argument("--codec", default="none")
    ap.add_argument("--replicas", default="1", help="pipeline replicas (auto or N)")
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--duration", type=float, default=12.0)
    ap.add_argument("--kill-at", type=float, default=5.0)
    ap.add_argument("--ttl", type=float, default=0.5)
    ap.add_argument("--inflight", type=int, default=8)
    ap.add_argument("--links", default="auto", choices=["auto", "dev", "shm", "tcp"],
                    help="same-host stage->stage hops (DEFER links)")
    ap.add_argument("--fault", default="kill", choices=["kill", "hang"])
    ap.add_argument("--hb-timeout", type=float, default=0.06,
                    help="heartbeat silence that counts as death (DEFER default 0.25)")
    ap.add_argument("--json", default="")
    a = ap.parse_args()

    m = resnet(a.model, seed=0, input_shape=(a.image, a.image, 3))
    cuts, _ = plan_cuts(m.graph, a.workers, batch=a.batch)
    d = DEFER(membership_port=0, result_port=0, worker_wait=120, batch=a.batch, codec=a.codec, weight_codec="lz4",
              max_inflight=a.inflight, task_timeout=30, min_workers=a.workers, transport=a.transport,
              replicas=a.replicas, links=a.links, hb_timeout=a.hb_timeout)
    d.membership_server.start()
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    procs = {}
    for i in range(a.workers):
        wid = f"w{i}"
        procs[wid] = subprocess.Popen(
            [sys.executable, "-m", f"{PKG}.node", "--membership-port", str(d.membership_port), "--data-port", "0",
             "--config-port", "0", "--device", a.device, "--id", wid, "--ttl", str(a.ttl)],
            env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, start_new_session=True)
    inq, outq = queue.Queue(a.inflight), queue.Queue()
    threading.Thread(target=d.run_defer, args=(m, cuts, inq, outq), daemon=True).start()
    x = np.random.default_rng(0).standard_normal((a.batch, a.image, a.image, 3)).astype(np.float32)
    stop = threading.Event()
    sent = [0]

    def feeder():
        while not stop.is_set():
            try:
                inq.put(x, timeout=0.1)
                sent[0] += 1
            except queue.Full:
                continue

    # wait for the pipeline to come up, and for the whole model to be resident on
    # every worker (background push after the first epoch), before the clock starts
    while d.pipeline is None:
        time.sleep(0.05)
    deadline = time.time() + 120
    while time.time() < deadline and sum(1 for v in d._resident.values() if v) < a.workers:
        time.sleep(0.1)
    time.sleep(d.prepare_delay + 1.5)   # prepare hints: next plans' slices built in the background
    threading.Thread(target=feeder, daemon=True).start()
    got = 0
    t0 = time.time()
    t_kill = None
    victim = None
    try:
        while time.time() - t0 < a.duration:
            if t_kill is None and time.time() - t0 >= a.kill_at:
                victim = d.pipeline.workers[len(d.pipeline.workers) // 2]
                if a.fault == "kill":
                    os.killpg(procs[victim].pid, signal.SIGKILL)
                else:
                    d.inject_fault(victim, "hang")
                t_kill = time.time()
            try:
                outq.get(timeout=0.1)
                got += 1
            except queue.Empty:
                pass
        stop.set()
        # drain: every request sent must come back exactly once
        deadline = time.time() + 60
        while got < sent[0] - inq.qsize() and time.time() < deadline:
            try:
                outq.get(timeout=0.5)
                got += 1
            except queue.Empty:
                pass
    finally:
        stop.set()
        d.shutdown(stop_workers=True)
        for p in procs.values():
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
    ts = np.array(d.completion_times)
    pre = ts[(ts > t0 + 1.0) & (ts < t_kill)] if t_kill else ts
    rate_pre = len(pre) / max(1e-9, (t_kill - t0 - 1.0)) * a.batch if t_kill else None
    rec = d.recoveries[0] if d.recoveries else None
    rts = d.recovery_to_steady_ms(t_kill=t_kill) if t_kill else []
    post = ts[ts > (rec["t_ready"] + 1.0)] if rec else np.array([])
    rate_post = (len(post) - 1) / (post[-1] - post[0]) * a.batch if len(post) > 2 else None
    out = {
        "metric": f"recovery-to-steady ms after a worker {'kill' if a.fault == 'kill' else 'hang'}",
        "fault": a.fault, "hangs": d.hangs,
        "value": round(rts[0], 1) if rts else None,
        "unit": "ms",
        "workers": a.workers, "device": a.device, "transport": a.transport, "model": a.model, "batch": a.batch,
        "cuts_before": cuts, "cuts_after": d.pipeline.part_at if d.pipeline else None, "victim": victim,
        "detect_ms": round((rec["t_fail"] - t_kill) * 1e3, 1) if rec and t_kill else None,
        "reconfigure_ms": round(rec["reconfig_ms"], 1) if rec else None,
        "replayed": rec["replayed"] if rec else None,
        "throughput_before_img_s": rate_pre, "throughput_after_img_s": rate_post,
        "requests_sent": sent[0], "results": got, "duplicates_dropped": d.duplicates_dropped,
        "exactly_once": got == sent[0] - inq.qsize(),
        "detected_by": next((e for _, e in d.events if t_kill and _ > t_kill), None),
        "events": [(round(t - t0, 3), e) for t, e in d.events],
    }
    print(json.dumps(out, indent=1))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
    sys.stdout.flush()
    os._exit(0)        # daemon I/O threads may sit in native recv(); skip finalization
