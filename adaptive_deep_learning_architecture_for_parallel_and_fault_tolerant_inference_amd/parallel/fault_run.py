"""Fault-injection run (BASELINE.json config 4: "8-stage with one worker killed
mid-run"), usable as a library call, a CLI and a `bench.py` sub-run.

A DEFER dispatcher (this process, which never touches a GPU) and N worker
processes (`python -m <pkg>.node`, one per GPU with ``devices="each"``) serve a
bs=32 request stream.  At `kill_at` seconds the worker holding the middle stage
is SIGKILLed (``fault="kill"``) or wedged (``fault="hang"``: its compute loop
stops while its process and heartbeats keep running).  Reported:

* ``detect_ms``: kill -> the dispatcher's first failure verdict (native UDP
  heartbeat silence, session EOF, lease expiry or the progress watch);
* ``reconfigure_ms``: the new epoch formed on the survivors (re-plan, configure,
  communicator rendezvous);
* ``value`` = recovery-to-steady ms: kill -> the END of the first 0.5 s sliding
  window after the kill whose throughput is >= 95 % of the post-recovery steady
  state; ``ready_ms`` (kill -> the new epoch serving) and
  ``window_start_ms`` are reported beside it;
* ``exactly_once``: every request answered once, none lost or duplicated.

Everything runs at the DEFER defaults (fp32, ``transport="auto"``: RCCL p2p when
every stage has its own GPU, heartbeat timeout 0.25 s) unless overridden.

The reference only tracks in-flight tasks with a start time for a watchdog it
never defines (`src/dispatcher.py:186-194,302-304`); see SURVEY §5.3.
"""
from __future__ import annotations

import argparse
import json
import os
import queue
import signal
import subprocess
import sys
import threading
import time
from typing import List, Optional

import numpy as np

PKG = (__package__ or "adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.parallel").rsplit(".", 1)[0]
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def worker_devices(devices: str, n: int) -> List[str]:
    """``"each"``: worker i on cuda:(i mod visible GPUs) (one per GPU when there
    are enough; the count is read without initialising HIP); ``"cpu"``; a single
    device for all; or a comma list."""
    if devices == "each":
        import torch
        ndev = torch.cuda.device_count()
        if ndev == 0:
            return ["cpu"] * n
        return [f"cuda:{i % ndev}" for i in range(n)]
    parts = [d for d in devices.split(",") if d]
    if len(parts) == 1:
        return parts * n
    if len(parts) != n:
        raise ValueError(f"{len(parts)} devices for {n} workers")
    return parts


def run(workers: int = 4, devices: str = "cpu", model: str = "resnet_tiny", image: int = 64, batch: int = 1,
        duration: float = 12.0, kill_at: float = 5.0, ttl: float = 0.5, inflight: int = 8,
        transport: str = "auto", codec: str = "none", replicas: str = "1", links: str = "auto",
        fault: str = "kill", hb_timeout: Optional[float] = None, precision: Optional[str] = None,
        ready_timeout: float = 150.0, log=None) -> dict:
    from ..dispatcher import DEFER
    from ..graph.planner import plan_cuts
    from ..models.model import resnet

    from ..utils.telemetry import PhaseStamps
    st = PhaseStamps("fault_run", stream=log if log is not None else open(os.devnull, "w"))

    def say(msg):
        if log is not None:
            print(f"fault_run: {msg}", file=log, flush=True)

    t_start = time.time()
    kw = {"input_shape": (image, image, 3)}
    if model == "resnet_tiny":
        kw["classes"] = 10
    m = resnet(model, seed=0, **kw)
    cuts, _ = plan_cuts(m.graph, workers, batch=batch, precision=precision or "fp32")
    dkw = {}
    if hb_timeout is not None:
        dkw["hb_timeout"] = hb_timeout
    if precision is not None:
        dkw["precision"] = precision
    d = DEFER(membership_port=0, result_port=0, worker_wait=120, batch=batch, codec=codec, weight_codec="lz4",
              max_inflight=inflight, task_timeout=30, min_workers=workers, transport=transport,
              replicas=replicas, links=links, **dkw)
    d.membership_server.start()
    st.stamp("dispatcher_up", port=d.membership_port)
    devs = worker_devices(devices, workers)
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""), OMP_NUM_THREADS="1")
    import tempfile
    logdir = tempfile.mkdtemp(prefix="fault_run_")
    procs = {}
    logs = {}
    for i in range(workers):
        wid = f"w{i}"
        logs[wid] = open(os.path.join(logdir, f"{wid}.log"), "w")       # a worker that dies early says why
        procs[wid] = subprocess.Popen(
            [sys.executable, "-m", f"{PKG}.node", "--membership-port", str(d.membership_port), "--data-port", "0",
             "--config-port", "0", "--device", devs[i], "--id", wid, "--ttl", str(ttl), "--parent-pid", str(os.getpid())],
            env=env, stdout=subprocess.DEVNULL, stderr=logs[wid], start_new_session=True)
    st.stamp("workers_spawned", devices=",".join(devs))

    def worker_tails(n=300):
        out = {}
        for wid, f in logs.items():
            f.flush()
            try:
                with open(f.name) as g:
                    txt = g.read().strip()
            except OSError:
                txt = ""
            if txt:
                out[wid] = txt[-n:]
        return out
    inq, outq = queue.Queue(inflight), queue.Queue()
    threading.Thread(target=d.run_defer, args=(m, cuts, inq, outq), daemon=True).start()
    x = np.random.default_rng(0).standard_normal((batch, image, image, 3)).astype(np.float32)
    stop = threading.Event()
    sent = [0]

    def feeder():
        while not stop.is_set():
            try:
                inq.put(x, timeout=0.1)
                sent[0] += 1
            except queue.Full:
                continue

    got = 0
    t0 = t_kill = None
    victim = None
    epoch_transport = None
    try:
        # the pipeline must be up, and the whole model resident on every worker
        # (background push after the first epoch), before the clock starts
        deadline = time.time() + ready_timeout
        while d.pipeline is None and time.time() < deadline:
            time.sleep(0.05)
        if d.pipeline is None:
            raise RuntimeError(f"no pipeline formed within {ready_timeout:.0f} s; events {d.events[-3:]}; "
                               f"worker stderr {worker_tails()}")
        epoch_transport = d.epoch_transport(d.pipeline.records)
        st.stamp("pipeline_up", stages=len(d.pipeline.workers), transport=epoch_transport)
        say(f"pipeline up after {time.time() - t_start:.1f} s: {len(d.pipeline.workers)} stages, "
            f"transport {epoch_transport}")
        while time.time() < deadline and sum(1 for v in d._resident.values() if v) < workers:
            time.sleep(0.1)
        st.stamp("models_resident")
        time.sleep(d.prepare_delay + 1.5)   # prepare hints: next plans' slices built in the background
        threading.Thread(target=feeder, daemon=True).start()
        t0 = time.time()
        st.stamp("feeding")
        while time.time() - t0 < duration:
            if t_kill is None and time.time() - t0 >= kill_at:
                victim = d.pipeline.workers[len(d.pipeline.workers) // 2]
                if fault == "kill":
                    os.killpg(procs[victim].pid, signal.SIGKILL)
                else:
                    d.inject_fault(victim, "hang")
                t_kill = time.time()
                st.stamp(fault, victim=victim)
                say(f"{fault} {victim} at t={t_kill - t0:.2f} s")
            try:
                outq.get(timeout=0.1)
                got += 1
            except queue.Empty:
                pass
        stop.set()
        st.stamp("window_done", results=got, recoveries=len(d.recoveries))
        # drain: every request sent must come back exactly once
        deadline = time.time() + 60
        while got < sent[0] - inq.qsize() and time.time() < deadline:
            try:
                outq.get(timeout=0.5)
                got += 1
            except queue.Empty:
                pass
        st.stamp("drained", results=got, sent=sent[0])
    finally:
        stop.set()
        d.shutdown(stop_workers=True)
        for p in procs.values():
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
        for p in procs.values():
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                pass
        for f in logs.values():
            f.close()
        st.stamp("teardown")
    ts = np.array(d.completion_times)
    pre = ts[(ts > t0 + 1.0) & (ts < t_kill)] if t_kill else ts
    rate_pre = len(pre) / max(1e-9, (t_kill - t0 - 1.0)) * batch if t_kill else None
    rec = d.recoveries[0] if d.recoveries else None
    wins = d.recovery_windows(t_kill=t_kill) if t_kill else []
    rts = [w["end_ms"] for w in wins]
    post = ts[ts > (rec["t_ready"] + 1.0)] if rec else np.array([])
    rate_post = (len(post) - 1) / (post[-1] - post[0]) * batch if len(post) > 2 else None
    answered = sent[0] - inq.qsize()
    out = {
        "metric": f"recovery-to-steady ms after a worker {'kill' if fault == 'kill' else 'hang'}",
        "value": round(rts[0], 1) if rts else None, "unit": "ms",
        "ok": bool(rts) and got == answered,
        "fault": fault, "hangs": d.hangs,
        "workers": workers, "devices": devs, "transport": transport, "epoch_transport": epoch_transport,
        "precision": d.precision, "hb_timeout": d.hb_timeout, "model": model, "batch": batch,
        "cuts_before": cuts, "cuts_after": d.pipeline.part_at if d.pipeline else None, "victim": victim,
        "ready_ms": round((rec["t_ready"] - t_kill) * 1e3, 1) if rec and t_kill else None,
        "window_start_ms": round(wins[0]["start_ms"], 1) if wins else None,
        "detect_ms": round((rec["t_fail"] - t_kill) * 1e3, 1) if rec and t_kill else None,
        "reconfigure_ms": round(rec["reconfig_ms"], 1) if rec else None,
        "replayed": rec["replayed"] if rec else None,
        "throughput_before_img_s": round(rate_pre, 1) if rate_pre else None,
        "throughput_after_img_s": round(rate_post, 1) if rate_post else None,
        "requests_sent": sent[0], "results": got, "duplicates_dropped": d.duplicates_dropped,
        "exactly_once": got == answered,
        "detected_by": next((e for t, e in d.events if t_kill and t > t_kill), None),
        "events": [(round(t - (t0 or t_start), 3), e) for t, e in d.events],
        "wall_s": round(time.time() - t_start, 1),
        "phases": dict(st.phases),
    }
    want = expected_transport(transport, devs)
    if want is not None and epoch_transport is not None and epoch_transport != want:
        # one worker per GPU at transport "auto" must run its hops over RCCL p2p, not a fallback
        out["ok"] = False
        out["error"] = f"epoch transport {epoch_transport!r}, expected {want!r} with devices {devs}"
    return out


def expected_transport(transport: str, devs: List[str]) -> Optional[str]:
    """The stage -> stage transport DEFER must pick for these workers: "rccl" when
    transport is "auto" and every worker has a GPU of its own (one process per
    MI355X); None when the run does not pin it."""
    if transport != "auto" or len(devs) < 2:
        return None
    if all(d.startswith("cuda") for d in devs) and len(set(devs)) == len(devs):
        return "rccl"
    return None


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--model", default="resnet_tiny")
    ap.add_argument("--image", type=int, default=64)
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--device", "--devices", dest="devices", default="cpu",
                    help="cpu | cuda:0 (all workers share it) | each (worker i on GPU i) | comma list")
    ap.add_argument("--transport", default="auto", choices=["auto", "tcp", "rccl", "gloo"])
    ap.add_argument("--codec", default="none")
    ap.add_argument("--replicas", default="1", help="pipeline replicas (auto or N)")
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--duration", type=float, default=12.0)
    ap.add_argument("--kill-at", type=float, default=5.0)
    ap.add_argument("--ttl", type=float, default=0.5)
    ap.add_argument("--inflight", type=int, default=8)
    ap.add_argument("--links", default="auto", choices=["auto", "dev", "shm", "tcp"],
                    help="same-host stage->stage hops of the tcp transport (DEFER links)")
    ap.add_argument("--fault", default="kill", choices=["kill", "hang"])
    ap.add_argument("--hb-timeout", type=float, default=None,
                    help="heartbeat silence that counts as death (default: DEFER's, 0.25 s)")
    ap.add_argument("--precision", default=None, choices=[None, "fp32", "bf16"],
                    help="worker precision (default: DEFER's, fp32)")
    ap.add_argument("--ready-timeout", type=float, default=150.0)
    ap.add_argument("--json", default="")
    return ap.parse_args(argv)


def _terminate(signum, frame):
    # a parent's time limit (bench.py run_subrun) sends SIGTERM: unwind through run()'s `finally`, which
    # shuts the dispatcher down and kills the worker process groups (they run in sessions of their own)
    raise SystemExit(128 + signum)


def main(argv=None) -> int:
    signal.signal(signal.SIGTERM, _terminate)
    from ..utils.telemetry import PhaseStamps
    # bench.py's sub-run limit: a hang dumps every thread's stack 10 s before it
    PhaseStamps.arm_faulthandler(float(os.environ.get("ADAPT_SUB_LIMIT_S", "0") or 0))
    a = parse(argv)
    out = run(workers=a.workers, devices=a.devices, model=a.model, image=a.image, batch=a.batch,
              duration=a.duration, kill_at=a.kill_at, ttl=a.ttl, inflight=a.inflight, transport=a.transport,
              codec=a.codec, replicas=a.replicas, links=a.links, fault=a.fault, hb_timeout=a.hb_timeout,
              precision=a.precision, ready_timeout=a.ready_timeout, log=sys.stderr)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)
    else:
        print(json.dumps(out, indent=1))
    return 0


if __name__ == "__main__":
    rc = main()
    sys.stdout.flush()
    sys.stderr.flush()
    os._exit(rc)        # daemon I/O threads may sit in native recv(); skip finalization
