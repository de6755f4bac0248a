"""Command line: ``python -m adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd <cmd>``

The reference has no CLI: `bash src/start_etcd.sh`, `python -m src.node`
(edit the source for the dispatcher IP) and `python test/test.py` (edit the
worker list / cut list in the source) (`README.md:36-56`).  Subcommands:

  membership   run the membership service (etcd stand-in, port 2379)
  node         run a worker (one per GPU)
  serve        dispatcher + synthetic request stream, prints throughput
               (`test/test.py`); --spawn N starts N local workers
  local-infer  single-device throughput (`test/local_infer.py`)
  plan         balanced cut planner: cuts, per-stage cost, frontier bytes
  summary      model summary (layers, shapes, params)

--model takes a family name (resnet50/101/152, vgg16/19, mobilenet_v2,
densenet121/169/201) or a Keras ``model.to_json()`` file (*.json), with
--weights pointing at its ``get_weights()`` list saved as .npz.

All take --config FILE (YAML) plus ADAPT_* environment overrides (utils/config.py).
"""
from __future__ import annotations

import argparse
import os
import queue
import signal
import subprocess
import sys
import threading
import time

import numpy as np

from .utils.config import AdaptConfig

PKG = __package__


def _common(ap):
    ap.add_argument("--config", default=None, help="YAML config file")
    ap.add_argument("--model", default=None)
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--part-at", default=None, help="comma-separated cut layers or auto:K")


def _cfg(a, **extra) -> AdaptConfig:
    ov = {"model": a.model, "batch": a.batch, "part_at": a.part_at}
    ov.update(extra)
    return AdaptConfig.load(a.config, overrides=ov)


def _model(cfg: AdaptConfig):
    from .graph.manifest import load_keras_weight_list, load_model
    from .models.model import Model, resnet
    if cfg.model.endswith(".json"):
        # a Keras architecture (`model.to_json()`, what the reference ships to its workers);
        # weights: --weights <Keras get_weights() .npz>, else seeded random init
        with open(cfg.model) as f:
            m = Model.from_keras_json(f.read(), seed=cfg.seed)
    else:
        m = resnet(cfg.model, seed=cfg.seed, input_shape=tuple(cfg.image), classes=cfg.classes)
    if cfg.weights:
        if cfg.weights.endswith(".npz"):
            m.weights = load_keras_weight_list(m.graph, cfg.weights)
        else:
            g, w = load_model(cfg.weights)
            m = Model(g, w)
    return m


def cmd_membership(argv):
    from .membership.server import main
    main(argv)


def cmd_node(argv):
    from .node import main
    main(argv)


def cmd_serve(argv):
    ap = argparse.ArgumentParser(prog="serve")
    _common(ap)
    ap.add_argument("--requests", type=int, default=100)
    ap.add_argument("--spawn", type=int, default=0, help="start N local workers")
    ap.add_argument("--device", default=None, help="device for spawned workers (cpu, cuda, cuda:i)")
    ap.add_argument("--transport", default=None)
    ap.add_argument("--codec", default=None)
    ap.add_argument("--replicas", default=None, help="pipeline replicas: auto (live // stages) or N")
    ap.add_argument("--ingest", default="auto", choices=["auto", "tcp"],
                    help="auto: same-host shared-memory request slots; tcp: inline on the socket")
    ap.add_argument("--links", default="auto", choices=["auto", "dev", "shm", "tcp"],
                    help="stage->stage hops between workers on one host: auto = device-to-device IPC slots when "
                         "both are GPU workers, else page-locked shared-memory slots; shm = always host slots; "
                         "tcp = inline on the socket")
    ap.add_argument("--uint8", action="store_true", help="send uint8 images (4x fewer bytes), preprocessed on the GPU")
    ap.add_argument("--preprocess", default="none", choices=["none", "caffe", "tf", "torch"],
                    help="Keras preprocess_input mode applied by stage 0 to uint8 requests")
    ap.add_argument("--dtype", default="fp32", choices=["bf16", "fp32"],
                    help="worker compute precision (fp32 = the reference's Keras float32)")
    a = ap.parse_args(argv)
    cfg = _cfg(a, transport=a.transport, codec=a.codec, replicas=a.replicas)
    from .dispatcher import DEFER
    m = _model(cfg)
    cuts = cfg.cuts(m.graph, precision=a.dtype)
    d = DEFER(membership_port=cfg.membership_port, result_port=cfg.result_port, chunk_size=cfg.chunk_size,
              batch=cfg.batch, codec=cfg.codec, weight_codec=cfg.weight_codec, max_inflight=cfg.max_inflight,
              task_timeout=cfg.task_timeout, worker_wait=max(cfg.worker_wait, 60 if a.spawn else 0),
              elastic=cfg.elastic, ordered=cfg.ordered, transport=cfg.transport, min_workers=max(1, a.spawn),
              replicas=cfg.replicas, ingest=a.ingest, preprocess=a.preprocess, precision=a.dtype,
              links=a.links)
    d.membership_server.start()
    procs = []
    for i in range(a.spawn):
        dev = a.device or "cpu"
        if dev == "cuda":
            dev = f"cuda:{i}"
        procs.append(subprocess.Popen([sys.executable, "-m", f"{PKG}.node", "--membership-port",
                                       str(d.membership_port), "--data-port", "0", "--config-port", "0",
                                       "--device", dev, "--id", f"local{i}", "--ttl", str(cfg.lease_ttl),
                                       "--parent-pid", str(os.getpid())],
                                      start_new_session=True))
    inq, outq = queue.Queue(cfg.max_inflight * 2), queue.Queue()
    rng = np.random.default_rng(cfg.seed)
    if a.uint8:
        x = rng.integers(0, 256, (cfg.batch,) + tuple(cfg.image), dtype=np.uint8)
    else:
        x = rng.standard_normal((cfg.batch,) + tuple(cfg.image)).astype(np.float32)
    t = threading.Thread(target=d.run_defer, args=(m, cuts, inq, outq), daemon=True)
    start = time.time()
    t.start()

    def feed():
        for _ in range(a.requests):
            inq.put(x)

    threading.Thread(target=feed, daemon=True).start()
    try:
        t_first = None
        for i in range(a.requests):
            outq.get(timeout=600)
            if t_first is None:
                t_first = time.time()
        end = time.time()
        run = end - start
        print(f"{a.requests} results in {run:.3f} seconds (incl. partition + slice push)")
        print(f"Throughput: {a.requests * cfg.batch / run:.2f} img/s ({a.requests / run:.2f} req/s)")
        if a.requests > 1 and end > t_first:
            steady = (a.requests - 1) / (end - t_first)
            print(f"Steady-state: {steady * cfg.batch:.2f} img/s ({steady:.2f} req/s) after the first result")
        for ts, ev in d.events:
            print(f"  [{ts - start:8.3f}s] {ev}")
    finally:
        d.shutdown(stop_workers=True)
        for p in procs:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass


def cmd_local_infer(argv):
    ap = argparse.ArgumentParser(prog="local-infer")
    _common(ap)
    ap.add_argument("--requests", type=int, default=10)
    ap.add_argument("--device", default=None)
    a = ap.parse_args(argv)
    cfg = _cfg(a)
    m = _model(cfg)
    x = np.random.default_rng(cfg.seed).standard_normal((cfg.batch,) + tuple(cfg.image)).astype(np.float32)
    m.predict(x, device=a.device)          # build / capture
    start = time.time()
    for _ in range(a.requests):
        res = m.predict(x, device=a.device)
    run = time.time() - start
    print(res.shape)
    print(f"{a.requests} results in {run:.4f} seconds")
    print(f"Throughput: {a.requests / run:.2f} req/s ({a.requests * cfg.batch / run:.1f} img/s at batch {cfg.batch})")


def cmd_plan(argv):
    ap = argparse.ArgumentParser(prog="plan")
    _common(ap)
    ap.add_argument("--stages", type=int, default=2)
    ap.add_argument("--dtype", default="fp32", choices=["bf16", "fp32"],
                    help="activation precision of the job (frontier bytes, conv rate)")
    a = ap.parse_args(argv)
    cfg = _cfg(a)
    from .graph.planner import balance_ratio, plan_cuts
    from .graph.slicer import frontier_bytes, partition
    m = _model(cfg)
    b = max(cfg.batch, 1)
    cuts = cfg.cuts(m.graph, precision=a.dtype) if cfg.part_at else \
        plan_cuts(m.graph, a.stages, batch=b, precision=a.dtype)[0]
    _, per = plan_cuts(m.graph, len(cuts) + 1, batch=b, candidates=cuts, precision=a.dtype) if cuts else ([], [0])
    print(f"part_at = {cuts}   (max stage / ideal = {balance_ratio(per):.3f})")
    ab = 4 if a.dtype == "fp32" else 2
    for s, t in zip(partition(m.graph, cuts), per):
        fb = frontier_bytes(m.graph, s.outputs, ab) * b
        print(f"  {s.name}: {len(s.layers):3d} layers, est {t * 1e3:7.3f} ms, sends {s.outputs} ({fb / 1e6:.1f} MB {a.dtype})")


def cmd_summary(argv):
    ap = argparse.ArgumentParser(prog="summary")
    _common(ap)
    a = ap.parse_args(argv)
    _model(_cfg(a)).summary()


COMMANDS = {"membership": cmd_membership, "node": cmd_node, "serve": cmd_serve, "local-infer": cmd_local_infer,
            "plan": cmd_plan, "summary": cmd_summary}


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] not in COMMANDS:
        print(__doc__)
        sys.exit(0 if not argv else 2)
    code = 0
    try:
        COMMANDS[argv[0]](argv[1:])
    except SystemExit as e:
        code = e.code if isinstance(e.code, int) else (0 if e.code is None else 1)
    except BaseException:  # noqa: BLE001
        import traceback
        traceback.print_exc()
        code = 1
    # Leave without interpreter finalization: daemon I/O threads may still sit in
    # native recv() calls with the GIL released, and CPython 3.10 retires such
    # threads with a forced unwind that aborts the process (node.py does the same).
    sys.stdout.flush()
    sys.stderr.flush()
    os._exit(code)


if __name__ == "__main__":
    main()
