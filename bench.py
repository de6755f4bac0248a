#!/usr/bin/env python3
"""Headline benchmark: ResNet-50 inference images/sec (whole node), bs=32 per
pipeline micro-batch, synthetic 224x224x3 input, random-init weights
(BASELINE.json: "images/sec (whole node) ResNet-50 bs=32 at 1/2/4/8 MI355X").

Single GPU:    python bench.py --steps 50 --warmup 10
N GPUs:        python bench.py --gpus N           (starts N rank processes itself,
                   parallel/launch.py), or under torchrun:
               python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
                   --master-addr 127.0.0.1 --master-port P bench.py --gpus N

Precision: the reference computes in Keras float32 (`src/node.py:177`,
`test/local_infer.py:22`), so the primary ``value`` is fp32 end to end
(fp32 activations and weights on the fp32 matrix cores).  The same run also
times the bf16 build (fp32 accumulation) and reports it as ``value_bf16``.

Parallelism (``--mode``) of the headline:
  dp    every GPU runs the whole model on its own bs=32 batch (replicas)
  pp    the model is cut into N stages (balanced planner or --part-at), one per
        GPU; bs=32 micro-batches stream through RCCL send/recv over xGMI
  ppdp  R replicas of a k-stage pipeline (R*k = N), --stages k
A step = one bs=32 batch per pipeline replica slot: dp processes 32*N images
per step, pp keeps N micro-batches in flight and completes N per step, so
per-GPU work is fixed as N grows (weak scaling) in every mode.

Control traffic (barriers, the max over ranks, result agreement) always runs
on a host (gloo) process group; activations move over the native RCCL p2p
layer (`parallel/rccl.py`), so no eager ProcessGroupNCCL stream competes with
the pipeline's compute and link streams for the 4 hardware queues.

With N > 1 (dp mode) the same invocation then measures BASELINE.json's other
configs as *sub-runs*: after the headline ranks are done, rank 0 starts each
one as a fresh job of its own (`parallel/launch.py`, one process per GPU, a
time limit each, stdout to stderr), so a failing or hanging sub-run is killed
and recorded as ``{"ok": false, "error": ...}`` while the headline line is
always printed:

  pp       every N: the reference's layer-partitioned chain as an N-stage
           pipeline over RCCL p2p, logits checked against the unsliced forward,
           stage0 -> stage1 p2p rate; N == 2 uses config 2's
           part_at=['conv3_block1_1_conv'] (a multi-tensor frontier), N == 8
           config 3's lz4 activation compression on a side stream (wire_ratio)
  pp_r152  N == 4: config 5, ResNet-152 as a 4-stage bf16 pipeline
  fault    N >= 2: config 4, a DEFER serving run at its defaults (fp32,
           transport auto = RCCL p2p with one stage per GPU, 0.25 s heartbeat)
           whose middle stage is SIGKILLed: recovery_ms, detect_ms,
           exactly_once (`parallel/fault_run.py`)
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import time

PKG = "adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd"
# before the first HIP call: a pipeline stage's streams must not share the default 4
# hardware queues (a spinning receive would hold back compute; utils/hwqueues.py)
__import__(f"{PKG}.utils.hwqueues", fromlist=["ensure_hw_queues"]).ensure_hw_queues()

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")),
                    help="ranks (one per GPU); without torchrun the script launches them itself")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--mode", default="dp", choices=["dp", "pp", "ppdp"])
    ap.add_argument("--stages", type=int, default=0, help="stages per pipeline for ppdp")
    ap.add_argument("--part-at", default="", help="comma-separated cut layers (pp)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--tune", action="store_true", help="autotune conv tiles before timing")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--streams", type=int, default=1,
                    help="independent bs=--batch micro-batches in flight per GPU (dp mode)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (production); gloo = host-staged rehearsal (several ranks per GPU)")
    ap.add_argument("--dtype", default="fp32", choices=["bf16", "fp32"],
                    help="headline precision: fp32 end to end (the reference's Keras float32, default) or bf16 "
                         "(fp32 accumulation)")
    ap.add_argument("--no-bf16", action="store_true", help="skip the bf16 companion timing (value_bf16)")
    ap.add_argument("--no-pp", action="store_true", help="N > 1: skip the pipeline sub-benchmark")
    ap.add_argument("--pp-dtype", default="", choices=["", "bf16", "fp32"],
                    help="precision of the pipeline sub-benchmark (default: --dtype)")
    ap.add_argument("--codec", default="none", choices=["none", "lz4", "zvc"],
                    help="pp/ppdp: compress stage-boundary activations on a side stream (BASELINE config 3)")
    ap.add_argument("--no-fault", action="store_true", help="N > 1: skip the kill/recovery sub-run (config 4)")
    ap.add_argument("--no-subruns", action="store_true", help="N > 1: headline only")
    ap.add_argument("--sub-budget", type=float, default=420.0,
                    help="seconds all sub-runs together may take (each also has its own limit)")
    ap.add_argument("--fault-duration", type=float, default=10.0)
    # internal: this process is one rank of a sub-run job started by the headline's rank 0
    ap.add_argument("--sub", default="", choices=["", "pp"], help=argparse.SUPPRESS)
    ap.add_argument("--out", default="", help=argparse.SUPPRESS)
    return ap.parse_args(argv)


BASELINE_IMG_S = None   # the reference publishes no absolute number
MODEL_NAMES = {"resnet50": "ResNet-50", "resnet101": "ResNet-101", "resnet152": "ResNet-152", "vgg16": "VGG16",
               "vgg19": "VGG19", "mobilenet_v2": "MobileNetV2", "densenet121": "DenseNet121",
               "efficientnetb0": "EfficientNetB0", "inception_v3": "InceptionV3"}
# logits tolerance of a pipelined forward against the unsliced one: a cut changes
BF16_MIN_WARMUP = 20      # untimed steps before the value_bf16 companion's K timed steps
# where bf16 rounding happens (a fused epilogue becomes a stored bf16 frontier)
PP_LOGIT_RTOL = {"bf16": 5e-2, "fp32": 1e-3}


def make_record(args, world: int, n_gpus: int, backend: str, value: float, elapsed: float, image, job,
                bf16: dict = None, pp: dict = None, subs: dict = None) -> dict:
    """The one JSON line rank 0 prints (the driver's contract)."""
    rec = {
        "metric": f"images/sec (whole node) {MODEL_NAMES.get(args.model, args.model)} bs={args.batch}",
        "value": round(value, 2),
        "unit": "images/s",
        "n_gpus": n_gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": (round(value / BASELINE_IMG_S, 4) if BASELINE_IMG_S else None),
        "dtype": args.dtype,
        "data": f"synthetic {'x'.join(map(str, image))} NHWC fp32 input, random-init weights (seeded)",
        "config": {"model": args.model, "global_batch": job["global_batch"], "seq_len": None,
                   "image": list(image), "parallelism": job["parallelism"], "part_at": job["part_at"],
                   "micro_batch": args.batch, "hipgraph": not args.no_graph,
                   "ranks": world, "backend": backend if world > 1 else None,
                   "control": "gloo" if world > 1 else None},
    }
    if job.get("codec"):
        rec["config"]["codec"] = job["codec"]
        rec["config"]["wire_ratio"] = job.get("wire_ratio")
    if bf16:
        rec["value_bf16"] = round(bf16["value"], 2)
        rec["ms_per_step_bf16"] = round(bf16["elapsed"] / args.steps * 1e3, 4)
        rec["warmup_bf16"] = bf16.get("warmup", args.warmup)
    if pp is not None:
        rec["pp"] = pp
    for k, v in (subs or {}).items():
        rec[k] = v
    return rec


def make_pp_record(value: float, elapsed: float, steps: int, stages: int, part_at, dtype: str, ok: bool,
                   max_logit_rel: float, top1_agree: float, p2p_gbps, rccl_ranks: int, backend: str) -> dict:
    return {"value": round(value, 2), "unit": "images/s", "ms_per_step": round(elapsed / steps * 1e3, 4),
            "stages": stages, "part_at": list(part_at), "dtype": dtype, "ok": bool(ok),
            "max_logit_rel": (round(max_logit_rel, 6) if max_logit_rel is not None else None),
            "top1_agree": top1_agree,
            "p2p_GBps": (round(p2p_gbps, 2) if p2p_gbps else None), "rccl_ranks": rccl_ranks,
            "backend": backend}


def _max_over_ranks(x: float, world: int) -> float:
    """MAX over ranks on the host (gloo) control group."""
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.item()


def timed(job, steps: int, warmup: int, dev, world: int, stamps=None) -> float:
    """W untimed steps, then exactly K steps bracketed by barrier + synchronize;
    returns the slowest rank's seconds.  `stamps` (PhaseStamps): the first
    step (a pipeline's first p2p), the end of warmup and of the timed steps."""
    if hasattr(job, "set_total_steps"):
        job.set_total_steps(warmup + steps)
    for i in range(warmup):
        job.step()
        if i == 0 and stamps is not None:
            torch.cuda.synchronize(dev)
            stamps.stamp("first_step")
    torch.cuda.synchronize(dev)
    if stamps is not None:
        stamps.stamp("warmup_done")
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        job.step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if stamps is not None:
        stamps.stamp("timed_done", steps=steps)
    if hasattr(job, "finish"):
        job.finish()
    return _max_over_ranks(elapsed, world)


def _p2p_rates(job, dev, world: int, mib: int = 64, reps: int = 10) -> dict:
    """Every adjacent stage pair's rate on the pipeline's own links, all pairs at
    once (as a pipeline drives them): each stage sends `reps` x `mib` MiB to its
    next stage while receiving as much from its previous one, and the receiver's
    time gives the pair's rate.  Returns {"a-b": bytes/s} (global ranks), the
    same dict on every rank; host-staged (gloo) pipelines time the same
    exchange through host copies."""
    n = mib << 20
    sbuf = torch.empty(n, dtype=torch.uint8, device=dev)
    rbuf = torch.empty(n, dtype=torch.uint8, device=dev)
    links = getattr(job, "links", None)
    nxt, prv = job.next, job.prev
    dt = 0.0
    for it in range(2):                                 # warm-up round, then the timed round
        torch.cuda.synchronize(dev)
        dist.barrier()
        t0 = time.perf_counter()
        if links is not None:
            ws, wr = None, None
            for _ in range(reps):
                if nxt is not None:
                    ws = links.isend([sbuf])
                if prv is not None:
                    wr = links.irecv([rbuf])
            if wr is not None:
                wr.wait_host(timeout_s=60)
            dt = time.perf_counter() - t0
            if ws is not None:
                ws.wait_host(timeout_s=60)
        else:
            hs, hr = sbuf.cpu(), torch.empty(n, dtype=torch.uint8)
            for _ in range(reps):
                reqs = []
                if nxt is not None:
                    reqs.append(dist.isend(hs, nxt))
                if prv is not None:
                    reqs.append(dist.irecv(hr, prv))
                for r in reqs:
                    r.wait()
                if prv is not None:
                    rbuf.copy_(hr)
            torch.cuda.synchronize(dev)
            dt = time.perf_counter() - t0
        torch.cuda.synchronize(dev)
    mine = (prv, dist.get_rank(), dt) if prv is not None else None
    allp = [None] * world
    dist.all_gather_object(allp, mine)
    return {f"{a}-{b}": n * reps / t for (a, b, t) in (x for x in allp if x) if t > 0}


def _stamps(rank: int):
    from importlib import import_module
    return import_module(f"{PKG}.utils.telemetry").PhaseStamps(f"bench r{rank}")


def run_pp(args, g, weights, world: int, rank: int, dev, backend: str, runner, executor, part_at,
           stamps=None) -> dict:
    """The reference's layer-partitioned chain over RCCL, verified against an unsliced forward.
    Per-phase stamps go to stderr (and the record's ``phases``): link init per pair, first step
    (first p2p), warmup, timed, p2p rates, verification, teardown (``links_drained``)."""
    dtype = args.pp_dtype or args.dtype
    st = stamps or _stamps(rank)
    t_build = time.perf_counter()
    job = runner.build_job(g, weights, mode="pp", world=world, rank=rank, device=dev, batch=args.batch,
                           part_at=part_at, graph=not args.no_graph, host_staged=(backend != "nccl"),
                           codec=args.codec, precision=dtype)
    build_s = time.perf_counter() - t_build
    links = getattr(job, "links", None)
    mine = {}
    if links is not None:
        for c in links.comms():
            mine[c.name.rsplit("/link", 1)[-1]] = round(c._c.init_ms, 1)
    st.stamp("build_job", stage=job.stage, build_s=round(build_s, 2), link_init_ms=mine or None)
    image = tuple(g.layers[g.input].out_shape)
    x = torch.randn((args.batch,) + image, generator=torch.Generator().manual_seed(4321)).to(dev)
    job.set_synthetic_input(x)
    elapsed = timed(job, args.steps, args.warmup, dev, world, stamps=st)
    value = job.images_per_step * args.steps / elapsed
    rates = _p2p_rates(job, dev, world)
    st.stamp("p2p_rates", pairs={k: round(v / 1e9, 1) for k, v in rates.items()})
    rate = rates.get("0-1")
    inits = [None] * world
    dist.all_gather_object(inits, mine)
    link_init = {}
    for d_ in inits:
        for k, v in (d_ or {}).items():
            link_init[k] = max(link_init.get(k, 0.0), v)
    ok, rel, top1 = 1, None, None
    if job.next is None:                       # last stage: logits vs the unsliced model on its own GPU
        full = executor.SliceExecutor(g, weights, args.batch, device=dev, precision=dtype)
        full(x)
        want = full.logits().double()
        got = job.ex.logits().double()
        rel = ((got - want).abs().max() / want.abs().max()).item()
        top1 = (got.argmax(-1) == want.argmax(-1)).float().mean().item()
        ok = int(rel <= PP_LOGIT_RTOL[dtype] and top1 == 1.0)
        del full
    flag = torch.tensor([ok, rel if rel is not None else 0.0, top1 if top1 is not None else 1.0],
                        dtype=torch.float64)
    flags = [torch.zeros_like(flag) for _ in range(world)]
    dist.all_gather(flags, flag)                # host control group
    oks = [int(f[0].item()) for f in flags]
    last = flags[world - 1] if job.replicas == 1 else max(flags, key=lambda f: f[1].item())
    native = getattr(job, "links", None) is not None
    if native and rank == 0 and rate:
        from importlib import import_module
        planner = import_module(f"{PKG}.graph.planner")
        try:
            planner.LINK_FILE.write_text(json.dumps({"link_bw": rate, "source": "bench.py pp stage0->1 RCCL p2p",
                                                     "mib": 64}))
        except OSError:
            pass
    rec = make_pp_record(value, elapsed, args.steps, job.stages, job.part_at, dtype, min(oks) == 1,
                         last[1].item(), last[2].item(), rate / 1e9 if rate else None,
                         world if native else 0, "rccl-native" if native else backend)
    st.stamp("verified", ok=min(oks) == 1)
    rec["model"] = args.model
    rec["build_s"] = round(build_s, 2)
    rec["p2p_GBps_pairs"] = {k: round(v / 1e9, 2) for k, v in rates.items()}
    rec["link_init_ms"] = link_init or None
    link = getattr(job, "link", None)
    if args.codec != "none":
        ratio = getattr(link, "ratio", None)
        rec["codec"] = args.codec
        rec["wire_ratio"] = round(ratio, 4) if ratio else None
        rec["codec_default"] = "none"          # DEFER(link_codec=...) default: xGMI links stay uncompressed
    if hasattr(job, "close"):
        rec["links_drained"] = bool(job.close())
    st.stamp("teardown", links_drained=rec.get("links_drained"))
    rec["phases"] = dict(st.phases)
    return rec


# ---------------------------------------------------------------- sub-runs
SUB_LIMIT_S = {"pp": 90.0, "pp_r152": 90.0, "fault": 240.0}   # N = 4 worst case: 420 s


def plan_subruns(args, world: int, backend: str) -> list:
    """(name, kind, argv, nprocs, limit_s, label) of the BASELINE.json configs a
    `--gpus N` dp run measures after its headline."""
    if args.no_subruns or args.mode != "dp" or world < 2:
        return []
    common = ["--steps", str(args.steps), "--warmup", str(args.warmup), "--batch", str(args.batch),
              "--backend", backend, "--seed", str(args.seed)] + (["--no-graph"] if args.no_graph else [])
    subs = []
    if not args.no_pp:
        pp = ["--sub", "pp", "--model", args.model, "--pp-dtype", args.pp_dtype or args.dtype] + common
        label = f"{world}-stage pipeline, planner cuts"
        if args.part_at:
            pp += ["--part-at", args.part_at]
            label = f"{world}-stage pipeline, part_at={args.part_at}"
        elif world == 2 and args.model == "resnet50":
            pp += ["--part-at", "conv3_block1_1_conv"]
            label = "BASELINE config 2: 2-stage, part_at=['conv3_block1_1_conv'] (multi-tensor frontier)"
        if args.codec != "none":
            pp += ["--codec", args.codec]
        elif world == 8:
            pp += ["--codec", "lz4"]
            label = ("BASELINE config 3: 8-stage pipeline, lz4 activation compression on a side stream -- a "
                     "measured cost, not a gain: GPU LZ4 reaches ratio 1.07-1.09 on fp32 frontiers at 51-82 GB/s "
                     "encode (profiles/r5/codec_fp32_r50_bs32.txt), below the xGMI link it would relieve, so "
                     "DEFER's per-link default keeps xGMI uncompressed (link_codec='none')")
        subs.append(("pp", "bench", pp, world, SUB_LIMIT_S["pp"], label))
        if world == 4:
            r152 = ["--sub", "pp", "--model", "resnet152", "--pp-dtype", "bf16"] + common
            subs.append(("pp_r152", "bench", r152, 4, SUB_LIMIT_S["pp_r152"],
                         "BASELINE config 5: ResNet-152 4-stage bf16"))
    if not args.no_fault:
        image = "224"
        fault = ["--workers", str(world), "--devices", "each", "--model", args.model, "--image", image,
                 "--batch", str(args.batch), "--duration", str(args.fault_duration),
                 "--kill-at", str(max(2.0, 0.4 * args.fault_duration))]
        subs.append(("fault", "fault", fault, 1, SUB_LIMIT_S["fault"],
                     f"BASELINE config 4: {world}-stage DEFER, middle worker SIGKILLed, DEFER defaults"))
    return subs


def subrun_limit(plan: list, i: int, left: float) -> float:
    """Time limit of sub-run `i` of `plan` with `left` seconds of the shared budget remaining: its own
    limit, but never eating into the limits of the sub-runs still to come (the fault run, last, keeps
    its whole limit even when the pipeline sub-runs before it hit theirs)."""
    reserve = sum(p[4] for p in plan[i + 1:])
    return max(0.0, min(plan[i][4], left - reserve))


def fault_ready_timeout(limit_s: float, duration: float) -> float:
    """fault_run's wait for its first pipeline, so that the run ends inside its limit: the limit less
    the measured window, the settle time (~4 s) and the exactly-once drain (<= 60 s)."""
    return max(20.0, limit_s - duration - 70.0)


def run_subrun(name: str, kind: str, argv: list, nprocs: int, limit_s: float, label: str, launch) -> dict:
    """One sub-run as a fresh job (a process per rank, its own time limit);
    returns its record, or {"ok": false, "error": ...}.  Never raises."""
    import glob
    import tempfile
    out = os.path.join(tempfile.gettempdir(), f"bench_{name}_{os.getpid()}_{int(time.time() * 1e3)}.json")
    t0 = time.monotonic()
    print(f"bench: sub-run {name} ({label}): {nprocs} process(es), limit {limit_s:.0f} s", file=sys.stderr,
          flush=True)
    os.environ["ADAPT_SUB_LIMIT_S"] = f"{limit_s:.1f}"         # children arm faulthandler from it
    try:
        if kind == "bench":
            rc = launch.launch_local(argv + ["--out", out], nprocs, script=os.path.abspath(__file__),
                                     timeout_s=limit_s, stdout=sys.stderr)
        else:
            rc = launch.launch_local(argv + ["--json", out], 1, module=f"{PKG}.parallel.fault_run",
                                     timeout_s=limit_s, stdout=sys.stderr)
    except Exception as e:  # noqa: BLE001 - a sub-run never takes the headline down
        rc = -1
        err = f"{type(e).__name__}: {e}"
    else:
        err = None
    wall = time.monotonic() - t0
    rec = None
    try:
        with open(out) as f:
            rec = json.load(f)
    except (OSError, ValueError):
        pass
    errs = []
    for p in sorted(glob.glob(out + ".rank*.err")):
        try:
            with open(p) as f:
                errs.append(f.read().strip()[-600:])
        except OSError:
            pass
        os.unlink(p)
    if os.path.exists(out):
        os.unlink(out)
    if rec is None or rc != 0:
        why = err or (errs[0] if errs else ("time limit reached" if rc == 124 else f"exit code {rc}"))
        rec = dict(rec or {}, ok=False, error=why, rc=rc)
    rec.setdefault("ok", True)
    rec["label"] = label
    rec["wall_s"] = round(wall, 1)
    print(f"bench: sub-run {name} done in {wall:.1f} s, ok={rec['ok']}", file=sys.stderr, flush=True)
    return rec


def sub_main(args) -> int:
    """One rank of a `--sub pp` job: a pipeline over RCCL p2p (or the gloo
    rehearsal), result to ``--out`` (rank 0), errors to ``--out.rank<r>.err``."""
    from importlib import import_module
    import datetime
    import traceback
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    st = _stamps(rank)
    # a hang on the 8-GPU node dumps every thread's stack 10 s before the parent's limit
    st.arm_faulthandler(float(os.environ.get("ADAPT_SUB_LIMIT_S", "0") or 0))
    try:
        ndev = torch.cuda.device_count()
        dev_idx = local % max(1, ndev)
        torch.cuda.set_device(dev_idx)
        dev = torch.device("cuda", dev_idx)
        backend = "gloo" if (args.backend == "nccl" and world > ndev) else args.backend
        dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=150))
        st.stamp("init_process_group", world=world, backend=backend)
        zoo = import_module(f"{PKG}.models.zoo")
        resnet = import_module(f"{PKG}.models.resnet")
        runner = import_module(f"{PKG}.parallel.runner")
        executor = import_module(f"{PKG}.runtime.executor")
        g = zoo.build_model(args.model)
        weights = resnet.init_weights(g, seed=args.seed)
        part_at = [c for c in args.part_at.split(",") if c]
        rec = run_pp(args, g, weights, world, rank, dev, backend, runner, executor, part_at, stamps=st)
        if rank == 0 and args.out:
            with open(args.out + ".tmp", "w") as f:
                json.dump(rec, f)
            os.replace(args.out + ".tmp", args.out)
        dist.barrier()
        dist.destroy_process_group()
        return 0
    except BaseException as e:  # noqa: BLE001 - reported to the parent, which records ok: false
        if args.out:
            try:
                with open(f"{args.out}.rank{rank}.err", "w") as f:
                    f.write(f"rank {rank}: {type(e).__name__}: {e}\n" + traceback.format_exc()[-400:])
            except OSError:
                pass
        traceback.print_exc()
        return 3             # the launcher then ends the other ranks (blocked on this one's links)


def main(argv=None):
    args = parse(argv)
    if args.sub:
        sys.stdout.flush()
        rc = sub_main(args)
        sys.stderr.flush()
        os._exit(rc)          # RCCL / gloo threads of an aborted job must not block interpreter exit
    from importlib import import_module
    launch = import_module(f"{PKG}.parallel.launch")
    if args.gpus > 1 and not launch.launched_by_torchrun():
        # no torchrun: become the launcher (before any HIP call in this process)
        sys.exit(launch.launch_local(sys.argv[1:], args.gpus, script=os.path.abspath(__file__)))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and rank == 0:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}; using the launched world", file=sys.stderr)
    ndev = torch.cuda.device_count()
    dev_idx = local % max(1, ndev)
    torch.cuda.set_device(dev_idx)
    dev = torch.device("cuda", dev_idx)
    backend = args.backend
    if world > 1 and backend == "nccl" and world > ndev:
        # RCCL refuses two ranks on one device: rehearse the schedule host-staged
        if rank == 0:
            print(f"bench: {world} ranks on {ndev} GPU(s): RCCL needs one GPU per rank, using gloo "
                  f"(host-staged rehearsal)", file=sys.stderr)
        backend = "gloo"
    if world > 1:
        # host control group only: the data plane is the native RCCL layer
        import datetime
        dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=300))

    resnet = import_module(f"{PKG}.models.resnet")
    zoo = import_module(f"{PKG}.models.zoo")
    runner = import_module(f"{PKG}.parallel.runner")

    g = zoo.build_model(args.model)
    weights = resnet.init_weights(g, seed=args.seed)
    part_at = [s for s in args.part_at.split(",") if s]
    image = tuple(g.layers[g.input].out_shape)          # 224x224x3 (ResNet-50); the model's own size otherwise

    def headline(precision: str, warmup: int):
        job = runner.build_job(g, weights, mode=args.mode, world=world, rank=rank, device=dev, batch=args.batch,
                               stages=args.stages, part_at=part_at, graph=not args.no_graph, tune=args.tune,
                               host_staged=(backend != "nccl"), streams=args.streams, codec=args.codec,
                               precision=precision)
        # synthetic input, resident on device (data="synthetic")
        gen = torch.Generator(device=dev).manual_seed(1234 + rank)
        job.set_synthetic_input(torch.randn((args.batch,) + image, generator=gen, device=dev))
        elapsed = timed(job, args.steps, warmup, dev, world)
        info = {"global_batch": job.global_batch, "parallelism": job.parallelism, "part_at": job.part_at}
        link = getattr(job, "link", None)
        if args.codec != "none" and link is not None:
            info["codec"] = args.codec
            info["wire_ratio"] = round(link.ratio, 4) if link.ratio else None
        value = job.images_per_step * args.steps / elapsed
        if hasattr(job, "close"):
            job.close()
        del job
        torch.cuda.empty_cache()
        return value, elapsed, info

    value, elapsed, info = headline(args.dtype, args.warmup)
    bf16 = None
    if args.dtype == "fp32" and not args.no_bf16:
        # the companion runs after the headline's teardown, on a card whose clocks dropped while the bf16 job
        # was built: at least 20 untimed steps (3 ms of work at W = 5 left 20-step timings 2-3 % low); still
        # exactly K timed steps
        w16 = max(args.warmup, BF16_MIN_WARMUP)
        v16, e16, _ = headline("bf16", w16)
        bf16 = {"value": v16, "elapsed": e16, "warmup": w16}

    n_gpus = 1
    if world > 1:
        # distinct physical devices: ranks rehearsing on one GPU count once
        devs = [None] * world
        dist.all_gather_object(devs, (socket.gethostname(), dev_idx))
        n_gpus = launch.distinct_devices(devs)
        dist.barrier()
        dist.destroy_process_group()
    if rank != 0:
        return
    # BASELINE configs 2-5: fresh jobs, one at a time, each with a time limit; rank 0 does
    # not touch its GPU meanwhile (its executors are freed) and the other ranks have exited
    del weights
    torch.cuda.empty_cache()
    subs = {}
    budget_end = time.monotonic() + args.sub_budget
    plan = plan_subruns(args, world, backend)
    for i, (name, kind, sargv, nprocs, limit, label) in enumerate(plan):
        lim = subrun_limit(plan, i, budget_end - time.monotonic())
        if lim < 30:
            subs[name] = {"ok": False, "error": f"sub-run budget ({args.sub_budget:.0f} s) spent", "label": label}
            continue
        if kind == "fault":
            sargv = sargv + ["--ready-timeout", f"{fault_ready_timeout(lim, args.fault_duration):.0f}"]
        subs[name] = run_subrun(name, kind, sargv, nprocs, lim, label, launch)
    print(json.dumps(make_record(args, world, n_gpus, backend, value, elapsed, image, info, bf16, subs=subs)),
          flush=True)


if __name__ == "__main__":
    main()
