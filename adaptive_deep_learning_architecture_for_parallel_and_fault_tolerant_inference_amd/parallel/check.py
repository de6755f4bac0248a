"""Multi-GPU correctness and link checks (one rank per MI355X, RCCL over xGMI).

    python -m <pkg>.parallel.check --gpus 2 --part-at conv3_block1_1_conv
    python -m <pkg>.parallel.check --gpus 8 --codec lz4            # planner cuts, 8 stages
    python -m <pkg>.parallel.check --gpus 2 --p2p-bw               # RCCL p2p GB/s per size

Without torchrun the script launches its own ranks (parallel/launch.py).

``pipeline`` mode runs a `PipelineJob` (the bench's pp data plane: RCCL
isend/irecv between neighbouring stages, double-buffered) on a seeded input
and has the last rank compare the pre-softmax logits with an *unsliced*
`SliceExecutor` forward of the same input on its own GPU: the max logit error
relative to the largest logit must stay within `--rtol` and top-1 must agree
on every image.  This is the reference's
layer-partitioned chain (`src/dispatcher.py:39-53`, `src/node.py:163-179`)
checked end to end.

``p2p-bw`` times RCCL send/recv (the native comm layer, `parallel/rccl.py`)
between ranks 0 and 1 for 1-64 MiB messages
(the link the planner's `link_bw` stands for) and prints one JSON line; with
``--out`` it is also written for `graph.planner.load_calibration`.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

PKG = "adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "2")))
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--part-at", default="")
    ap.add_argument("--codec", default="none", choices=["none", "lz4", "zvc"])
    ap.add_argument("--steps", type=int, default=3)
    # logits, not probabilities: a cut moves where bf16 rounding happens (a fused epilogue
    # becomes a stored bf16 frontier), so bf16 logits differ by up to a few 1e-2 of the largest
    # logit; fp32 end to end stays within 1e-3
    ap.add_argument("--rtol", type=float, default=0.0, help="logit tolerance (0: 5e-2 bf16, 1e-3 fp32)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--p2p-bw", action="store_true")
    ap.add_argument("--out", default="")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: host-staged rehearsal, several ranks may share one GPU")
    ap.add_argument("--min-top1", type=float, default=1.0)
    return ap.parse_args(argv)


def _p2p_bw(rank: int, world: int, dev, out: str) -> dict:
    import torch
    import torch.distributed as dist
    from torch.distributed import distributed_c10d as c10d

    from .rccl import PairLinks
    res = {}
    if rank > 1:
        dist.barrier()
        return res
    links = PairLinks(c10d._get_default_store(), "p2pbw", rank, 0 if rank == 1 else None, 1 if rank == 0 else None,
                      dev)
    for mib in (1, 4, 16, 64):
        n = mib << 20
        t = torch.empty(n, dtype=torch.uint8, device=dev)
        reps = 20
        for it in range(2):                        # warm-up round, then the timed round
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(reps):
                w = links.isend([t]) if rank == 0 else links.irecv([t])
            w.wait_host(timeout_s=60)
            torch.cuda.synchronize(dev)
            dt = time.perf_counter() - t0
        res[f"{mib}MiB"] = round(n * reps / dt / 1e9, 2)
    links.destroy()
    dist.barrier()
    if rank == 0:
        rec = {"metric": "rccl p2p GB/s (rank0 -> rank1)", "gbps": res,
               "link_bw": max(res.values()) * 1e9}
        print(json.dumps(rec), flush=True)
        if out:
            with open(out, "w") as f:
                json.dump(rec, f)
    return res


def main(argv=None) -> int:
    a = parse(argv)
    from importlib import import_module
    launch = import_module(f"{PKG}.parallel.launch")
    if not launch.launched_by_torchrun():
        return launch.launch_local(list(sys.argv[1:] if argv is None else argv), a.gpus,
                                   module=f"{PKG}.parallel.check", timeout_s=900)
    import torch
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    ndev = torch.cuda.device_count()
    if a.backend == "nccl" and ndev < world:
        print(f"check: {world} ranks need {world} GPUs, found {ndev}", file=sys.stderr)
        return 3
    local = local % max(1, ndev)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if a.backend == "nccl":
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group("gloo")
    try:
        if a.p2p_bw:
            _p2p_bw(rank, world, dev, a.out)
            return 0
        zoo = import_module(f"{PKG}.models.zoo")
        resnet = import_module(f"{PKG}.models.resnet")
        runner = import_module(f"{PKG}.parallel.runner")
        g = zoo.build_model(a.model)
        w = resnet.init_weights(g, seed=0)
        cuts = [c for c in a.part_at.split(",") if c]
        job = runner.build_job(g, w, mode="pp", world=world, rank=rank, device=dev, batch=a.batch,
                               part_at=cuts, graph=True, codec=a.codec, host_staged=a.backend != "nccl",
                               precision=a.dtype)
        image = tuple(g.layers[g.input].out_shape)
        x = torch.randn((a.batch,) + image, generator=torch.Generator().manual_seed(7)).to(dev)
        job.set_synthetic_input(x)
        job.set_total_steps(a.steps)
        for _ in range(a.steps):
            job.step()
        job.finish()
        torch.cuda.synchronize(dev)
        ok = 1
        rec = {}
        if job.next is None:                          # last stage: compare with the unsliced model
            ex_mod = import_module(f"{PKG}.runtime.executor")
            full = ex_mod.SliceExecutor(g, w, a.batch, device=dev, precision=a.dtype)
            full(x)
            want = full.logits().double()
            got = job.ex.logits().double()
            rel = ((got - want).abs().max() / want.abs().max()).item()
            top1 = (got.argmax(-1) == want.argmax(-1)).float().mean().item()
            rtol = a.rtol or (5e-2 if a.dtype == "bf16" else 1e-3)
            ok = int(rel <= rtol and top1 >= a.min_top1)
            rec = {"check": "pipeline vs unsliced (logits)", "model": a.model, "stages": world,
                   "part_at": job.part_at, "codec": a.codec, "backend": a.backend, "dtype": a.dtype,
                   "batch": a.batch, "max_logit_rel": rel, "rtol": rtol, "top1_agree": top1, "ok": bool(ok),
                   "rccl_native": getattr(job, "links", None) is not None}
        flag = torch.tensor([ok], device=dev if a.backend == "nccl" else "cpu")
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if rec:
            print(json.dumps(rec), flush=True)
        if hasattr(job, "close"):
            job.close()
        return 0 if flag.item() == 1 else 1
    finally:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
