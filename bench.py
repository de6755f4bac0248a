#!/usr/bin/env python3
"""Headline benchmark: ResNet-50 inference images/sec (whole node), bs=32 per
pipeline micro-batch, synthetic 224x224x3 input, random-init weights
(BASELINE.json: "images/sec (whole node) ResNet-50 bs=32 at 1/2/4/8 MI355X").

Single GPU:    python bench.py --steps 50 --warmup 10
N GPUs:        python bench.py --gpus N           (starts N rank processes itself,
                   parallel/launch.py), or under torchrun:
               python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
                   --master-addr 127.0.0.1 --master-port P bench.py --gpus N

Parallelism (``--mode``):
  dp    every GPU runs the whole model on its own bs=32 batch (replicas)
  pp    the model is cut into N stages (balanced planner or --part-at), one per
        GPU; bs=32 micro-batches stream through RCCL send/recv over xGMI
  ppdp  R replicas of a k-stage pipeline (R*k = N), --stages k
A step = one bs=32 batch per pipeline replica slot: dp processes 32*N images
per step, pp keeps N micro-batches in flight and completes N per step, so
per-GPU work is fixed as N grows (weak scaling) in every mode.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import time

import torch
import torch.distributed as dist

PKG = "adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd"


def parse():
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
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"],
                    help="compute precision: bf16 (fp32 accumulation) or fp32 end to end (the reference's "
                         "Keras float32, on the fp32 matrix cores)")
    ap.add_argument("--codec", default="none", choices=["none", "lz4", "zvc"],
                    help="pp/ppdp: compress stage-boundary activations on a side stream (BASELINE config 3)")
    return ap.parse_args()


BASELINE_IMG_S = None   # the reference publishes no absolute number
MODEL_NAMES = {"resnet50": "ResNet-50", "resnet101": "ResNet-101", "resnet152": "ResNet-152", "vgg16": "VGG16",
               "vgg19": "VGG19", "mobilenet_v2": "MobileNetV2", "densenet121": "DenseNet121",
               "efficientnetb0": "EfficientNetB0", "inception_v3": "InceptionV3"}


def main():
    args = parse()
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
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    resnet = import_module(f"{PKG}.models.resnet")
    zoo = import_module(f"{PKG}.models.zoo")
    runner = import_module(f"{PKG}.parallel.runner")

    g = zoo.build_model(args.model)
    weights = resnet.init_weights(g, seed=args.seed)
    part_at = [s for s in args.part_at.split(",") if s]
    job = runner.build_job(g, weights, mode=args.mode, world=world, rank=rank, device=dev, batch=args.batch,
                           stages=args.stages, part_at=part_at, graph=not args.no_graph, tune=args.tune,
                           host_staged=(backend != "nccl"), streams=args.streams, codec=args.codec,
                           precision=args.dtype)
    # synthetic input, resident on device (data="synthetic")
    gen = torch.Generator(device=dev).manual_seed(1234 + rank)
    image = tuple(g.layers[g.input].out_shape)          # 224x224x3 (ResNet-50); the model's own size otherwise
    job.set_synthetic_input(torch.randn((args.batch,) + image, generator=gen, device=dev))

    if hasattr(job, "set_total_steps"):
        job.set_total_steps(args.warmup + args.steps)
    for _ in range(args.warmup):
        job.step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        job.step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if hasattr(job, "finish"):
        job.finish()
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        t = t.to(dev) if backend == "nccl" else t
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    images = job.images_per_step * args.steps
    value = images / elapsed
    n_gpus = 1
    if world > 1:
        # distinct physical devices: ranks rehearsing on one GPU count once
        devs = [None] * world
        dist.all_gather_object(devs, (socket.gethostname(), dev_idx))
        n_gpus = launch.distinct_devices(devs)
    if rank == 0:
        rec = {
            "metric": (f"images/sec (whole node) {MODEL_NAMES.get(args.model, args.model)} bs={args.batch}"),
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
            "config": {"model": args.model, "global_batch": job.global_batch, "seq_len": None,
                       "image": list(image), "parallelism": job.parallelism, "part_at": job.part_at,
                       "micro_batch": args.batch, "hipgraph": not args.no_graph,
                       "ranks": world, "backend": backend if world > 1 else None},
        }
        link = getattr(job, "link", None)
        if args.codec != "none" and link is not None:
            rec["config"]["codec"] = args.codec
            rec["config"]["wire_ratio"] = round(link.ratio, 4) if link.ratio else None
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
