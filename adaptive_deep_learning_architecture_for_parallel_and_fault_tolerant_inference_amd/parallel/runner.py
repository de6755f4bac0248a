"""Parallel job assembly: DP replicas, PP stages, and PP x DP.

`bench.py` and the DEFER dispatcher's data plane both build jobs here.
Topologies:

* ``dp``   : R = world replicas of the whole model (the reference's implicit
             "any idle worker can serve any partition", `src/dispatcher.py:178`)
* ``pp``   : one pipeline, stage i on rank i (the reference's layer-partitioned
             chain, `src/dispatcher.py:39-53`), balanced cuts from the planner
             unless `part_at` is given
* ``ppdp`` : world / k replicas of a k-stage pipeline
"""
from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np
import torch
import torch.distributed as dist

from ..graph.planner import plan_cuts
from ..graph.slicer import partition, subgraph
from ..runtime.executor import SliceExecutor
from .pipeline import StageLink, stage_ranks


class DPJob:
    def __init__(self, g, weights, world: int, rank: int, device, batch: int, graph: bool = True, tune: bool = False):
        self.ex = SliceExecutor(g, weights, batch, device=device, tune=tune)
        if graph:
            self.ex.capture()
        self.images_per_step = batch * world
        self.global_batch = batch * world
        self.parallelism = f"dp{world}"
        self.part_at: List[str] = []
        self.input_name = g.input

    def set_synthetic_input(self, x: torch.Tensor) -> None:
        self.ex.input_buf(self.input_name).copy_(x)

    def step(self) -> None:
        self.ex.forward(0)

    def outputs(self):
        return {o: self.ex.output_buf(o) for o in self.ex.outputs}


class PipelineJob:
    """One stage of a (replicated) pipeline; step() = `stages` micro-batch ticks."""

    def __init__(self, g, weights, world: int, rank: int, device, batch: int, stages: int,
                 part_at: Optional[List[str]] = None, graph: bool = True, tune: bool = False, nsets: int = 2):
        if world % stages:
            raise ValueError(f"world {world} not divisible by stages {stages}")
        self.stages = stages
        self.replicas = world // stages
        self.replica = rank // stages
        self.stage = rank % stages
        if not part_at:
            part_at, _ = plan_cuts(g, stages, batch=batch)
        if len(part_at) != stages - 1:
            raise ValueError(f"{stages} stages need {stages - 1} cuts, got {part_at}")
        self.part_at = list(part_at)
        self.slices = partition(g, self.part_at)
        sl = self.slices[self.stage]
        self.slice = sl
        sg = subgraph(g, sl)
        self.ex = SliceExecutor(sg, {k: v for k, v in weights.items()}, batch, device=device, tune=tune,
                                num_sets=nsets)
        if graph:
            self.ex.capture()
        rk = stage_ranks(self.stage, stages, self.replica)
        self.prev, self.next = rk["prev"], rk["next"]
        in_bufs = [[self.ex.input_buf(n, j) for n in sl.inputs] for j in range(nsets)]
        out_bufs = [[self.ex.output_buf(n, j) for n in sl.outputs] for j in range(nsets)]
        self.link = StageLink(lambda j: self.ex.forward(j), in_bufs, out_bufs, self.prev, self.next)
        self.images_per_step = batch * world          # stages ticks x replicas x batch / stages-per-image
        self.global_batch = batch * world
        self.parallelism = f"pp{stages}" if self.replicas == 1 else f"pp{stages}xdp{self.replicas}"
        self._primed = False

    def set_synthetic_input(self, x: torch.Tensor) -> None:
        if self.stage == 0:
            for j in range(self.ex.num_sets):
                self.ex.input_buf(self.slice.inputs[0], j).copy_(x)

    def step(self) -> None:
        if not self._primed:
            self.link.prime()
            self._primed = True
        for _ in range(self.stages):
            self.link.step()

    def finish(self) -> None:
        self.link.drain()


def build_job(g, weights, mode: str, world: int, rank: int, device, batch: int = 32, stages: int = 0,
              part_at: Optional[List[str]] = None, graph: bool = True, tune: bool = False):
    if mode == "dp" or world == 1 and not part_at:
        return DPJob(g, weights, world, rank, device, batch, graph=graph, tune=tune)
    if mode == "pp":
        k = len(part_at) + 1 if part_at else world
        if k != world:
            raise ValueError(f"pp mode: {k} stages for {world} ranks")
        return PipelineJob(g, weights, world, rank, device, batch, k, part_at, graph=graph, tune=tune)
    if mode == "ppdp":
        k = stages or (len(part_at) + 1 if part_at else 2)
        return PipelineJob(g, weights, world, rank, device, batch, k, part_at, graph=graph, tune=tune)
    raise ValueError(f"unknown mode {mode}")
