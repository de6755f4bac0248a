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
from .pipeline import CompressedStageLink, StageLink, stage_ranks


class DPJob:
    """Whole-model replica per GPU.  With ``streams > 1`` the GPU keeps that many
    independent bs=`batch` micro-batches in flight on separate HIP streams (the
    reference's concurrent in-flight requests, `concurrency_sem`,
    `src/dispatcher.py:151,183`): each stream replays its own hipGraph over its
    own activation buffers while sharing the resident weights, so the small
    per-layer GEMMs of different micro-batches fill CUs the other leaves idle."""

    def __init__(self, g, weights, world: int, rank: int, device, batch: int, graph: bool = True, tune: bool = False,
                 streams: int = 1, precision: str = "fp32"):
        self.device = torch.device(device)
        self.exs = [SliceExecutor(g, weights, batch, device=device, tune=tune and i == 0, precision=precision)
                    for i in range(streams)]
        for ex in self.exs[1:]:           # share packed weights with the first executor
            ex.packed = self.exs[0].packed
            ex.cfg = dict(self.exs[0].cfg)
            ex._ensure_ws()               # private split-K workspace per stream
        self.ex = self.exs[0]
        self.streams = [torch.cuda.Stream(device=self.device) for _ in range(streams)] if streams > 1 else [None]
        if graph:
            for ex, s in zip(self.exs, self.streams):
                if s is None:
                    ex.capture()
                else:
                    with torch.cuda.stream(s):
                        ex.capture()
        self.images_per_step = batch * world * streams
        self.global_batch = batch * world * streams
        self.parallelism = f"dp{world}" + (f"x{streams}streams" if streams > 1 else "")
        self.part_at: List[str] = []
        self.input_name = g.input

    def set_synthetic_input(self, x: torch.Tensor) -> None:
        for ex in self.exs:
            ex.input_buf(self.input_name).copy_(x)

    def step(self) -> None:
        if len(self.exs) == 1:
            self.ex.forward(0)
            return
        cur = torch.cuda.current_stream(self.device)
        for ex, s in zip(self.exs, self.streams):
            s.wait_stream(cur)
            with torch.cuda.stream(s):
                ex.forward(0)
        for s in self.streams:
            cur.wait_stream(s)

    def outputs(self):
        return {o: self.ex.output_buf(o) for o in self.ex.outputs}


_JOB_SEQ = [0]      # every rank builds its jobs in the same order: a fresh store prefix per job


class PipelineJob:
    """One stage of a (replicated) pipeline; step() = `stages` micro-batch ticks."""

    def __init__(self, g, weights, world: int, rank: int, device, batch: int, stages: int,
                 part_at: Optional[List[str]] = None, graph: bool = True, tune: bool = False, nsets: int = 2,
                 host_staged: bool = False, codec: str = "none", precision: str = "fp32"):
        if world % stages:
            raise ValueError(f"world {world} not divisible by stages {stages}")
        self.stages = stages
        self.replicas = world // stages
        self.replica = rank // stages
        self.stage = rank % stages
        if not part_at:
            part_at, _ = plan_cuts(g, stages, batch=batch, precision=precision)
        if len(part_at) != stages - 1:
            raise ValueError(f"{stages} stages need {stages - 1} cuts, got {part_at}")
        self.part_at = list(part_at)
        self.slices = partition(g, self.part_at)
        sl = self.slices[self.stage]
        self.slice = sl
        sg = subgraph(g, sl)
        self.ex = SliceExecutor(sg, {k: v for k, v in weights.items()}, batch, device=device, tune=tune,
                                num_sets=nsets, precision=precision)
        if graph:
            self.ex.capture()
        rk = stage_ranks(self.stage, stages, self.replica)
        self.prev, self.next = rk["prev"], rk["next"]
        self.links = None
        if not host_staged and torch.device(device).type == "cuda":
            # RCCL over xGMI through the native comm layer: one non-blocking 2-rank
            # communicator per adjacent stage pair (unique ids over the job's store)
            from .rccl import PairLinks
            from torch.distributed import distributed_c10d as c10d
            _JOB_SEQ[0] += 1
            self.links = PairLinks(c10d._get_default_store(), f"pp{stages}/job{_JOB_SEQ[0]}", rank, self.prev,
                                   self.next, device)
        in_bufs = [[self.ex.input_buf(n, j) for n in sl.inputs] for j in range(nsets)]
        out_bufs = [[self.ex.output_buf(n, j) for n in sl.outputs] for j in range(nsets)]
        self.codec = codec
        if codec == "none":
            self.link = StageLink(lambda j: self.ex.forward(j), in_bufs, out_bufs, self.prev, self.next,
                                  host_staged=host_staged, links=self.links)
        else:
            # byte counts ride a host (gloo) control group; with host staging the
            # default group already is gloo
            ctl = None if host_staged else dist.new_group(backend="gloo")
            self.link = CompressedStageLink(lambda j: self.ex.forward(j), in_bufs, out_bufs, self.prev, self.next,
                                            codec=codec, ctl_group=ctl, host_staged=host_staged, links=self.links)
        self.images_per_step = batch * world          # stages ticks x replicas x batch / stages-per-image
        self.global_batch = batch * world
        self.parallelism = f"pp{stages}" if self.replicas == 1 else f"pp{stages}xdp{self.replicas}"
        self._primed = False

    def set_synthetic_input(self, x: torch.Tensor) -> None:
        if self.stage == 0:
            for j in range(self.ex.num_sets):
                self.ex.input_buf(self.slice.inputs[0], j).copy_(x)

    def set_total_steps(self, n: int) -> None:
        """Number of step() calls that will follow (lets the link avoid posting
        receives for micro-batches that never come)."""
        self._total_ticks = n * self.stages

    def step(self) -> None:
        if not self._primed:
            self.link.prime(getattr(self, "_total_ticks", None))
            self._primed = True
        for _ in range(self.stages):
            self.link.step()
        if hasattr(self.link, "flush"):
            self.link.flush()            # a step ends with every message posted (callers barrier between steps)

    def finish(self) -> None:
        self.link.drain()

    def close(self, timeout_s: float = 10.0) -> bool:
        """Teardown of the RCCL links (every rank of the pipeline calls it).  The
        link streams are drained with a bounded poll, then the communicators
        aborted; only then is the device synchronised, so a peer that died with
        a transfer pending cannot block this rank for good.  Returns whether
        the links drained cleanly."""
        ok = True
        if self.links is not None:
            ok = self.links.destroy(timeout_s)
            stuck = self.links.abort_stuck()
            self.links = None
            if stuck:
                # a device sync would wait on the transfer the abort could not end
                from .rccl import StuckAbort
                raise StuckAbort("pipeline links: ncclCommAbort exceeded its deadline; give the process up")
        torch.cuda.synchronize(self.ex.device)
        return ok

    def abort(self) -> None:
        """Abort the RCCL links from any thread (failure isolation in bench.py):
        RCCL kernels waiting on a peer return, pending host waits raise."""
        if self.links is not None:
            self.links.abort()


def build_job(g, weights, mode: str, world: int, rank: int, device, batch: int = 32, stages: int = 0,
              part_at: Optional[List[str]] = None, graph: bool = True, tune: bool = False,
              host_staged: bool = False, streams: int = 1, codec: str = "none", precision: str = "fp32"):
    if mode == "dp" or world == 1 and not part_at:
        return DPJob(g, weights, world, rank, device, batch, graph=graph, tune=tune, streams=streams,
                     precision=precision)
    if mode == "pp":
        k = len(part_at) + 1 if part_at else world
        if k != world:
            raise ValueError(f"pp mode: {k} stages for {world} ranks")
        return PipelineJob(g, weights, world, rank, device, batch, k, part_at, graph=graph, tune=tune,
                           host_staged=host_staged, codec=codec, precision=precision)
    if mode == "ppdp":
        k = stages or (len(part_at) + 1 if part_at else 2)
        return PipelineJob(g, weights, world, rank, device, batch, k, part_at, graph=graph, tune=tune,
                           host_staged=host_staged, codec=codec, precision=precision)
    raise ValueError(f"unknown mode {mode}")
