"""Single-node rank launcher: one process per MI355X, no torchrun needed.

`bench.py --gpus N` (and `cli.py`) call `launch_local` when they were *not*
started by `torch.distributed.run` (no ``WORLD_SIZE`` in the environment):
the parent parses its flags, picks a free rendezvous port on 127.0.0.1 and
starts N children of the same script with the torchrun environment contract
(``RANK``/``LOCAL_RANK``/``WORLD_SIZE``/``LOCAL_WORLD_SIZE``/``MASTER_ADDR``/
``MASTER_PORT``).  The parent never touches the GPU (no HIP call, so no
forbidden exec-after-init and no context on device 0 that rank 0 would
share); it forwards the children's output, kills the whole job if one rank
fails (a dead RCCL peer would otherwise leave the others blocked in a p2p
op) and exits with the first failing rank's code.

The reference starts one worker per host by hand (`README.md:44`,
`python -m src.node`); here the launcher is the one-host equivalent for the
collective data plane (one stage-pinned process per GPU).
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time
from typing import Dict, List, Optional, Sequence

RANK_ENV = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")
# set by a torchrun agent for *its* job; a job started from inside one of its ranks
# (bench.py's sub-runs) must not inherit them: with TORCHELASTIC_USE_AGENT_STORE
# the new job's rank 0 would join the agent's store instead of hosting its own
AGENT_ENV = ("GROUP_RANK", "GROUP_WORLD_SIZE", "ROLE_RANK", "ROLE_NAME", "ROLE_WORLD_SIZE",
             "LOCAL_WORLD_SIZE", "TORCH_NCCL_ASYNC_ERROR_HANDLING_DISABLED")


def free_port(host: str = "127.0.0.1") -> int:
    s = socket.socket()
    s.bind((host, 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launched_by_torchrun(env: Optional[Dict[str, str]] = None) -> bool:
    env = os.environ if env is None else env
    return "WORLD_SIZE" in env and "RANK" in env


def rank_envs(nprocs: int, port: int, base: Optional[Dict[str, str]] = None,
              master_addr: str = "127.0.0.1") -> List[Dict[str, str]]:
    """The per-rank environment of an `nprocs`-rank single-node job."""
    if nprocs < 1:
        raise ValueError(f"need at least one rank, got {nprocs}")
    base = dict(os.environ if base is None else base)
    for k in list(base):
        if k.startswith("TORCHELASTIC_") or k in AGENT_ENV:
            del base[k]
    out = []
    for r in range(nprocs):
        e = dict(base)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nprocs), LOCAL_WORLD_SIZE=str(nprocs),
                 MASTER_ADDR=master_addr, MASTER_PORT=str(port), GROUP_RANK="0", ROLE_RANK=str(r))
        # the box's HIP/RCCL runtime only supports dmabuf IPC between processes
        e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        out.append(e)
    return out


def launch_local(argv: Sequence[str], nprocs: int, script: Optional[str] = None, timeout_s: Optional[float] = None,
                 port: Optional[int] = None, poll_s: float = 0.05, module: Optional[str] = None,
                 stdout=None) -> int:
    """Run `python <script> <argv>` (or `python -m <module> <argv>`) as `nprocs`
    ranks; returns the job's exit code (124 on timeout).

    Ranks inherit stdout/stderr (rank 0 prints the bench line) unless `stdout`
    redirects them (bench.py's sub-runs send theirs to stderr, so the only
    JSON line on stdout is the record).  When any rank exits non-zero, or
    `timeout_s` passes, the rest of the job is terminated."""
    target = ["-m", module] if module else [script or sys.argv[0]]
    port = port or free_port()
    envs = rank_envs(nprocs, port)
    procs: List[subprocess.Popen] = []
    for e in envs:
        # each rank leads its own process group so a kill reaches its helpers too
        procs.append(subprocess.Popen([sys.executable, *target, *argv], env=e, start_new_session=True,
                                      stdout=stdout))
    t0 = time.monotonic()
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0]
                break
            if all(c == 0 for c in codes):
                break
            if timeout_s is not None and time.monotonic() - t0 > timeout_s:
                rc = 124
                break
            time.sleep(poll_s)
    finally:
        _terminate(procs)
    return rc


def _terminate(procs: List[subprocess.Popen], grace_s: float = 10.0) -> None:
    live = [p for p in procs if p.poll() is None]
    for p in live:
        try:
            os.killpg(p.pid, signal.SIGTERM)
        except (ProcessLookupError, PermissionError):
            pass
    deadline = time.monotonic() + grace_s
    for p in live:
        try:
            p.wait(timeout=max(0.0, deadline - time.monotonic()))
        except subprocess.TimeoutExpired:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except (ProcessLookupError, PermissionError):
                pass
            p.wait()


def distinct_devices(ranks_devices: Sequence[Sequence]) -> int:
    """Number of distinct physical GPUs among (host, device index) pairs: several
    ranks rehearsing on one GPU (gloo) count once."""
    return len({tuple(x) for x in ranks_devices})
