#!/usr/bin/env python3
"""RCCL p2p on one MI355X through the native comm layer (`parallel/rccl.py`):
a world=1 communicator sends BASELINE config 2's two-tensor frontier
(`part_at=['conv3_block1_1_conv']`, bs=32 bf16, 57 MB) to itself, grouped, N
times, checks it bit-exact and prints one JSON line.  Run it under
`rocprofv3 --kernel-trace --stats` to see the RCCL p2p kernels."""
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.parallel import rccl  # noqa: E402


def main(reps: int = 20) -> None:
    store = dist.HashStore()
    c = rccl.RcclComm(store, "selftest", 1, 0, "cuda:0")
    g = torch.Generator(device="cuda").manual_seed(0)
    a = torch.randn((32, 28, 28, 128), generator=g, device="cuda").to(torch.bfloat16)
    b = torch.randn((32, 56, 56, 256), generator=g, device="cuda").to(torch.bfloat16)
    ra, rb = torch.empty_like(a), torch.empty_like(b)
    c.p2p(sends=[(a, 0), (b, 0)], recvs=[(ra, 0), (rb, 0)]).wait_host(timeout_s=30)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        w = c.p2p(sends=[(a, 0), (b, 0)], recvs=[(ra, 0), (rb, 0)])
    w.wait_host(timeout_s=60)
    dt = time.perf_counter() - t0
    ok = torch.equal(ra.view(torch.int16), a.view(torch.int16)) and torch.equal(rb.view(torch.int16),
                                                                                   b.view(torch.int16))
    nbytes = (a.numel() + b.numel()) * 2
    print(json.dumps({"test": "rccl self p2p (world=1, grouped send+recv)", "rccl": rccl.native().load(""),
                      "rccl_version": rccl.native().version(), "bytes": nbytes, "reps": reps,
                      "GBps": round(nbytes * reps / dt / 1e9, 1), "bitexact": bool(ok)}), flush=True)
    c.destroy()
    if not ok:
        sys.exit(1)


_T0 = time.perf_counter()


def stamp(phase: str) -> None:
    """Per-phase progress on stderr: a hang on a GPU box then names its phase."""
    print(f"[rccl_selftest +{(time.perf_counter() - _T0) * 1e3:9.1f} ms] {phase}", file=sys.stderr, flush=True)


def unmatched(timeout_s: float = 5.0) -> None:
    """A world=1 receive with no matching send: RCCL must report it (synchronously
    or through the async-error watch, which then aborts the communicator), and a
    fresh communicator must work afterwards.  If the abort exceeds its deadline
    (`abort_stuck`) this process gives up like a worker does (exit 75) and
    prints that instead: a rebuild in a process whose abort is stuck is not
    attempted."""
    store = dist.HashStore()
    stamp("init (world=1, watch 200 us)")
    c = rccl.RcclComm(store, "unmatched", 1, 0, "cuda:0", watch_us=200, timeout_s=timeout_s)
    stamp(f"init done ({c._c.init_ms:.1f} ms)")
    y = torch.zeros(1 << 16, device="cuda", dtype=torch.int32)
    t0 = time.perf_counter()
    err = None
    try:
        stamp("enqueue: grouped recv with no send")
        w = c.p2p(recvs=[(y, 0)])
        stamp("enqueue returned; wait_host")
        w.wait_host(timeout_s=timeout_s)
        stamp("wait_host returned (no error?)")
    except Exception as e:  # noqa: BLE001
        err = f"{type(e).__name__}: {e}"
        stamp(f"reported: {err[:160]}")
    dt = (time.perf_counter() - t0) * 1e3
    stamp(f"abort entry (aborted already: {c.aborted})")
    if not c.aborted:
        c.abort()
    t_ab = time.perf_counter()
    while c._c.abort_ms == 0.0 and c.aborted and time.perf_counter() - t_ab < rccl.ABORT_DEADLINE_S + 1:
        time.sleep(1e-3)                # the watch thread's abort is still inside its deadline
    stamp(f"abort exit ({c._c.abort_ms:.1f} ms, stuck={c.abort_stuck})")
    rec = {"test": "unmatched self-receive", "reported": err, "ms": round(dt, 2),
           "abort_ms": round(c._c.abort_ms, 2), "abort_stuck": c.abort_stuck}
    if c.abort_stuck:
        rec["rebuilt_ok"] = None
        print(json.dumps(rec), flush=True)
        os._exit(75)
    stamp("rebuild init")
    c2 = rccl.RcclComm(store, "unmatched-rebuilt", 1, 0, "cuda:0", timeout_s=10.0)
    x = torch.full((4096,), 7, device="cuda", dtype=torch.int32)
    z = torch.zeros_like(x)
    stamp("rebuild p2p")
    c2.p2p(sends=[(x, 0)], recvs=[(z, 0)]).wait_host(timeout_s=10)
    ok = torch.equal(x, z)
    stamp("rebuild destroy")
    c2.destroy()
    stamp("done")
    rec["rebuilt_ok"] = bool(ok)
    print(json.dumps(rec), flush=True)
    if err is None or not ok:
        sys.exit(1)


def stuck(deadline_s: float = 1.0, stall_ms: int = 60000) -> None:
    """The deadline path of a bounded abort: ncclCommAbort is made to stall
    (`inject_abort_stall`) past the deadline; abort() must return at the
    deadline with abort_stuck set, and the worker-side give-up (node.py
    `Node.give_up`, process mode) must end the process with exit 75 at once."""
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.node import Node
    store = dist.HashStore()
    stamp("init")
    c = rccl.RcclComm(store, "stuck", 1, 0, "cuda:0", watch_us=1000, abort_deadline_s=deadline_s)
    x = torch.arange(1 << 16, device="cuda", dtype=torch.int32)
    z = torch.zeros_like(x)
    c.p2p(sends=[(x, 0)], recvs=[(z, 0)]).wait_host(timeout_s=10)
    stamp("healthy p2p done; injecting abort stall")
    c._c.inject_abort_stall(stall_ms)
    t0 = time.perf_counter()
    c.abort()
    ms = (time.perf_counter() - t0) * 1e3
    stamp(f"abort returned after {ms:.1f} ms, stuck={c.abort_stuck}")
    print(json.dumps({"test": "stuck abort", "abort_ms": round(ms, 2), "abort_stuck": c.abort_stuck,
                      "deadline_ms": deadline_s * 1e3, "bitexact_before": bool(torch.equal(x, z))}), flush=True)
    if not c.abort_stuck:
        sys.exit(1)
    node = Node(data_port=0, config_port=0, device="cuda:0", node_id="selftest", register=False,
                exit_on_unrecoverable=True)

    class _Rt:
        epoch = 1

    node.give_up(_Rt(), "injected: ncclCommAbort exceeded its deadline")
    sys.exit(1)                 # not reached: give_up exits 75


if __name__ == "__main__":
    import faulthandler
    # a hang dumps every thread's stack to stderr and ends the process before the caller's limit
    faulthandler.dump_traceback_later(float(os.environ.get("RCCL_SELFTEST_LIMIT_S", "45")), exit=True)
    if len(sys.argv) > 1 and sys.argv[1] == "unmatched":
        unmatched()
    elif len(sys.argv) > 1 and sys.argv[1] == "stuck":
        stuck()
    else:
        main()
