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


def unmatched(timeout_s: float = 5.0) -> None:
    """A world=1 receive with no matching send: RCCL must report it (synchronously
    or through the async-error watch, which then aborts the communicator), and a
    fresh communicator must work afterwards."""
    store = dist.HashStore()
    c = rccl.RcclComm(store, "unmatched", 1, 0, "cuda:0", watch_us=200)
    y = torch.zeros(1 << 16, device="cuda", dtype=torch.int32)
    t0 = time.perf_counter()
    err = None
    try:
        c.p2p(recvs=[(y, 0)]).wait_host(timeout_s=timeout_s)
    except Exception as e:  # noqa: BLE001
        err = f"{type(e).__name__}: {e}"
    dt = (time.perf_counter() - t0) * 1e3
    if not c.aborted:
        c.abort()
    c2 = rccl.RcclComm(store, "unmatched-rebuilt", 1, 0, "cuda:0")
    x = torch.full((4096,), 7, device="cuda", dtype=torch.int32)
    z = torch.zeros_like(x)
    c2.p2p(sends=[(x, 0)], recvs=[(z, 0)]).wait_host(timeout_s=30)
    ok = torch.equal(x, z)
    c2.destroy()
    print(json.dumps({"test": "unmatched self-receive", "reported": err, "ms": round(dt, 2),
                      "rebuilt_ok": bool(ok)}), flush=True)
    if err is None or not ok:
        sys.exit(1)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "unmatched":
        unmatched()
    else:
        main()
