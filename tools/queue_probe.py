#!/usr/bin/env python3
"""Hardware-queue probe (tests/test_stream_queues_gpu.py runs it in a child
process, so GPU_MAX_HW_QUEUES is read fresh): does a ResNet-50 slice's graph
replay on the compute stream finish while other streams hold spinning
kernels (`spin_flag`: host-released flag, wall-clock bound, always ends)?

Prints one JSON line:
  stage   the stream set of a pipeline stage process, built in its creation order
          (executor + capture stream, two RCCL link communicators, codec side
          stream, serving copy stream): replay ms with nothing spinning, with the
          two link streams spinning, and with links + side + copy spinning
  sweep   k = 1..8 fresh streams spinning: (compute finished, ms)

    GPU_MAX_HW_QUEUES=4 python tools/queue_probe.py
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

PKG = "adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd"


def replay_while_spinning(ex, K, streams, wait_s):
    flag = torch.zeros(1, dtype=torch.int32, pin_memory=True)
    outs = [torch.zeros(1, dtype=torch.int32, device="cuda") for _ in streams]
    torch.cuda.synchronize()
    evs = []
    for o, s in zip(outs, streams):
        K.spin_flag(flag.data_ptr(), o.data_ptr(), 8000.0, s.cuda_stream)
        e = torch.cuda.Event()
        e.record(s)
        evs.append(e)
    t0 = time.perf_counter()
    ex.forward(0)
    done = torch.cuda.Event()
    done.record()
    finished = False
    while time.perf_counter() - t0 < wait_s:
        if done.query():
            finished = True
            break
        time.sleep(1e-4)
    dt = time.perf_counter() - t0
    pending = all(not e.query() for e in evs)
    flag.fill_(1)
    torch.cuda.synchronize()
    verdicts = [int(o.item()) for o in outs]
    return {"ok": bool(finished and pending), "ms": round(dt * 1e3, 2), "released": all(v == 1 for v in verdicts)}


def main():
    from importlib import import_module
    resnet = import_module(f"{PKG}.models.resnet")
    slicer = import_module(f"{PKG}.graph.slicer")
    executor = import_module(f"{PKG}.runtime.executor")
    rccl = import_module(f"{PKG}.parallel.rccl")
    lib = import_module(f"{PKG}.ops._lib")
    K = lib.kernels()
    g = resnet.build_resnet("resnet50")
    w = resnet.init_weights(g, seed=0)
    sl = slicer.partition(g, ["conv4_block1_out"])[1]
    ex = executor.SliceExecutor(slicer.subgraph(g, sl), w, 32, device="cuda:0", precision="fp32")
    ex.capture()
    store = torch.distributed.HashStore()
    out_link = rccl.RcclComm(store, "q/link0-1", 1, 0, "cuda:0", timeout_s=60)
    in_link = rccl.RcclComm(store, "q/link1-2", 1, 0, "cuda:0", timeout_s=60)
    buf = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda")
    rcv = torch.empty_like(buf)
    for c in (out_link, in_link):
        c.p2p(sends=[(buf, 0)], recvs=[(rcv, 0)]).wait_host(timeout_s=30)
    side = torch.cuda.Stream()
    copy = lib.private_stream("cuda:0")
    t0 = time.perf_counter()
    ex.forward(0)
    torch.cuda.synchronize()
    alone = round((time.perf_counter() - t0) * 1e3, 2)
    rec = {"GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES"),
           "stage": {"alone_ms": alone,
                     "links": replay_while_spinning(ex, K, [out_link.stream, in_link.stream], 3.0),
                     "links_side_copy": replay_while_spinning(ex, K, [out_link.stream, in_link.stream, side, copy],
                                                              3.0)},
           "sweep": {}}
    for k in range(1, 9):
        rec["sweep"][k] = replay_while_spinning(ex, K, [torch.cuda.Stream() for _ in range(k)], 2.0)
    out_link.destroy()
    in_link.destroy()
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
