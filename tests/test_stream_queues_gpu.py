"""A pipeline stage's compute stream must not queue behind its link streams.

A stage process owns more HIP streams than the box's GPU_MAX_HW_QUEUES = 4
hardware queues: the compute stream (graph replays), the executor's private
capture stream, one stream per RCCL link (`parallel/rccl.py`), RCCL's own
internal streams, the codec's side stream and the serving copy stream.  Streams
beyond the queue count share queues, and a packet in a shared queue waits for
the packets ahead of it.  A receive posted for micro-batch t+2 that spins
until its upstream peer sends would then hold back compute(t+1) on a shared
queue, silently serialising the pipeline.

This test builds that stream set in the order a stage process creates it
(`parallel/runner.py` PipelineJob: executor + capture, then the two links, then
the codec side stream), parks a spinning kernel (`spin_flag`, a host-released
flag with a wall-clock bound, so it always ends) on every link stream, and
requires a ResNet-50 slice's graph replay on the compute stream to finish while
the spinners are still pending.

The reference's hop is a blocking TCP send from the worker's compute loop
(`src/node.py:163-179`), so its compute and transfer never overlap at all.
"""
import datetime
import time

import pytest
import torch

pytestmark = pytest.mark.gpu

PKG = "adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd"


def _spin(K, flag, out, stream, timeout_ms=8000.0):
    K.spin_flag(flag.data_ptr(), out.data_ptr(), timeout_ms, stream.cuda_stream)
    ev = torch.cuda.Event()
    ev.record(stream)
    return ev


def _replay_while_spinning(ex, K, spin_streams, wait_s=5.0):
    """Park a spinner on each stream, replay the slice on the current stream;
    returns (replay finished while every spinner was pending, replay seconds,
    spinner verdicts)."""
    flag = torch.zeros(1, dtype=torch.int32, pin_memory=True)
    outs = [torch.zeros(1, dtype=torch.int32, device="cuda") for _ in spin_streams]
    torch.cuda.synchronize()
    evs = [_spin(K, flag, o, s) for o, s in zip(outs, spin_streams)]
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
    flag.fill_(1)                                   # release the spinners
    torch.cuda.synchronize()
    verdicts = [int(o.item()) for o in outs]
    return finished and pending, dt, verdicts


@pytest.fixture(scope="module")
def stage():
    from importlib import import_module
    resnet = import_module(f"{PKG}.models.resnet")
    slicer = import_module(f"{PKG}.graph.slicer")
    executor = import_module(f"{PKG}.runtime.executor")
    g = resnet.build_resnet("resnet50")
    w = resnet.init_weights(g, seed=0)
    sl = slicer.partition(g, ["conv4_block1_out"])[1]            # the second half of a 2-stage cut
    ex = executor.SliceExecutor(slicer.subgraph(g, sl), w, 32, device="cuda:0", precision="fp32")
    ex.capture()
    return ex


def test_compute_runs_while_rccl_link_streams_spin(stage):
    from importlib import import_module
    rccl = import_module(f"{PKG}.parallel.rccl")
    K = import_module(f"{PKG}.ops._lib").kernels()
    if not rccl.available():
        pytest.fail("native RCCL layer (_comm) not loadable on a GPU box")
    store = torch.distributed.HashStore()
    # a stage's two links (world-1 communicators: same streams and RCCL resources, no peer needed)
    out_link = rccl.RcclComm(store, "q/link0-1", 1, 0, "cuda:0", timeout_s=60)
    in_link = rccl.RcclComm(store, "q/link1-2", 1, 0, "cuda:0", timeout_s=60)
    try:
        buf = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda")
        rcv = torch.empty_like(buf)
        for c in (out_link, in_link):             # materialise RCCL's per-communicator resources
            c.p2p(sends=[(buf, 0)], recvs=[(rcv, 0)]).wait_host(timeout_s=30)
        side = torch.cuda.Stream()                 # the codec side stream (CompressedStageLink)
        from importlib import import_module as im
        copy = im(f"{PKG}.ops._lib").private_stream("cuda:0")     # the serving H2D copy stream
        t_ref = time.perf_counter()
        stage.forward(0)
        torch.cuda.synchronize()
        t_ref = time.perf_counter() - t_ref
        ok, dt, verdicts = _replay_while_spinning(stage, K, [out_link.stream, in_link.stream])
        print(f"replay alone {t_ref * 1e3:.2f} ms; with both link streams spinning {dt * 1e3:.2f} ms, "
              f"spinners {verdicts}")
        assert verdicts == [1, 1], "a spinner timed out: the test's bound, not the flag, ended it"
        assert ok, f"compute waited for a spinning link stream (replay {dt:.3f} s)"
        ok2, dt2, v2 = _replay_while_spinning(stage, K, [out_link.stream, in_link.stream, side, copy])
        print(f"with links + codec side + copy streams spinning: {dt2 * 1e3:.2f} ms, spinners {v2}")
        assert v2 == [1, 1, 1, 1] and ok2, f"compute waited for a spinning auxiliary stream ({dt2:.3f} s)"
    finally:
        out_link.destroy()
        in_link.destroy()


def test_stream_count_sweep_reports_queue_sharing(stage):
    """Diagnostic: park spinners on k fresh streams (k = 1..8) and report whether
    the compute stream still runs.  Asserted for k <= 3 (fewer streams than
    hardware queues); larger k is printed for the record."""
    from importlib import import_module
    K = import_module(f"{PKG}.ops._lib").kernels()
    res = {}
    for k in range(1, 9):
        streams = [torch.cuda.Stream() for _ in range(k)]
        ok, dt, verdicts = _replay_while_spinning(stage, K, streams, wait_s=3.0)
        res[k] = (ok, round(dt * 1e3, 2))
        assert all(v == 1 for v in verdicts)
    print("spinning streams -> (compute finished, ms):", res)
    assert all(res[k][0] for k in (1, 2, 3)), res
