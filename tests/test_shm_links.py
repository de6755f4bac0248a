"""Same-host stage -> stage links through shared memory (transport/shm.py
LinkPool): the frontier goes into a slot, only a descriptor crosses the TCP
hop (the reference sends every activation through the socket,
`src/node.py:163-179`).  CPU workers in-process; the GPU path (device -> page-
locked slot -> device) is exercised by tests/test_shm_links_gpu.py.
"""
import os
import queue
import threading
import time

import numpy as np
import pytest

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.dispatcher import DEFER
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.model import resnet
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.node import Node
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.transport import shm

pytestmark = pytest.mark.skipif(not shm.available(), reason="no writable /dev/shm")


@pytest.fixture(scope="module")
def tiny():
    return resnet("resnet_tiny", input_shape=(32, 32, 3), classes=10, seed=5)


def _wait(pred, timeout=30.0):
    t0 = time.time()
    while time.time() - t0 < timeout:
        if pred():
            return True
        time.sleep(0.05)
    return False


def _links():
    """This process's link segments (xdist workers run other pipelines at the same time)."""
    return sorted(f for f in os.listdir(shm.SHM_DIR) if f.startswith(f"adapt-link-{os.getpid()}-"))


def _run(tiny, links, n_nodes=3, kill=False):
    d = DEFER(membership_port=0, result_port=0, worker_wait=20, ordered=True, batch=2, weight_codec="lz4",
              min_workers=n_nodes, replicas=1, links=links)
    d.membership_server.start()
    nodes = [Node(membership_port=d.membership_port, data_port=0, config_port=0, device="cpu",
                  node_id=f"{links}{i}", heartbeat_ttl=2.0) for i in range(n_nodes)]
    for nd in nodes:
        nd.run(block=False)
    before = set(_links())
    try:
        inq, outq = queue.Queue(), queue.Queue()
        cuts = ["conv3_block1_out", "conv4_block1_out"][: n_nodes - 1]
        threading.Thread(target=d.run_defer, args=(tiny, cuts, inq, outq), daemon=True).start()
        assert _wait(lambda: d.pipeline is not None)
        rng = np.random.default_rng(3)
        xs = [rng.standard_normal((2, 32, 32, 3)).astype(np.float32) for _ in range(16)]
        want = tiny.predict(np.concatenate(xs), device="cpu")
        for x in xs[:8]:
            inq.put(x)
        got = [outq.get(timeout=60) for _ in range(8)]
        stages = [next(nd for nd in nodes if nd.node_id == w) for w in d.pipeline.workers]
        info = [(nd.runtime.link, None if nd.runtime._linkpool is None else
                 (len(nd.runtime._linkpool._all), nd.runtime._linkpool.max_slots)) for nd in stages]
        if kill:
            e0 = d.pipeline.epoch
            stages[1].stop()                               # the middle stage: both its links break
            assert _wait(lambda: d.pipeline is not None and d.pipeline.epoch > e0)
        for x in xs[8:]:
            inq.put(x)
        got += [outq.get(timeout=60) for _ in range(8)]
        time.sleep(0.2)
        assert outq.empty()                                # exactly once
        np.testing.assert_allclose(np.concatenate(got), want, rtol=1e-4, atol=1e-5)
        return info, before
    finally:
        d.shutdown(stop_workers=True)
        for nd in nodes:
            nd.stop()


def test_same_host_hops_use_shared_memory_slots(tiny):
    info, before = _run(tiny, "auto")
    assert [lk for lk, _ in info] == ["shm", "shm", "tcp"]       # the last hop goes to the dispatcher
    for _, (n_slots, max_slots) in info[:2]:
        assert 1 <= n_slots <= max_slots                        # slots are recycled, not one per request
    assert set(_links()) <= before                              # every link segment unlinked at shutdown


def test_links_tcp_keeps_frontier_on_the_socket(tiny):
    info, _ = _run(tiny, "tcp")
    assert [lk for lk, _ in info] == ["tcp", "tcp", "tcp"] and all(p is None for _, p in info)


def test_shm_link_survives_a_stage_kill(tiny):
    info, before = _run(tiny, "auto", n_nodes=3, kill=True)
    assert info[0][0] == "shm"
    assert set(_links()) <= before


def test_link_pool_handoff_flag():
    pool = shm.LinkPool(max_slots=2)
    try:
        a = pool.put(np.arange(6, dtype=np.float32))
        b = pool.put(np.arange(6, dtype=np.float32) + 1)
        assert a.slot is not b.slot and a.slot.mm[0] == 1 and b.slot.mm[0] == 1
        stop = threading.Event()
        stop.set()
        with pytest.raises(RuntimeError):                     # both in flight: the sender waits
            pool.acquire(24, stop)
        name = a.slot.name
        np.testing.assert_array_equal(shm.view(name, shm.LINK_HDR, np.float32, (6,)), np.arange(6))
        shm.release(name)                                     # receiver side: copy done
        c = pool.acquire(24)
        assert c is a.slot
        shm.detach([name])
    finally:
        pool.close()


def test_release_after_detach_is_a_no_op():
    pool = shm.LinkPool(max_slots=1)
    try:
        a = pool.put(np.arange(4, dtype=np.float32))
        name = a.slot.name
        np.testing.assert_array_equal(shm.view(name, shm.LINK_HDR, np.float32, (4,)), np.arange(4))
        shm.detach([name])
        shm.release(name)                                     # late release of a torn-down epoch's slot
        assert name not in shm._attached                      # not mapped again
        assert a.slot.mm[0] == 1                              # and the sender's flag is untouched
    finally:
        pool.close()


def test_device_link_descriptor_roundtrip():
    """The "dev" container carries a device link slot's name and offset; the receiver
    decodes it to a DevArray (its device address is resolved lazily on the GPU)."""
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd import codec as C
    buf = C.wrap(b"adapt-link-1-e2-s0-abc-3\0" + (256).to_bytes(8, "little"), "dev", np.uint16, (4, 28, 28, 128),
                 bf16=True)
    a = C.decode(buf, copy=False)
    assert isinstance(a, shm.DevArray)
    assert (a.name, a.offset, a.dtype, a.shape) == ("adapt-link-1-e2-s0-abc-3", 256, np.dtype(np.uint16),
                                                    (4, 28, 28, 128))
    assert a.nbytes == 4 * 28 * 28 * 128 * 2
    assert C.codec_of(buf) == "dev" and C.is_bf16(buf) and C.shm_name(buf) == a.name and shm.is_link(a.name)


def test_full_dev_shm_raises_instead_of_sigbus(monkeypatch):
    """tmpfs accepts an ftruncate past its size limit and SIGBUSes on the first
    write; segments are reserved with posix_fallocate, so a full /dev/shm is a
    ShmFull exception (the dispatcher then sends the request inline)."""
    import errno
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.transport import shm

    def enospc(fd, off, n):
        raise OSError(errno.ENOSPC, "No space left on device")

    monkeypatch.setattr(shm.os, "posix_fallocate", enospc)
    pool = shm.ShmPool()
    with pytest.raises(shm.ShmFull):
        pool.put(np.zeros((4, 1024), np.float32))
    assert not [f for f in os.listdir(shm.SHM_DIR) if f.startswith(pool.prefix)]      # nothing left behind
    lp = shm.LinkPool()
    with pytest.raises(shm.ShmFull):
        lp.acquire(4096)
    monkeypatch.undo()
    s = lp.acquire(4096)                        # space again: the link works
    assert s.nbytes == 4096
    lp.close()
    pool.close()


def test_dispatcher_ingest_falls_back_inline_when_shm_full(tiny, monkeypatch):
    import errno
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.transport import shm

    def enospc(fd, off, n):
        raise OSError(errno.ENOSPC, "No space left on device")

    d = DEFER(membership_port=0, result_port=0, worker_wait=10, batch=2, weight_codec="lz4")
    d.membership_server.start()
    node = Node(membership_port=d.membership_port, data_port=0, config_port=0, device="cpu", node_id="f0",
                heartbeat_ttl=1.0)
    node.run(block=False)
    try:
        monkeypatch.setattr(shm.os, "posix_fallocate", enospc)
        inq, outq = queue.Queue(), queue.Queue()
        threading.Thread(target=d.run_defer, args=(tiny, [], inq, outq), daemon=True).start()
        x = np.random.default_rng(0).standard_normal((2, 32, 32, 3)).astype(np.float32)
        inq.put(x)
        y = outq.get(timeout=60)
        np.testing.assert_allclose(y, tiny.predict(x, device="cpu"), rtol=1e-4, atol=1e-5)
        assert any("fell back to inline" in e for _, e in d.events)
    finally:
        d.shutdown(stop_workers=True)
        node.stop()
