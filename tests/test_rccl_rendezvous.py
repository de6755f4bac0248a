"""CPU tests of the pipeline's RCCL rendezvous (`parallel/rccl.py` PairLinks)
with a fake `_comm` module: 8 threads play the 8 stages of a pipeline.

The reference forwards activations over TCP with a fresh connection per hop
(`src/dispatcher.py:204-220`), so it has no rendezvous to deadlock.  Here each
adjacent stage pair shares a 2-rank RCCL communicator whose unique id is
published by the upstream rank over the job's store; the non-blocking init
only completes once both ranks joined.  These tests check, without a GPU, that
no start order of the stages can deadlock the 8-stage start, that a stage
whose peer never arrives fails within its timeout, and that a half-built pair
is aborted instead of leaking.
"""
import datetime
import itertools
import random
import threading
import time

import pytest
import torch

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.parallel import rccl


class _FakeComm:
    """Non-blocking communicator: construction returns at once, `wait_ready`
    completes when every rank of the unique id has constructed its handle."""

    registry = {}
    lock = threading.Condition()
    created = []

    def __init__(self, uid, nranks, rank, dev, blocking, name):
        self.uid, self.nranks, self.rank, self.name = bytes(uid), nranks, rank, name
        self.aborted = False
        self.failed = False
        self.error_text = ""
        self.init_ms = 0.0
        with _FakeComm.lock:
            _FakeComm.registry.setdefault(self.uid, set()).add(rank)
            _FakeComm.created.append(self)
            _FakeComm.lock.notify_all()

    def start_watch(self, us, abort_on_error):
        pass

    def wait_ready(self, timeout_s):
        t0 = time.monotonic()
        with _FakeComm.lock:
            ok = _FakeComm.lock.wait_for(
                lambda: self.aborted or len(_FakeComm.registry[self.uid]) == self.nranks, timeout_s)
        if self.aborted:
            raise RuntimeError("rccl_p2p: communicator aborted")
        if not ok:
            raise RuntimeError(f"rccl_p2p: init not complete after {timeout_s} s")
        self.init_ms = (time.monotonic() - t0) * 1e3

    def abort(self):
        with _FakeComm.lock:
            self.aborted = True
            _FakeComm.lock.notify_all()
        return 0.0


class _FakeModule:
    Comm = _FakeComm

    @staticmethod
    def unique_id():
        return random.getrandbits(128 * 8).to_bytes(128, "little")


class _FakeStream:
    def __init__(self, device=None):
        self.device = device


@pytest.fixture
def fake_comm(monkeypatch):
    monkeypatch.setattr(rccl, "native", lambda: _FakeModule)
    monkeypatch.setattr(torch.cuda, "Stream", _FakeStream)
    _FakeComm.registry.clear()
    _FakeComm.created.clear()
    yield _FakeComm


def _start_pipeline(store, order, stages=8, delays=None, timeout_s=20.0, prefix="pp8/job1", missing=()):
    """Start the stages' PairLinks in `order` (thread start order, optional
    per-stage start delays); returns {stage: PairLinks or exception}."""
    out = {}

    def run(r):
        if delays:
            time.sleep(delays[r])
        prev = r - 1 if r > 0 else None
        nxt = r + 1 if r < stages - 1 else None
        try:
            out[r] = rccl.PairLinks(store, prefix, r, prev, nxt, f"cuda:{r}", timeout_s=timeout_s, watch_us=0)
        except Exception as e:  # noqa: BLE001 - reported to the test
            out[r] = e

    ts = {r: threading.Thread(target=run, args=(r,), daemon=True) for r in order if r not in missing}
    for r in order:
        if r in ts:
            ts[r].start()
    for t in ts.values():
        t.join(timeout_s + 10)
        assert not t.is_alive(), "a stage is still blocked in the rendezvous"
    return out


@pytest.mark.parametrize("order", [list(range(8)), list(range(7, -1, -1)), [3, 7, 0, 5, 1, 6, 2, 4]])
def test_eight_stage_rendezvous_any_start_order(fake_comm, order):
    store = torch.distributed.HashStore()
    out = _start_pipeline(store, order)
    for r in range(8):
        links = out[r]
        assert isinstance(links, rccl.PairLinks), links
        assert (links.inp is None) == (r == 0) and (links.out is None) == (r == 7)
    # every adjacent pair shares one communicator uid, upstream is comm rank 0
    for r in range(7):
        a, b = out[r].out._c, out[r + 1].inp._c
        assert a.uid == b.uid and a.rank == 0 and b.rank == 1
    assert len({c.uid for c in fake_comm.created}) == 7


def test_rendezvous_random_orders_and_delays(fake_comm):
    rng = random.Random(7)
    for trial in range(12):
        order = list(range(8))
        rng.shuffle(order)
        delays = [rng.random() * 0.05 for _ in range(8)]
        store = torch.distributed.HashStore()
        out = _start_pipeline(store, order, delays=delays, prefix=f"pp8/trial{trial}")
        assert all(isinstance(out[r], rccl.PairLinks) for r in range(8)), (order, out)


def test_missing_peer_times_out_and_aborts_half_built_links(fake_comm):
    """Stage 4 never arrives: stage 3's out-link and stage 5's in-link cannot
    form.  Both fail within the timeout, and stage 3's already-created
    in-link / stage 5's out-link are aborted rather than leaked."""
    store = torch.distributed.HashStore()
    store.set_timeout(datetime.timedelta(seconds=2))
    t0 = time.monotonic()
    out = _start_pipeline(store, list(range(8)), timeout_s=1.0, missing=(4,))
    assert time.monotonic() - t0 < 15
    assert isinstance(out[3], Exception) and isinstance(out[5], Exception)
    for r in (0, 1, 2, 6, 7):
        assert isinstance(out[r], rccl.PairLinks), out[r]
    names = {c.name: c for c in fake_comm.created}
    # stage 3 built link2-3 (its in-link) and link3-4 (its out-link): both aborted
    assert names["pp8/job1/link3-4"].aborted
    stage3_in = [c for c in fake_comm.created if c.name == "pp8/job1/link2-3" and c.rank == 1]
    assert stage3_in and all(c.aborted for c in stage3_in)


def test_pairs_from_itertools_cover_every_two_stage_order(fake_comm):
    """Two stages, both start orders, with the downstream stage first."""
    for order in itertools.permutations(range(2)):
        store = torch.distributed.HashStore()
        out = _start_pipeline(store, list(order), stages=2, prefix=f"pp2/{order}")
        assert isinstance(out[0], rccl.PairLinks) and isinstance(out[1], rccl.PairLinks)


def test_loopback_communicator_is_opt_in_only(monkeypatch):
    """The one-GPU stand-in for RCCL links (parallel/loopback_comm.py) is chosen only by the explicit
    test flag: unset, any other value, or a missing RCCL never select it."""
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.parallel import \
        loopback_comm
    monkeypatch.delenv(loopback_comm.ENV_FLAG, raising=False)
    assert not loopback_comm.selected()
    for v in ("0", "true", "yes", ""):
        monkeypatch.setenv(loopback_comm.ENV_FLAG, v)
        assert not loopback_comm.selected()
    monkeypatch.setenv(loopback_comm.ENV_FLAG, "1")
    assert loopback_comm.selected()
