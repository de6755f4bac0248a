"""etcd-style membership store / server / client (CPU)."""
import json
import threading
import time

import pytest

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.membership.client import (
    MembershipClient, MembershipError, Registration, live_workers)
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.membership.server import MembershipServer
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.membership.store import KVStore


class FakeClock:
    def __init__(self):
        self.t = 0.0

    def __call__(self):
        return self.t


def test_revisions_and_versions():
    s = KVStore(start_expiry_thread=False)
    r1 = s.put("/a", b"1")
    r2 = s.put("/a", b"2")
    kv = s.get("/a")
    assert r2 == r1 + 1 and kv.version == 2 and kv.create_revision == r1 and kv.mod_revision == r2
    s.put("/b/x", b"x")
    s.put("/b/y", b"y")
    assert [k.key for k in s.get_prefix("/b/")] == ["/b/x", "/b/y"]
    assert s.delete_prefix("/b/") == 2 and s.get_prefix("/b/") == []
    assert s.delete("/a") and not s.delete("/a")


def test_lease_expiry_deletes_keys_and_fires_watch():
    clk = FakeClock()
    s = KVStore(clock=clk, start_expiry_thread=False)
    w = s.watch("/workers/")
    lid = s.lease_grant(1.0)
    s.put("/workers/w0", b"{}", lease=lid)
    s.put("/workers/w1", b"{}", lease=s.lease_grant(5.0))
    clk.t = 0.9
    assert s.lease_keepalive(lid) == 1.0           # refreshed -> expires at 1.9
    clk.t = 1.5
    assert s.expire_leases() == []
    clk.t = 2.0
    assert s.expire_leases() == [lid]
    assert s.get("/workers/w0") is None and s.get("/workers/w1") is not None
    evs = [w.get(0) for _ in range(3)]
    assert [(e.type, e.kv.key) for e in evs] == [("PUT", "/workers/w0"), ("PUT", "/workers/w1"),
                                                ("DELETE", "/workers/w0")]
    assert s.lease_keepalive(lid) == -1.0


def test_watch_history_replay_and_cas():
    s = KVStore(start_expiry_thread=False)
    r = s.put("/p/epoch", b"1")
    s.put("/p/epoch", b"2")
    w = s.watch("/p/", start_revision=r)
    assert [w.get(0).kv.value for _ in range(2)] == [b"1", b"2"]
    ok, _ = s.compare_and_swap("/p/epoch", b"2", b"3")
    bad, _ = s.compare_and_swap("/p/epoch", b"2", b"4")
    assert ok and not bad and s.get("/p/epoch").value == b"3"
    assert s.compare_and_swap("/p/new", None, b"x")[0]


def test_server_client_roundtrip_and_registration():
    srv = MembershipServer(port=0).start()
    try:
        c = MembershipClient(port=srv.port)
        assert c.put("/k", b"v") > 0 and c.get("/k").value == b"v"
        assert c.get("/missing") is None
        events = []
        got = threading.Event()

        def cb(ev):
            events.append((ev.type, ev.kv.key))
            if ev.type == "DELETE":
                got.set()

        w = c.watch("/workers/", cb)
        reg = Registration(MembershipClient(port=srv.port), "gpu3", {"device": "cuda:3"}, ttl=0.3)
        time.sleep(0.5)                                   # > ttl: keepalive must hold the key
        assert live_workers(c) == {"gpu3": {"device": "cuda:3"}}
        reg.put(state="BUSY")
        assert json.loads(c.get("/workers/gpu3").value)["state"] == "BUSY"
        reg.close(revoke=False)                           # crash: heartbeats stop
        assert got.wait(3.0)
        assert live_workers(c) == {}
        assert ("PUT", "/workers/gpu3") in events and events[-1] == ("DELETE", "/workers/gpu3")
        w.cancel()
        with pytest.raises(MembershipError):
            c.put("/x", b"y", lease=12345)                # unknown lease
    finally:
        srv.stop()
