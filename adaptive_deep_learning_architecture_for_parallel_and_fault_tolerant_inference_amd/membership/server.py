"""TCP front-end for the membership store (our stand-in for the etcd server
the reference launches with `src/start_etcd.sh` on port 2379).

Protocol: framed messages (8-byte BE length, the same framing as the data
plane, csrc/runtime/framing.cpp) carrying JSON objects.  Request
``{"op": ..., **args}`` -> response ``{"ok": bool, ...}``; values travel
base64-encoded.  A ``watch`` request turns its connection into an event
stream (one JSON event per frame) until the client closes it.

Run standalone:  python -m <pkg>.membership.server --port 2379
"""
from __future__ import annotations

import argparse
import base64
import json
import socket
import threading
import time
from typing import Optional

from ..node_state import socket_recv, socket_send
from .store import Event, KeyValue, KVStore

CHUNK = 1 << 16


def kv_to_json(kv: Optional[KeyValue]):
    if kv is None:
        return None
    return {"key": kv.key, "value": base64.b64encode(kv.value).decode(), "create_revision": kv.create_revision,
            "mod_revision": kv.mod_revision, "version": kv.version, "lease": kv.lease}


def ev_to_json(ev: Event):
    return {"type": ev.type, "kv": kv_to_json(ev.kv), "prev": kv_to_json(ev.prev)}


class MembershipServer:
    def __init__(self, store: Optional[KVStore] = None, host: str = "0.0.0.0", port: int = 2379):
        self.store = store or KVStore()
        self.sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self.sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self.sock.bind((host, port))
        self.sock.listen(128)
        self.port = self.sock.getsockname()[1]
        self._stop = threading.Event()
        self._conns = set()
        self._thread = threading.Thread(target=self._accept_loop, daemon=True, name="membership-accept")

    def start(self) -> "MembershipServer":
        self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        try:
            self.sock.close()
        except OSError:
            pass
        for c in list(self._conns):
            try:
                c.shutdown(socket.SHUT_RDWR)
                c.close()
            except OSError:
                pass

    def _accept_loop(self) -> None:
        while not self._stop.is_set():
            try:
                conn, _ = self.sock.accept()
            except OSError:
                break
            conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            self._conns.add(conn)
            threading.Thread(target=self._serve, args=(conn,), daemon=True, name="membership-conn").start()

    def _handle(self, req: dict) -> dict:
        s = self.store
        op = req.get("op")
        if op == "put":
            rev = s.put(req["key"], base64.b64decode(req["value"]), int(req.get("lease") or 0))
            return {"ok": True, "revision": rev}
        if op == "get":
            return {"ok": True, "kv": kv_to_json(s.get(req["key"])), "revision": s.revision}
        if op == "get_prefix":
            return {"ok": True, "kvs": [kv_to_json(k) for k in s.get_prefix(req["prefix"])], "revision": s.revision}
        if op == "delete":
            return {"ok": True, "deleted": s.delete(req["key"])}
        if op == "delete_prefix":
            return {"ok": True, "deleted": s.delete_prefix(req["prefix"])}
        if op == "cas":
            exp = req.get("expected")
            ok, rev = s.compare_and_swap(req["key"], None if exp is None else base64.b64decode(exp),
                                         base64.b64decode(req["value"]), int(req.get("lease") or 0))
            return {"ok": True, "swapped": ok, "revision": rev}
        if op == "lease_grant":
            return {"ok": True, "lease": s.lease_grant(float(req["ttl"]))}
        if op == "lease_keepalive":
            return {"ok": True, "ttl": s.lease_keepalive(int(req["lease"]))}
        if op == "lease_revoke":
            return {"ok": True, "revoked": s.lease_revoke(int(req["lease"]))}
        if op == "lease_ttl":
            return {"ok": True, "ttl": s.lease_ttl(int(req["lease"]))}
        if op == "status":
            return {"ok": True, "revision": s.revision, "time": time.time()}
        return {"ok": False, "error": f"unknown op {op!r}"}

    def _serve(self, conn: socket.socket) -> None:
        try:
            while not self._stop.is_set():
                raw = socket_recv(conn, CHUNK)
                if not raw:
                    break
                req = json.loads(raw)
                if req.get("op") == "watch":
                    self._stream_watch(conn, req)
                    break
                try:
                    resp = self._handle(req)
                except Exception as e:      # report, keep serving
                    resp = {"ok": False, "error": f"{type(e).__name__}: {e}"}
                socket_send(json.dumps(resp).encode(), conn, CHUNK)
        except (OSError, RuntimeError, ValueError):
            pass
        finally:
            self._conns.discard(conn)
            try:
                conn.close()
            except OSError:
                pass

    def _stream_watch(self, conn: socket.socket, req: dict) -> None:
        w = self.store.watch(req["prefix"], req.get("start_revision"))
        socket_send(json.dumps({"ok": True, "watch_id": w.id, "revision": self.store.revision}).encode(), conn, CHUNK)
        # detect client close: a reader thread that returns when recv sees EOF
        closed = threading.Event()

        def reader():
            try:
                while socket_recv(conn, CHUNK):
                    pass
            except (OSError, RuntimeError):
                pass
            closed.set()

        threading.Thread(target=reader, daemon=True).start()
        try:
            while not closed.is_set() and not self._stop.is_set():
                ev = w.get(timeout=0.1)
                if ev is None:
                    continue
                socket_send(json.dumps(ev_to_json(ev)).encode(), conn, CHUNK)
        except (OSError, RuntimeError):
            pass
        finally:
            w.cancel()


def main(argv=None):
    ap = argparse.ArgumentParser(description="ADAPT membership service (etcd-style KV, leases, watch)")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=2379)
    a = ap.parse_args(argv)
    srv = MembershipServer(host=a.host, port=a.port).start()
    print(f"membership service listening on {a.host}:{srv.port}", flush=True)
    try:
        while True:
            time.sleep(3600)
    except KeyboardInterrupt:
        srv.stop()


if __name__ == "__main__":
    main()
