"""Membership client (the reference's `etcd3.client(host, port=2379)`,
`src/node_state.py:18`) plus the worker-side registration helper that the
reference never wrote: a leased ``/workers/{id}`` record kept alive by a
heartbeat thread (SURVEY §5.3 "New (MI355X)")."""
from __future__ import annotations

import base64
import json
import socket
import threading
from typing import Callable, Dict, List, Optional

from ..node_state import socket_recv, socket_send
from .store import Event, KeyValue, KVStore

CHUNK = 1 << 16


class MembershipError(RuntimeError):
    """The server rejected a request."""


def _kv(d) -> Optional[KeyValue]:
    if d is None:
        return None
    return KeyValue(d["key"], base64.b64decode(d["value"]), d["create_revision"], d["mod_revision"],
                    d["version"], d.get("lease", 0))


class MembershipClient:
    """Blocking request/response client; thread-safe (one lock per connection)."""

    def __init__(self, host: str = "127.0.0.1", port: int = 2379, timeout: float = 5.0):
        self.host, self.port, self.timeout = host, port, timeout
        self._lock = threading.Lock()
        self._sock: Optional[socket.socket] = None

    def _conn(self) -> socket.socket:
        if self._sock is None:
            s = socket.create_connection((self.host, self.port), timeout=self.timeout)
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            self._sock = s
        return self._sock

    def _call(self, **req) -> dict:
        with self._lock:
            resp = None
            for attempt in range(2):        # one transparent reconnect
                try:
                    s = self._conn()
                    socket_send(json.dumps(req).encode(), s, CHUNK, int(self.timeout * 1000))
                    raw = socket_recv(s, CHUNK, int(self.timeout * 1000))
                    if not raw:
                        raise ConnectionError("membership server closed the connection")
                    resp = json.loads(raw)
                    break
                except (OSError, ConnectionError, RuntimeError):
                    self.close()
                    if attempt:
                        raise ConnectionError(f"membership service {self.host}:{self.port} unreachable")
            if not resp.get("ok"):
                raise MembershipError(resp.get("error", "membership error"))
            return resp

    def close(self) -> None:
        if self._sock is not None:
            try:
                self._sock.close()
            except OSError:
                pass
            self._sock = None

    # ----------------------------------------------------------- KV API
    def put(self, key: str, value, lease: Optional[int] = None) -> int:
        if isinstance(value, str):
            value = value.encode()
        return self._call(op="put", key=key, value=base64.b64encode(value).decode(), lease=lease or 0)["revision"]

    def get(self, key: str) -> Optional[KeyValue]:
        return _kv(self._call(op="get", key=key)["kv"])

    def get_prefix(self, prefix: str) -> List[KeyValue]:
        return [_kv(d) for d in self._call(op="get_prefix", prefix=prefix)["kvs"]]

    def delete(self, key: str) -> bool:
        return self._call(op="delete", key=key)["deleted"]

    def delete_prefix(self, prefix: str) -> int:
        return self._call(op="delete_prefix", prefix=prefix)["deleted"]

    def compare_and_swap(self, key: str, expected: Optional[bytes], value, lease: Optional[int] = None):
        if isinstance(value, str):
            value = value.encode()
        r = self._call(op="cas", key=key, expected=None if expected is None else base64.b64encode(expected).decode(),
                       value=base64.b64encode(value).decode(), lease=lease or 0)
        return r["swapped"], r["revision"]

    def lease_grant(self, ttl: float) -> int:
        return self._call(op="lease_grant", ttl=ttl)["lease"]

    def lease_keepalive(self, lease: int) -> float:
        return self._call(op="lease_keepalive", lease=lease)["ttl"]

    def lease_revoke(self, lease: int) -> bool:
        return self._call(op="lease_revoke", lease=lease)["revoked"]

    @property
    def revision(self) -> int:
        return self._call(op="status")["revision"]

    # ------------------------------------------------------------ watch
    def watch(self, prefix: str, callback: Callable[[Event], None], start_revision: Optional[int] = None) -> "RemoteWatch":
        return RemoteWatch(self.host, self.port, prefix, callback, start_revision)


class RemoteWatch:
    """A dedicated connection streaming watch events to `callback` on a thread."""

    def __init__(self, host, port, prefix, callback, start_revision=None):
        self.sock = socket.create_connection((host, port), timeout=5.0)
        self.sock.settimeout(None)
        req = {"op": "watch", "prefix": prefix}
        if start_revision is not None:
            req["start_revision"] = start_revision
        socket_send(json.dumps(req).encode(), self.sock, CHUNK)
        ack = json.loads(socket_recv(self.sock, CHUNK))
        self.revision = ack.get("revision")
        self.callback = callback
        self._stop = threading.Event()
        self.thread = threading.Thread(target=self._loop, daemon=True, name=f"watch:{prefix}")
        self.thread.start()

    def _loop(self):
        try:
            while not self._stop.is_set():
                raw = socket_recv(self.sock, CHUNK)
                if not raw:
                    break
                d = json.loads(raw)
                self.callback(Event(d["type"], _kv(d["kv"]), _kv(d.get("prev"))))
        except (OSError, RuntimeError, ValueError):
            pass

    def cancel(self):
        self._stop.set()
        try:
            self.sock.shutdown(socket.SHUT_RDWR)
        except OSError:
            pass
        self.sock.close()


class Registration:
    """Leased ``/workers/{id}`` record with a keepalive heartbeat.

    If the process dies the heartbeats stop, the lease expires after `ttl`
    seconds and the key disappears -> the dispatcher's watch sees a DELETE.
    `client` may be a `MembershipClient` or an in-process `KVStore`.
    """

    def __init__(self, client, worker_id: str, record: Dict, ttl: float = 1.0, prefix: str = "/workers/"):
        self.client = client
        self.key = prefix + worker_id
        self.ttl = ttl
        self.record = dict(record)
        self.lease = client.lease_grant(ttl)
        self._stop = threading.Event()
        self._lock = threading.Lock()
        self.put()
        self.thread = threading.Thread(target=self._beat, daemon=True, name=f"keepalive:{worker_id}")
        self.thread.start()

    def put(self, **updates) -> None:
        with self._lock:
            self.record.update(updates)
            self.client.put(self.key, json.dumps(self.record).encode(), lease=self.lease)

    def _beat(self) -> None:
        period = self.ttl / 3.0
        while not self._stop.wait(period):
            try:
                if self.client.lease_keepalive(self.lease) < 0:
                    # lease lost (e.g. we were partitioned away): re-register
                    self.lease = self.client.lease_grant(self.ttl)
                    self.put()
            except (OSError, ConnectionError, RuntimeError):
                continue

    def close(self, revoke: bool = True) -> None:
        self._stop.set()
        if revoke:
            try:
                self.client.lease_revoke(self.lease)
            except (OSError, ConnectionError, RuntimeError):
                pass


def live_workers(client, prefix: str = "/workers/") -> Dict[str, dict]:
    out = {}
    for kv in client.get_prefix(prefix):
        try:
            out[kv.key[len(prefix):]] = json.loads(kv.value)
        except ValueError:
            continue
    return out
