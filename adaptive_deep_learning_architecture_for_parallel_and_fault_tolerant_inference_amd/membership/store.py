"""etcd-style membership store: revisioned KV + TTL leases + prefix watches.

The reference relies on an external etcd v3 server (`src/start_etcd.sh`,
`src/node_state.py:16-20`) for the ``/workers/{ip}`` registry that drives
worker discovery (`src/dispatcher.py:282-295`) — etcd is neither installed
nor downloadable here, so this module implements the
subset of etcd v3 semantics the system needs:

* monotonically increasing store revision; every key carries
  create/mod revisions and a version,
* ``put / get / get_prefix / delete / delete_prefix``,
* ``compare_and_swap`` (a one-key txn) for epoch bumps,
* leases: ``lease_grant(ttl)``, ``lease_keepalive``, ``lease_revoke``; keys
  attached to an expired/revoked lease are deleted (DELETE events fire),
* watches on a key prefix from a start revision, delivered in revision
  order through a queue (history is kept for replay).

It is used in-process by tests and by the dispatcher, and served over TCP by
`membership.server` for worker processes.
"""
from __future__ import annotations

import itertools
import queue
import threading
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Tuple


@dataclass
class KeyValue:
    key: str
    value: bytes
    create_revision: int
    mod_revision: int
    version: int
    lease: int = 0


@dataclass
class Event:
    type: str              # "PUT" | "DELETE"
    kv: KeyValue
    prev: Optional[KeyValue] = None


@dataclass
class Lease:
    id: int
    ttl: float
    expiry: float
    keys: set = field(default_factory=set)


class Watch:
    def __init__(self, store: "KVStore", prefix: str, wid: int):
        self.store = store
        self.prefix = prefix
        self.id = wid
        self.events: "queue.Queue[Event]" = queue.Queue()
        self.cancelled = False

    def get(self, timeout: Optional[float] = None) -> Optional[Event]:
        try:
            return self.events.get(timeout=timeout)
        except queue.Empty:
            return None

    def cancel(self) -> None:
        self.cancelled = True
        self.store._remove_watch(self)


class KVStore:
    def __init__(self, clock: Callable[[], float] = time.monotonic, expiry_interval: float = 0.05,
                 history: int = 100000, start_expiry_thread: bool = True):
        self._lock = threading.RLock()
        self._kv: Dict[str, KeyValue] = {}
        self._rev = 0
        self._leases: Dict[int, Lease] = {}
        self._lease_ids = itertools.count(0x1000)
        self._watch_ids = itertools.count(1)
        self._watches: List[Watch] = []
        self._history: List[Event] = []
        self._history_max = history
        self._clock = clock
        self._closed = threading.Event()
        self._expiry_interval = expiry_interval
        if start_expiry_thread:
            threading.Thread(target=self._expiry_loop, daemon=True, name="kv-lease-expiry").start()

    # ---------------------------------------------------------- internals
    def _emit(self, ev: Event) -> None:
        self._history.append(ev)
        if len(self._history) > self._history_max:
            del self._history[: len(self._history) - self._history_max]
        for w in list(self._watches):
            if ev.kv.key.startswith(w.prefix):
                w.events.put(ev)

    def _remove_watch(self, w: Watch) -> None:
        with self._lock:
            if w in self._watches:
                self._watches.remove(w)

    @property
    def revision(self) -> int:
        with self._lock:
            return self._rev

    # ------------------------------------------------------------- KV ops
    def put(self, key: str, value: bytes, lease: int = 0) -> int:
        if isinstance(value, str):
            value = value.encode()
        with self._lock:
            if lease and lease not in self._leases:
                raise KeyError(f"lease {lease:#x} not found")
            self._rev += 1
            prev = self._kv.get(key)
            if prev is not None and prev.lease and prev.lease != lease and prev.lease in self._leases:
                self._leases[prev.lease].keys.discard(key)
            kv = KeyValue(key, bytes(value), prev.create_revision if prev else self._rev, self._rev,
                          (prev.version + 1) if prev else 1, lease)
            self._kv[key] = kv
            if lease:
                self._leases[lease].keys.add(key)
            self._emit(Event("PUT", kv, prev))
            return self._rev

    def get(self, key: str) -> Optional[KeyValue]:
        with self._lock:
            return self._kv.get(key)

    def get_prefix(self, prefix: str) -> List[KeyValue]:
        with self._lock:
            return [self._kv[k] for k in sorted(self._kv) if k.startswith(prefix)]

    def _delete_locked(self, key: str) -> bool:
        prev = self._kv.pop(key, None)
        if prev is None:
            return False
        self._rev += 1
        if prev.lease and prev.lease in self._leases:
            self._leases[prev.lease].keys.discard(key)
        self._emit(Event("DELETE", KeyValue(key, b"", prev.create_revision, self._rev, 0, 0), prev))
        return True

    def delete(self, key: str) -> bool:
        with self._lock:
            return self._delete_locked(key)

    def delete_prefix(self, prefix: str) -> int:
        with self._lock:
            keys = [k for k in self._kv if k.startswith(prefix)]
            for k in keys:
                self._delete_locked(k)
            return len(keys)

    def compare_and_swap(self, key: str, expected: Optional[bytes], value: bytes, lease: int = 0) -> Tuple[bool, int]:
        """Put `value` iff the current value equals `expected` (None = key absent)."""
        if isinstance(value, str):
            value = value.encode()
        with self._lock:
            cur = self._kv.get(key)
            curv = cur.value if cur else None
            if curv != expected:
                return False, self._rev
            return True, self.put(key, value, lease)

    # ------------------------------------------------------------- leases
    def lease_grant(self, ttl: float) -> int:
        with self._lock:
            lid = next(self._lease_ids)
            self._leases[lid] = Lease(lid, float(ttl), self._clock() + float(ttl))
            return lid

    def lease_keepalive(self, lid: int) -> float:
        """Refresh a lease; returns its TTL, or -1 if it no longer exists."""
        with self._lock:
            L = self._leases.get(lid)
            if L is None:
                return -1.0
            L.expiry = self._clock() + L.ttl
            return L.ttl

    def lease_ttl(self, lid: int) -> float:
        with self._lock:
            L = self._leases.get(lid)
            return -1.0 if L is None else max(0.0, L.expiry - self._clock())

    def lease_revoke(self, lid: int) -> bool:
        with self._lock:
            L = self._leases.pop(lid, None)
            if L is None:
                return False
            for k in sorted(L.keys):
                kv = self._kv.get(k)
                if kv is not None and kv.lease == lid:
                    self._delete_locked(k)
            return True

    def expire_leases(self) -> List[int]:
        now = self._clock()
        with self._lock:
            dead = [lid for lid, L in self._leases.items() if L.expiry <= now]
            for lid in dead:
                self.lease_revoke(lid)
            return dead

    def _expiry_loop(self) -> None:
        while not self._closed.wait(self._expiry_interval):
            self.expire_leases()

    # ------------------------------------------------------------ watches
    def watch(self, prefix: str, start_revision: Optional[int] = None) -> Watch:
        """Watch `prefix`; with `start_revision`, replay history events with
        revision >= start_revision first (etcd semantics)."""
        with self._lock:
            w = Watch(self, prefix, next(self._watch_ids))
            if start_revision is not None:
                for ev in self._history:
                    if ev.kv.mod_revision >= start_revision and ev.kv.key.startswith(prefix):
                        w.events.put(ev)
            self._watches.append(w)
            return w

    def close(self) -> None:
        self._closed.set()
        with self._lock:
            self._watches.clear()
