"""Worker state + framed socket helpers (public API of `src/node_state.py`).

* `socket_send(bytes, sock, chunk_size)` / `socket_recv(sock, chunk_size)`:
  same wire format as the reference (`src/node_state.py:39-161`): an 8-byte
  big-endian length header, then the body in `chunk_size` pieces; works on
  blocking and non-blocking sockets; `b''` on a clean EOF before the header,
  an error on a truncated frame.  The loops run natively without the GIL
  (csrc/runtime/framing.cpp).
* `NodeState(chunk_size, dispatcher_ip)`: per-worker state with the locked
  `chunk_size` / `next_node` properties and a state enum, registered with the
  membership service under ``/workers/{id}`` (the reference creates an etcd
  client and key but never writes it, `src/node_state.py:16-20`; we hold a
  lease with keepalive).
* `StateEnum`: IDLE=0, BUSY=1, UNKNOWN=2, PARSE_ERROR=3 (`src/node_state.py:164-168`).
"""
from __future__ import annotations

import json
import socket
import threading
from enum import Enum
from typing import Any, Dict, Optional

from .native import runtime


class StateEnum(Enum):
    IDLE = 0
    BUSY = 1
    UNKNOWN = 2
    PARSE_ERROR = 3


def socket_send(bytes_to_send, sock: socket.socket, chunk_size: int, timeout_ms: int = -1) -> None:
    """Send one frame (u64 BE length + body) over `sock`."""
    runtime().send_frame(sock.fileno(), memoryview(bytes_to_send).cast("B"), int(chunk_size), timeout_ms)


def socket_send_parts(parts, sock: socket.socket, chunk_size: int, timeout_ms: int = -1) -> None:
    """Send one frame whose body is the concatenation of `parts` (buffers), without
    joining them in memory first."""
    runtime().send_frame_parts(sock.fileno(), [memoryview(p).cast("B") for p in parts], int(chunk_size),
                               timeout_ms)


def socket_recv(sock: socket.socket, chunk_size: int, timeout_ms: int = -1) -> bytes:
    """Receive one frame; returns b'' on a clean close before any header byte."""
    data = runtime().recv_frame(sock.fileno(), int(chunk_size), timeout_ms, 0)
    return b"" if data is None else data


class NodeState:
    """Thread-safe per-worker state (`src/node_state.py:9-36`)."""

    def __init__(self, chunk_size: int = 512 * 1000, dispatcher_ip: str = "127.0.0.1",
                 membership_port: int = 2379, node_id: Optional[str] = None, connect: bool = False) -> None:
        self._lock = threading.Lock()
        self._chunk_size = chunk_size
        self._next_node = ""
        self._state_enum = StateEnum.IDLE
        self.dispatcher_ip = dispatcher_ip
        self.membership_port = membership_port
        try:
            self._my_ip = socket.gethostbyname(socket.gethostname())
        except OSError:
            self._my_ip = "127.0.0.1"
        self.node_id = node_id or self._my_ip
        self._worker_key = f"/workers/{self.node_id}"
        self.model = None          # loaded slice executor (src/node.py:48)
        self.weights = None        # received weight list (src/node.py:45)
        self.partition_index: Optional[int] = None
        self.epoch = 0
        self.extra: Dict[str, Any] = {}
        self._client = None
        if connect:
            self.connect()

    # -------------------------------------------------------- membership
    def connect(self):
        from .membership.client import MembershipClient
        self._client = MembershipClient(self.dispatcher_ip, self.membership_port)
        return self._client

    @property
    def client(self):
        return self._client

    @property
    def worker_key(self) -> str:
        return self._worker_key

    def record(self) -> Dict[str, Any]:
        with self._lock:
            return {"id": self.node_id, "ip": self._my_ip, "state": self._state_enum.name,
                    "partition": self.partition_index, "epoch": self.epoch, **self.extra}

    def publish(self) -> None:
        if self._client is not None:
            self._client.put(self._worker_key, json.dumps(self.record()).encode(), lease=self.extra.get("lease"))

    # -------------------------------------------------------- properties
    @property
    def chunk_size(self) -> int:
        with self._lock:
            return self._chunk_size

    @property
    def next_node(self) -> str:
        with self._lock:
            return self._next_node

    @next_node.setter
    def next_node(self, nx: str) -> None:
        with self._lock:
            self._next_node = nx

    @property
    def state(self) -> StateEnum:
        with self._lock:
            return self._state_enum

    @state.setter
    def state(self, s: StateEnum) -> None:
        with self._lock:           # the reference writes _state_enum unlocked (src/node.py:82)
            self._state_enum = s
