"""Data-plane messages on TCP links (dispatcher <-> stage 0 / last stage, and
stage <-> stage in TCP ("RCCL-less") mode).

Reference: a request on :6000 is ``u32be partition_index`` + one frame of
``lz4(zfp(x))`` followed by SHUT_WR on a fresh connection per message
(`src/dispatcher.py:204-220`); results come back on :6003 as bare frames with
no request id (`src/dispatcher.py:121-151`).  We keep persistent connections
and make every message self-identifying so replays after a failure can be
de-duplicated:

    frame 0 : header  = "ADPT" | u32 partition | u64 req_id | u32 epoch | u32 count | u32 ntensors   (BE)
    frame 1..ntensors : codec-encoded tensors (codec/__init__.py), frontier order

`count` is the number of valid images (a partial micro-batch is zero-padded
by the receiver).
"""
from __future__ import annotations

import socket
import struct
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

from .. import codec as C
from . import shm
from ..node_state import socket_recv, socket_send, socket_send_parts

MAGIC = b"ADPT"
HDR = struct.Struct(">4sIQIII")


@dataclass
class Message:
    partition: int
    req_id: int
    epoch: int
    count: int
    tensors: List[np.ndarray] = field(default_factory=list)
    bf16: List[bool] = field(default_factory=list)     # tensor carries bfloat16 bits (uint16 view)
    # same-host link slots (transport/shm.py LinkPool) the tensors are views of: the
    # receiver clears their hand-off flags once its copy out of them has completed
    links: List[str] = field(default_factory=list)


def send_message(sock: socket.socket, m: Message, codec: str = "lz4", chunk_size: int = 512000,
                 timeout_ms: int = -1) -> None:
    socket_send(HDR.pack(MAGIC, m.partition, m.req_id, m.epoch, m.count, len(m.tensors)), sock, chunk_size,
                timeout_ms)
    flags = m.bf16 or [False] * len(m.tensors)
    for t, b in zip(m.tensors, flags):
        if isinstance(t, tuple):
            # (container header, payload view) from the GPU side-stream codec
            socket_send_parts(list(t), sock, chunk_size, timeout_ms)
        elif hasattr(t, "container"):
            # a same-host shared-memory slot (transport/shm.py): only its descriptor travels
            socket_send(t.container(), sock, chunk_size, timeout_ms)
        elif isinstance(t, (bytes, bytearray)):
            # a container already encoded elsewhere (GPU side-stream codec)
            socket_send(t, sock, chunk_size, timeout_ms)
        else:
            # header + payload as one frame; a raw payload goes out straight from
            # the array's memory (no tobytes / concatenation copies)
            socket_send_parts(C.encode_parts(t, codec, bf16=b), sock, chunk_size, timeout_ms)


def recv_message(sock: socket.socket, chunk_size: int = 512000, timeout_ms: int = -1,
                 keep_encoded: tuple = ()) -> Optional[Message]:
    """Receive one message.  Tensors whose codec is in `keep_encoded` stay as the
    received container bytes (a GPU stage decodes them on the device)."""
    h = socket_recv(sock, chunk_size, timeout_ms)
    if not h:
        return None
    magic, part, rid, epoch, count, nt = HDR.unpack(h)
    if magic != MAGIC:
        raise ValueError("bad data-plane message magic")
    ts, bf, links = [], [], []
    for _ in range(nt):
        buf = socket_recv(sock, chunk_size, timeout_ms)
        if not buf:
            raise ConnectionError("closed inside a message")
        bf.append(C.is_bf16(buf))
        if keep_encoded and C.codec_of(buf) in keep_encoded:
            ts.append(buf)
        else:
            ts.append(C.decode(buf, copy=False))      # read-only view of the received frame
            name = C.shm_name(buf) if C.codec_of(buf) in ("shm", "dev") else None
            if name is not None and shm.is_link(name):
                links.append(name)
    return Message(part, rid, epoch, count, ts, bf, links)


def connect(host: str, port: int, timeout: float = 5.0, hello: Optional[bytes] = None) -> socket.socket:
    s = socket.create_connection((host, port), timeout=timeout)
    s.settimeout(None)
    s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
    if hello is not None:
        socket_send(hello, s, 1 << 16)
    return s


def listen(host: str = "0.0.0.0", port: int = 0, backlog: int = 64) -> socket.socket:
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    s.bind((host, port))
    s.listen(backlog)
    return s
