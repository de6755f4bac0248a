"""Array codecs for the wire (weights, activations, inputs, results).

Reference: every array crossing a socket is ``lz4.frame.compress(
zfpy.compress_numpy(arr))`` (`src/dispatcher.py:92-98`, `src/node.py:122-125`),
unconditionally.  We keep that codec as ``"zfp+lz4"`` (native, see
csrc/runtime) and add policies, because over xGMI compression only pays when
codec throughput beats the link:

* ``"zfp+lz4"``  reference behaviour (float32/float64 arrays)
* ``"lz4"``      LZ4 frame over the raw bytes (any dtype, incl. bf16)
* ``"none"``     raw bytes

Every encoded message is self-describing::

    u8 codec | u8 dtype | u8 ndim | u8 flags | u64 shape[ndim] | payload

so the receiver never needs out-of-band metadata.  A codec that would expand
the data falls back to ``none`` for that message.
"""
from __future__ import annotations

import struct
from typing import Optional, Tuple

import numpy as np

from ..native import runtime

# "shm": the payload is a reference (segment name + offset) to a same-host
# shared-memory slot holding the raw array (transport/shm.py); "dev": the same
# for a device link slot (device memory exported by IPC handle), decoded to a
# `shm.DevArray` that only a GPU stage consumes
CODECS = {"none": 0, "lz4": 1, "zfp+lz4": 2, "zfp": 3, "zvc": 4, "shm": 5, "dev": 6}
_CODEC_NAMES = {v: k for k, v in CODECS.items()}
# dtype codes (bf16 travels as raw 16-bit words)
DTYPES = {0: np.float32, 1: np.float64, 2: np.float16, 3: np.uint16, 4: np.int32, 5: np.int64, 6: np.uint8,
          7: np.int8, 8: np.bool_}
BF16 = 9          # flag value: payload is bfloat16 (numpy has no bf16; carried as uint16)
_DT_CODE = {np.dtype(v): k for k, v in DTYPES.items()}


def zfp_shape(shape) -> Tuple[int, ...]:
    """The 1-4 dimensional array zfp codes for a tensor of `shape`: adjacent axes
    folded so that the 4^d blocks need the least edge padding (ties: the most
    axes, then the innermost split).  Padded blocks are coded as real data, so
    NHWC maps of 7x7 or 14x14 kept as 4-D grew by (8/7)^2 or (16/14)^2 and the
    codec expanded them (x0.75, profiles/r5/codec_fp32_r50_bs32.txt); (B*H*W, C)
    or (B, H*W, C) have no padding there.  The container records this shape, and
    both ends of a wire derive it from the message shape."""
    shape = tuple(int(v) for v in shape)
    if len(shape) == 0:
        return (1,)
    n = len(shape)
    best = None
    for mask in range(1 << (n - 1)):                  # bit i set: a split after axis i
        if bin(mask).count("1") > 3:
            continue
        dims, cur = [], 1
        for i, v in enumerate(shape):
            cur *= v
            if i == n - 1 or mask >> i & 1:
                dims.append(cur)
                cur = 1
        padded = 1
        for v in dims:
            padded *= (v + 3) // 4 * 4
        key = (padded, -len(dims), -mask)
        if best is None or key < best[0]:
            best = (key, tuple(dims))
    return best[1]


def _header(codec: int, dtype_code: int, shape: Tuple[int, ...]) -> bytes:
    return struct.pack(f"<BBBB{len(shape)}Q", codec, dtype_code, len(shape), 0, *shape)


def _parse(buf: bytes):
    codec, dt, nd, _flags = struct.unpack_from("<BBBB", buf, 0)
    shape = struct.unpack_from(f"<{nd}Q", buf, 4)
    return codec, dt, tuple(shape), 4 + 8 * nd


def encode(arr: np.ndarray, codec: str = "zfp+lz4", bf16: bool = False, threads: int = 4) -> bytes:
    """Encode an ndarray.  `bf16=True` marks a uint16 array as bfloat16 payload."""
    hdr, payload = encode_parts(arr, codec, bf16, threads)
    return hdr + bytes(payload)


def encode_parts(arr: np.ndarray, codec: str = "zfp+lz4", bf16: bool = False, threads: int = 4):
    """(header bytes, payload buffer) of `encode`, without concatenating them:
    for ``none`` the payload is a zero-copy view of `arr`, and the framing layer
    sends both parts as one frame (`send_frame_parts`)."""
    arr = np.asarray(arr)
    if not arr.flags.c_contiguous:
        arr = arr.copy(order="C")            # (np.ascontiguousarray would promote 0-d to 1-d)
    rt = runtime()
    dt_code = BF16 if bf16 else _DT_CODE.get(arr.dtype)
    if dt_code is None:
        raise TypeError(f"unsupported dtype {arr.dtype}")
    c = CODECS[codec]
    if c in (2, 3) and arr.dtype not in (np.float32, np.float64):
        c = 1                               # zfp is float32/float64 only
    if c == 4 and arr.dtype.itemsize not in (2, 4):
        c = 1                               # zvc works on 2- or 4-byte elements
    arr_z = arr.reshape(zfp_shape(arr.shape)) if c in (2, 3) else arr
    raw = arr.reshape(-1).view(np.uint8) if arr.size else np.zeros(0, np.uint8)
    if c == 0:
        payload = memoryview(raw)
    elif c == 1:
        payload = rt.lz4_compress(raw)
    elif c == 2:
        payload = rt.lz4_compress(rt.zfp_compress(arr_z, threads))
    elif c == 3:
        payload = rt.zfp_compress(arr_z, threads)
    else:
        payload = rt.zvc_compress(raw, arr.dtype.itemsize)
    if c != 0 and len(payload) >= raw.nbytes:
        c, payload = 0, memoryview(raw)
    return _header(c, dt_code, arr.shape), payload


def wrap(payload: bytes, codec: str, dtype, shape, bf16: bool = False) -> bytes:
    """Container around a payload that was already encoded elsewhere (e.g. by the
    GPU codecs on a side stream); `decode` reads it like any other message."""
    dt_code = BF16 if bf16 else _DT_CODE[np.dtype(dtype)]
    return _header(CODECS[codec], dt_code, tuple(int(s) for s in shape)) + payload


def payload_of(buf):
    """(codec name, dtype code, shape, payload memoryview) of an encoded message."""
    codec, dt, shape, off = _parse(buf)
    return _CODEC_NAMES[codec], dt, shape, memoryview(buf)[off:]


def decode(buf, threads: int = 4, copy: bool = True) -> np.ndarray:
    """Inverse of `encode`.  bfloat16 payloads come back as uint16 arrays
    (use `is_bf16` to tell); everything else with its own dtype.  With
    ``copy=False`` raw / LZ4 / ZVC payloads come back as read-only views of the
    received (or decompressed) buffer instead of fresh copies."""
    buf = bytes(buf) if not isinstance(buf, (bytes, bytearray, memoryview)) else buf
    codec, dt, shape, off = _parse(buf)
    rt = runtime()
    body = memoryview(buf)[off:]
    np_dt = np.uint16 if dt == BF16 else DTYPES[dt]

    def _fin(a):
        a = a.reshape(shape)
        return a.copy() if copy else a
    if codec == 0:
        return _fin(np.frombuffer(body, dtype=np_dt))
    if codec == 1:
        return _fin(np.frombuffer(rt.lz4_decompress(body), dtype=np_dt))
    if codec == 2:
        return rt.zfp_decompress(rt.lz4_decompress(body), threads).reshape(shape)
    if codec == 3:
        return rt.zfp_decompress(body, threads).reshape(shape)
    if codec == 4:
        return _fin(np.frombuffer(rt.zvc_decompress(body), dtype=np_dt))
    if codec == 5:
        from ..transport import shm
        raw = bytes(body)
        cut = raw.index(b"\0")
        off = int.from_bytes(raw[cut + 1:cut + 9], "little")
        a = shm.view(raw[:cut].decode(), off, np_dt, shape, register_device=shm.REGISTER_DEVICE)
        return a.copy() if copy else a
    if codec == 6:
        from ..transport import shm
        raw = bytes(body)
        cut = raw.index(b"\0")
        return shm.DevArray(raw[:cut].decode(), int.from_bytes(raw[cut + 1:cut + 9], "little"), np_dt, shape)
    raise ValueError(f"unknown codec id {codec}")


def shm_name(buf) -> Optional[str]:
    """Segment name of a "shm" or "dev" container (None for every other codec)."""
    codec, _dt, _shape, off = _parse(buf)
    if codec not in (CODECS["shm"], CODECS["dev"]):
        return None
    raw = bytes(memoryview(buf)[off:])
    return raw[:raw.index(b"\0")].decode()


def is_bf16(buf) -> bool:
    return _parse(buf)[1] == BF16


def codec_of(buf) -> str:
    return _CODEC_NAMES[_parse(buf)[0]]


# reference-named helpers (`_comp` / `_decomp`, src/dispatcher.py:92-98)
def comp(arr: np.ndarray) -> bytes:
    return encode(arr, "zfp+lz4")


def decomp(byts) -> np.ndarray:
    return decode(byts)
