"""Native host runtime: framing transport, LZ4 frame codec, reversible zfp
codec, codec container (CPU).  Round trips must be bit-exact."""
import socket
import threading

import numpy as np
import pytest

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd import codec as C
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.native import runtime
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.node_state import (
    NodeState, StateEnum, socket_recv, socket_send)


@pytest.fixture(scope="module")
def rt():
    return runtime()


def test_xxh32_known_vectors(rt):
    # reference values of the xxHash32 specification
    assert rt.xxh32(b"", 0) == 0x02CC5D05
    assert rt.xxh32(b"a", 0) == 0x550D7456
    assert rt.xxh32(b"abc", 0) == 0x32D153FF
    assert rt.xxh32(b"Nobody inspects the spammish repetition", 0) == 0xE2293B2F


@pytest.mark.parametrize("n", [0, 1, 5, 13, 100, 4096, 70000, 5 << 20])
def test_lz4_frame_roundtrip(rt, n):
    rng = np.random.default_rng(n)
    for data in (rng.integers(0, 4, n, dtype=np.uint8).tobytes(), rng.integers(0, 256, n, dtype=np.uint8).tobytes(),
                 bytes(n)):
        c = rt.lz4_compress(data)
        assert c[:4] == b"\x04\x22\x4d\x18"               # LZ4 frame magic
        assert rt.lz4_decompress(c) == data


def test_lz4_block_and_corruption(rt):
    data = b"abcabcabcabc" * 1000 + b"tail-bytes"
    blk = rt.lz4_block_compress(data)
    assert len(blk) < len(data) / 10
    assert rt.lz4_block_decompress(blk, len(data)) == data
    fr = bytearray(rt.lz4_compress(data))
    fr[-1] ^= 0xFF                                         # content checksum
    with pytest.raises(RuntimeError):
        rt.lz4_decompress(bytes(fr))


@pytest.mark.parametrize("shape", [(1,), (7,), (3, 5), (4, 4, 4), (2, 9, 10, 3), (32, 7, 7, 16), (5, 1, 1, 1)])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_zfp_reversible_bit_exact(rt, shape, dtype):
    rng = np.random.default_rng(1)
    a = (rng.standard_normal(shape) * 10).astype(dtype)
    a.flat[0] = np.inf
    if a.size > 2:
        a.flat[1] = -0.0
        a.flat[2] = np.nan
    c = rt.zfp_compress(a)
    b = rt.zfp_decompress(c)
    assert b.dtype == a.dtype and b.shape == a.shape
    assert np.array_equal(a.view(np.uint8), b.view(np.uint8))


def test_zfp_compresses_smooth_data(rt):
    x = np.linspace(0, 1, 64 * 64, dtype=np.float32).reshape(64, 64)
    assert len(rt.zfp_compress(x)) < x.nbytes * 0.8


def test_zvc_host_codec(rt):
    rng = np.random.default_rng(4)
    for n, esz in ((1, 2), (63, 2), (4096, 2), (10_001, 2), (5000, 4)):
        a = rng.integers(0, 65535 if esz == 2 else 2**31, n).astype(np.uint16 if esz == 2 else np.uint32)
        a[rng.random(n) < 0.5] = 0
        s = rt.zvc_compress(a.view(np.uint8), esz)
        assert s[:4] == b"AZVC"
        assert np.array_equal(np.frombuffer(rt.zvc_decompress(s), a.dtype), a)
        if n >= 4096:
            assert len(s) < 0.7 * a.nbytes
    with pytest.raises(RuntimeError):
        rt.zvc_decompress(b"AZVC" + bytes(10))


@pytest.mark.parametrize("codec", ["none", "lz4", "zfp+lz4", "zfp", "zvc"])
def test_codec_container(codec):
    rng = np.random.default_rng(2)
    for a in (rng.standard_normal((2, 3, 4, 5, 6)).astype(np.float32), np.zeros((3, 4), np.float64),
              rng.integers(0, 9, (10,)).astype(np.int64), np.float32(3.5) * np.ones(())):
        e = C.encode(a, codec)
        b = C.decode(e)
        assert b.dtype == a.dtype and b.shape == a.shape and np.array_equal(a, b)
    bf = rng.integers(0, 65535, (4, 8)).astype(np.uint16)
    e = C.encode(bf, codec, bf16=True)
    assert C.is_bf16(e) and np.array_equal(C.decode(e), bf)
    # reference helpers
    w = rng.standard_normal((3, 3, 8, 16)).astype(np.float32)
    assert np.array_equal(C.decomp(C.comp(w)), w)


def test_framing_socketpair_blocking_and_nonblocking():
    a, b = socket.socketpair()
    payload = np.random.default_rng(0).integers(0, 256, 3_000_000, dtype=np.uint8).tobytes()
    b.setblocking(False)
    t = threading.Thread(target=lambda: (socket_send(payload, a, 512000), socket_send(b"", a, 7)))
    t.start()
    got = socket_recv(b, 4096)
    t.join()
    assert got == payload
    assert socket_recv(b, 4096) == b""          # zero-length frame
    a.close()
    assert socket_recv(b, 4096) == b""          # clean EOF before any header byte
    b.close()


def test_framing_truncated_frame_raises():
    a, b = socket.socketpair()
    a.sendall((100).to_bytes(8, "big") + b"x" * 10)
    a.close()
    with pytest.raises(RuntimeError):
        socket_recv(b, 1024)
    b.close()
    a, b = socket.socketpair()
    a.sendall(b"\x00\x00\x00")                  # partial header
    a.close()
    with pytest.raises(RuntimeError):
        socket_recv(b, 1024)


def test_wire_format_matches_reference_framing():
    a, b = socket.socketpair()
    socket_send(b"hello", a, 2)
    raw = b.recv(64)
    assert raw == (5).to_bytes(8, "big") + b"hello"


def test_node_state_api():
    ns = NodeState(chunk_size=512 * 1000, dispatcher_ip="127.0.0.1")
    assert ns.chunk_size == 512000 and ns.next_node == ""
    ns.next_node = "10.0.0.2"
    assert ns.next_node == "10.0.0.2"
    assert [e.value for e in StateEnum] == [0, 1, 2, 3]
    ns.state = StateEnum.BUSY
    assert ns.record()["state"] == "BUSY"


@pytest.mark.parametrize("chunk_blocks", [0, 1, 5])
@pytest.mark.parametrize("shape", [(7,), (5, 9), (3, 6, 10), (2, 5, 7, 9), (2, 2, 3, 5, 4)])
def test_zfp_container_versions_round_trip(shape, chunk_blocks):
    """zfp v1 (4096-block chunks) and v2 (chunk_blocks in the header, the GPU
    codec's layout with chunk_blocks=1) are lossless on any float32 data,
    including inf / nan / -0 / denormals."""
    rng = np.random.default_rng(len(shape) * 7 + chunk_blocks)
    a = rng.standard_normal(shape).astype(np.float32).reshape(-1)
    a[:4] = [np.inf, -np.inf, -0.0, 1e-42][: min(4, a.size)]
    if a.size > 5:
        a[5] = np.nan
    a = a.reshape(shape)
    if a.ndim > 4:
        a = a.reshape((-1,) + shape[-3:])
    rt = runtime()
    c = rt.zfp_compress(a, 4, chunk_blocks)
    dt, shp, off, cb = rt.zfp_info(c)
    assert tuple(shp) == a.shape and cb == (chunk_blocks or 4096)
    b = rt.zfp_decompress(c, 4)
    assert b.tobytes() == a.tobytes()


def test_zfp_wire_codec_cpu_round_trip():
    import torch
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.codec.wire import WireCodec
    t = torch.randn(2, 6, 5, 8)
    enc, dec = WireCodec("zfp", t), WireCodec("zfp", t)
    enc.encode(t)
    n = enc.nbytes()
    dec.wire[:n].copy_(enc.wire[:n])
    out = torch.empty_like(t)
    dec.decode(n, out)
    assert torch.equal(out, t)


def test_parallel_copy_into_matches_numpy():
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.native import runtime
    rng = np.random.default_rng(9)
    for n in (7, 1 << 20, (3 << 20) + 13):
        src = rng.integers(0, 256, n, dtype=np.uint8)
        for th in (1, 3, 4, 16):
            dst = np.zeros(n + 5, np.uint8)
            runtime().copy_into(dst, src, th)
            assert np.array_equal(dst[:n], src) and not dst[n:].any()
    with pytest.raises(RuntimeError):
        runtime().copy_into(np.zeros(3, np.uint8), np.zeros(4, np.uint8), 2)
