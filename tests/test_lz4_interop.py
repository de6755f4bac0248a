"""LZ4 frame interoperability with the system liblz4 (the C library that
python-lz4, the reference's codec, wraps: `src/dispatcher.py:92-98`).

* frames from our host encoder (csrc/runtime/lz4.cpp) decode with liblz4's
  LZ4F_decompress;
* frames from liblz4's LZ4F_compressFrame (linked or independent blocks, 64 KiB
  to 4 MiB block sizes, with and without checksums) decode with ours.

liblz4.so.1 is loaded with ctypes; the tests skip if it is absent.  The GPU
encoder's frames are checked against liblz4 in tests/test_codec_wire_gpu.py.
"""
import ctypes
import ctypes.util

import numpy as np
import pytest

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.native import runtime


def _lib():
    name = ctypes.util.find_library("lz4") or "liblz4.so.1"
    try:
        return ctypes.CDLL(name)
    except OSError:
        return None


LIB = _lib()
pytestmark = pytest.mark.skipif(LIB is None, reason="system liblz4 not loadable")


class Prefs(ctypes.Structure):
    # LZ4F_preferences_t (lz4frame.h, v1.9): frameInfo then compressionLevel, autoFlush, favorDecSpeed, reserved[3]
    _fields_ = [("blockSizeID", ctypes.c_int), ("blockMode", ctypes.c_int), ("contentChecksumFlag", ctypes.c_int),
                ("frameType", ctypes.c_int), ("contentSize", ctypes.c_ulonglong), ("dictID", ctypes.c_uint),
                ("blockChecksumFlag", ctypes.c_int), ("compressionLevel", ctypes.c_int),
                ("autoFlush", ctypes.c_uint), ("favorDecSpeed", ctypes.c_uint), ("reserved", ctypes.c_uint * 3)]


if LIB is not None:
    LIB.LZ4F_compressFrameBound.restype = ctypes.c_size_t
    LIB.LZ4F_compressFrameBound.argtypes = [ctypes.c_size_t, ctypes.c_void_p]
    LIB.LZ4F_compressFrame.restype = ctypes.c_size_t
    LIB.LZ4F_compressFrame.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
                                       ctypes.c_void_p]
    LIB.LZ4F_isError.restype = ctypes.c_uint
    LIB.LZ4F_isError.argtypes = [ctypes.c_size_t]
    LIB.LZ4F_getErrorName.restype = ctypes.c_char_p
    LIB.LZ4F_getErrorName.argtypes = [ctypes.c_size_t]
    LIB.LZ4F_createDecompressionContext.restype = ctypes.c_size_t
    LIB.LZ4F_createDecompressionContext.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
    LIB.LZ4F_freeDecompressionContext.restype = ctypes.c_size_t
    LIB.LZ4F_freeDecompressionContext.argtypes = [ctypes.c_void_p]
    LIB.LZ4F_decompress.restype = ctypes.c_size_t
    LIB.LZ4F_decompress.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_size_t),
                                    ctypes.c_void_p, ctypes.POINTER(ctypes.c_size_t), ctypes.c_void_p]


def lib_compress(data: bytes, block_id: int = 0, linked: bool = True, checksum: bool = False,
                 content_size: bool = False, level: int = 0) -> bytes:
    p = Prefs()
    p.blockSizeID = block_id              # 0 = default (64 KiB), 4..7 = 64 KiB..4 MiB
    p.blockMode = 0 if linked else 1
    p.contentChecksumFlag = int(checksum)
    p.contentSize = len(data) if content_size else 0
    p.compressionLevel = level
    cap = LIB.LZ4F_compressFrameBound(len(data), ctypes.byref(p))
    dst = ctypes.create_string_buffer(cap)
    n = LIB.LZ4F_compressFrame(dst, cap, data, len(data), ctypes.byref(p))
    assert not LIB.LZ4F_isError(n), LIB.LZ4F_getErrorName(n)
    return dst.raw[:n]


def lib_decompress(frame: bytes, size: int) -> bytes:
    ctx = ctypes.c_void_p()
    r = LIB.LZ4F_createDecompressionContext(ctypes.byref(ctx), 100)      # LZ4F_VERSION
    assert not LIB.LZ4F_isError(r)
    try:
        out = ctypes.create_string_buffer(max(size, 1))
        src = ctypes.create_string_buffer(frame, len(frame))
        got, pos = 0, 0
        while pos < len(frame):
            dsz = ctypes.c_size_t(size - got)
            ssz = ctypes.c_size_t(len(frame) - pos)
            hint = LIB.LZ4F_decompress(ctx, ctypes.byref(out, got), ctypes.byref(dsz),
                                       ctypes.byref(src, pos), ctypes.byref(ssz), None)
            assert not LIB.LZ4F_isError(hint), LIB.LZ4F_getErrorName(hint)
            got += dsz.value
            pos += ssz.value
            if hint == 0:
                break
        assert pos == len(frame) and got == size
        return out.raw[:size]
    finally:
        LIB.LZ4F_freeDecompressionContext(ctx)


def _payloads():
    rng = np.random.default_rng(0)
    act = np.maximum(rng.standard_normal(300_000), 0).astype(np.float32)
    bf16 = (act.view(np.uint32) >> 16).astype(np.uint16)
    return {
        "empty": b"",
        "one": b"x",
        "zeros_5MiB": bytes(5 << 20),
        "random_200k": rng.integers(0, 256, 200_000, dtype=np.uint8).tobytes(),
        "text": (b"ADAPT distributed inference over xGMI " * 5000),
        "relu_fp32": act.tobytes(),
        "relu_bf16": bf16.tobytes(),
        "block_edge": rng.integers(0, 4, (64 << 10) + 1, dtype=np.uint8).tobytes(),
    }


@pytest.mark.parametrize("name", list(_payloads()))
def test_our_frames_decode_with_liblz4(name):
    data = _payloads()[name]
    frame = bytes(runtime().lz4_compress(data, 1))
    assert lib_decompress(frame, len(data)) == data


@pytest.mark.parametrize("name", list(_payloads()))
@pytest.mark.parametrize("opts", [dict(), dict(linked=False), dict(block_id=7, checksum=True, content_size=True),
                                  dict(block_id=5, linked=True, checksum=True), dict(level=9)])
def test_liblz4_frames_decode_with_ours(name, opts):
    data = _payloads()[name]
    frame = lib_compress(data, **opts)
    assert bytes(runtime().lz4_decompress(frame)) == data
