"""zfp block geometry: adjacent axes folded to avoid edge-padded 4^d blocks (codec.zfp_shape).

The reference codes every hop with zfp (reversible) + LZ4 (`/root/reference/src/dispatcher.py:92-98`,
`src/node.py:122-125`); padded blocks are coded as data, so a 7x7 NHWC map kept 4-D grows by (8/7)^2.
"""
import numpy as np
import pytest

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd import codec
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.native import runtime


@pytest.mark.parametrize("shape,want", [
    ((32, 56, 56, 64), (32, 56, 56, 64)),       # no padding: keep every axis
    ((32, 14, 14, 1024), (32, 196, 1024)),
    ((32, 7, 7, 2048), (1568, 2048)),
    ((1, 1000), (1000,)),
    ((2, 3, 5, 7, 11), (2310,)),
    ((), (1,)),
])
def test_fold_picks_least_padding(shape, want):
    got = codec.zfp_shape(shape)
    assert got == want
    assert int(np.prod(got)) == max(1, int(np.prod(shape)))
    assert 1 <= len(got) <= 4


def _padded(dims):
    return int(np.prod([(v + 3) // 4 * 4 for v in dims]))


@pytest.mark.parametrize("shape", [(4, 7, 7, 64), (2, 14, 14, 32), (3, 5, 6, 7, 8)])
def test_fold_never_pads_more_than_the_plain_fold(shape):
    plain = shape if len(shape) <= 4 else (int(np.prod(shape[:-3])),) + shape[-3:]
    assert _padded(codec.zfp_shape(shape)) <= _padded(plain)


def test_small_map_round_trip_and_smaller_than_4d_coding():
    rng = np.random.default_rng(0)
    a = np.maximum(rng.standard_normal((4, 7, 7, 64)).astype(np.float32), 0)   # post-ReLU frontier
    buf = codec.encode(a, "zfp")
    assert np.array_equal(codec.decode(buf), a)
    folded = len(runtime().zfp_compress(a.reshape(codec.zfp_shape(a.shape)), 4))
    four_d = len(runtime().zfp_compress(a, 4))
    assert folded < four_d
