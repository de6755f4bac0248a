"""Slice format (wire + disk), dag_util API, Model wrapper (CPU)."""
import socket
import threading

import numpy as np
import pytest
import torch

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd import dag_util
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.graph.manifest import (
    SliceManifest, build_manifest, load_model, load_slice, recv_slice, save_model, save_slice, send_slice)
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.graph.slicer import partition
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.model import resnet
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.resnet import get_weights, set_weights


@pytest.fixture(scope="module")
def tiny():
    return resnet("resnet_tiny", input_shape=(32, 32, 3), classes=10, seed=3)


def test_get_set_weights_keras_order(tiny):
    g = tiny.graph
    ws = tiny.get_weights()
    assert len(ws) == len(g.weight_specs())
    assert ws[0].shape == (7, 7, 3, 64) and ws[1].shape == (64,)          # conv1 kernel HWIO, bias
    assert ws[2].shape == (64,) and len(ws) % 2 == 0                       # conv1_bn gamma ...
    back = set_weights(g, ws)
    assert all(np.array_equal(back[k], tiny.weights[k]) for k in back)
    with pytest.raises(ValueError):
        set_weights(g, ws[:-1])


def test_slice_wire_roundtrip(tiny):
    g = tiny.graph
    s = partition(g, ["conv3_block1_1_conv"])[1]
    m, arrays = build_manifest(g, s, tiny.weights)
    a, b = socket.socketpair()
    t = threading.Thread(target=send_slice, args=(a, m, arrays, 4096, "zfp+lz4"))
    t.start()
    m2, arrays2 = recv_slice(b, 4096)
    t.join()
    assert m2.part_index == 2 and m2.part_name == "part2"
    assert [x["name"] for x in m2.inputs] == ["conv2_block1_out", "conv3_block1_1_conv"]
    assert len(arrays2) == len(arrays) and all(np.array_equal(x, y) for x, y in zip(arrays, arrays2))
    assert m2.graph().input_names == s.inputs


def test_slice_disk_roundtrip(tmp_path, tiny):
    g = tiny.graph
    s = partition(g, ["conv4_block1_out"])[0]
    m, arrays = build_manifest(g, s, tiny.weights)
    save_slice(str(tmp_path / "p1"), m, arrays)
    m2, a2 = load_slice(str(tmp_path / "p1"))
    assert m2.to_json() == m.to_json() and all(np.array_equal(x, y) for x, y in zip(arrays, a2))
    save_model(str(tmp_path / "full"), g, tiny.weights)
    g2, w2 = load_model(str(tmp_path / "full"))
    assert g2.order == g.order and all(np.array_equal(w2[k], tiny.weights[k]) for k in w2)


def test_manifest_checksum_detects_corruption(tiny):
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.graph.manifest import verify_arrays
    g = tiny.graph
    m, arrays = build_manifest(g, partition(g, [])[0], tiny.weights)
    arrays[3] = arrays[3].copy()
    arrays[3].flat[0] += 1.0
    with pytest.raises(ValueError):
        verify_arrays(m, arrays)


def test_dag_util_api(tiny):
    g = tiny.graph
    assert dag_util.get_previous(tiny, "conv2_block1_add") == ["conv2_block1_0_bn", "conv2_block1_3_bn"]
    p1 = dag_util.construct_model(tiny, tiny.input, "conv3_block1_out", "part1")
    p2 = dag_util.construct_model(tiny, "conv3_block1_out", tiny.output, "part2")
    assert p1.graph.input_names == [tiny.input] and p2.graph.input_names == ["conv3_block1_out"]
    x = np.random.default_rng(0).standard_normal((2, 32, 32, 3)).astype(np.float32)
    want = tiny.predict(x, device="cpu")
    mid = p1.predict(x, device="cpu")
    got = p2.predict(mid, device="cpu")
    np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-6)
    # reference behaviour: a skip branch bypassing the cut raises in strict mode
    with pytest.raises(RuntimeError):
        dag_util.construct_model(tiny, "conv3_block1_1_conv", tiny.output, "p", strict=True)
    p = dag_util.construct_model(tiny, "conv3_block1_1_conv", tiny.output, "p")
    assert p.graph.input_names == ["conv2_block1_out", "conv3_block1_1_conv"]
    cache = {}
    assert dag_util.traverse_improved(tiny, "conv3_block1_out", "conv3_block1_1_conv", "p", None, cache) == \
        "conv3_block1_out"
    with pytest.raises(RuntimeError):
        dag_util.traverse_improved(tiny, "conv3_block1_out", "conv3_block1_1_conv", "p", None, {}, strict=True)


def test_model_summary_and_reference(tiny):
    s = tiny.summary(print_fn=None)
    assert "conv1_conv" in s and "Total params" in s
    y = tiny.predict(np.zeros((1, 32, 32, 3), np.float32), device="cpu")
    assert y.shape == (1, 10) and abs(float(y.sum()) - 1.0) < 1e-5


def test_reference_weight_push_framing(tiny):
    """DEFER._send_weights -> Node._recv_weights (`src/dispatcher.py:76-89`,
    `src/node.py:101-119`): u64be count + framed zfp+lz4 arrays, lossless."""
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.dispatcher import DEFER
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.node import Node
    arrays = [np.asarray(v, np.float32) for v in list(tiny.weights.values())[:12]]
    a, b = socket.socketpair()
    d = DEFER.__new__(DEFER)
    d.chunk_size = 4096
    n = Node.__new__(Node)
    t = threading.Thread(target=d._send_weights, args=(arrays, a, 4096))
    t.start()
    got = n._recv_weights(b, 4096)
    t.join()
    a.close()
    b.close()
    assert len(got) == len(arrays)
    for x, y in zip(arrays, got):
        assert x.shape == y.shape and np.array_equal(x, y)
    assert np.array_equal(DEFER._decomp(DEFER._comp(arrays[0])), arrays[0])
