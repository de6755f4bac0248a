"""Native CPU execution path (csrc/cpu/cpu_ops.cpp, runtime/cpu_executor.py).

The reference's single-device baseline is Keras `model.predict` in float32 on
whatever TF device the host has (`/root/reference/test/local_infer.py:18-28`);
BASELINE config 1 runs it on the CPU.  Every native op is checked against a
plain PyTorch fp32 reference of the same op, and whole models against the
`ops/reference.py` oracle.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models import resnet as R
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models import zoo
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.model import resnet
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops.reference import (
    ReferenceExecutor)
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.runtime import cpu_executor
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.runtime.stage import (
    StageCompute)

M = cpu_executor.native()
rng = np.random.default_rng(0)


def _rel(a, b):
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


@pytest.mark.parametrize("n,h,w,c,co,k,s,pads,act,res", [
    (2, 9, 11, 5, 7, 3, 1, (1, 1, 1, 1), 1, True),
    (1, 16, 16, 64, 64, 1, 1, (0, 0, 0, 0), 0, True),
    (2, 15, 13, 24, 130, 3, 2, (0, 1, 0, 1), 2, False),
    (1, 20, 20, 3, 64, 7, 2, (3, 3, 3, 3), 1, False),
    (3, 7, 7, 128, 96, 1, 2, (0, 0, 0, 0), 0, False),
    (1, 6, 6, 8, 16, 5, 1, (2, 2, 2, 2), 3, False),
])
def test_conv2d_matches_torch(n, h, w, c, co, k, s, pads, act, res):
    x = rng.standard_normal((n, h, w, c)).astype(np.float32)
    kern = (rng.standard_normal((k, k, c, co)) / np.sqrt(k * k * c)).astype(np.float32)
    b = rng.standard_normal(co).astype(np.float32)
    pt, pb, pl, pr = pads
    xt = F.pad(torch.from_numpy(x).permute(0, 3, 1, 2), (pl, pr, pt, pb))
    yt = F.conv2d(xt, torch.from_numpy(kern).permute(3, 2, 0, 1), torch.from_numpy(b), stride=s)
    yt = yt.permute(0, 2, 3, 1).contiguous()
    r = rng.standard_normal(yt.shape).astype(np.float32) if res else None
    if res:
        yt = yt + torch.from_numpy(r)
    yt = {0: yt, 1: torch.relu(yt), 2: torch.clamp(yt, 0, 6), 3: yt * torch.sigmoid(yt)}[act].numpy()
    y = np.empty(yt.shape, np.float32)
    M.conv2d(x, cpu_executor._pad_cout(kern, M.COB), b, y, s, pt, pl, act, 0.3, r)
    assert _rel(y, yt) < 2e-6


def test_dwconv_pools_and_eltwise_match_torch():
    x = rng.standard_normal((2, 10, 9, 24)).astype(np.float32)
    xt = torch.from_numpy(x).permute(0, 3, 1, 2)
    # depthwise 3x3 / s2, pads (0, 1) x (0, 1), relu6
    k = rng.standard_normal((3, 3, 24)).astype(np.float32)
    b = rng.standard_normal(24).astype(np.float32)
    yt = F.conv2d(F.pad(xt, (0, 1, 0, 1)), torch.from_numpy(k).permute(2, 0, 1)[:, None], torch.from_numpy(b),
                  stride=2, groups=24).clamp(0, 6).permute(0, 2, 3, 1).numpy()
    y = np.empty(yt.shape, np.float32)
    M.dwconv2d(x, k, b, y, 2, 0, 0, 2, 0.3)
    assert _rel(y, yt) < 2e-6
    # max pool 3x3/s2 over a folded ZeroPadding2D(1): the zeros take part
    yt = F.max_pool2d(F.pad(xt, (1, 1, 1, 1)), 3, 2).permute(0, 2, 3, 1).numpy()
    y = np.empty(yt.shape, np.float32)
    M.pool2d(x, y, 0, 3, 3, 2, 1, 1, True)
    np.testing.assert_array_equal(y, yt)
    # max pool 'same': padding excluded
    yt = F.max_pool2d(F.pad(xt, (0, 1, 0, 1), value=float("-inf")), 2, 2).permute(0, 2, 3, 1).numpy()
    y = np.empty(yt.shape, np.float32)
    M.pool2d(x, y, 0, 2, 2, 2, 0, 0, False)
    np.testing.assert_array_equal(y, yt)
    # avg pool 'same' 3x3/s1: TF divides by the in-image count
    ones = torch.ones_like(xt[:, :1])
    num = F.avg_pool2d(F.pad(xt, (1, 1, 1, 1)), 3, 1, divisor_override=1)
    den = F.avg_pool2d(F.pad(ones, (1, 1, 1, 1)), 3, 1, divisor_override=1)
    yt = (num / den).permute(0, 2, 3, 1).numpy()
    y = np.empty(yt.shape, np.float32)
    M.pool2d(x, y, 1, 3, 3, 1, 1, 1, False)
    assert _rel(y, yt) < 1e-6
    # global average / max
    g = np.empty((2, 24), np.float32)
    M.global_pool(x, g, 0)
    assert _rel(g, x.mean(axis=(1, 2))) < 1e-6
    M.global_pool(x, g, 1)
    np.testing.assert_array_equal(g, x.max(axis=(1, 2)))
    # affine + swish, binary with a per-image channel row, softmax, concat, zero pad
    sc, sh = rng.standard_normal(24).astype(np.float32), rng.standard_normal(24).astype(np.float32)
    y = np.empty_like(x)
    M.affine(x, sc, sh, y, 3, 0.3)
    v = x * sc + sh
    assert _rel(y, v / (1 + np.exp(-v))) < 1e-6
    row = rng.standard_normal((2, 24)).astype(np.float32)
    M.binary(x, row, y, 1, 0, 0.3)
    assert _rel(y, x * row[:, None, None, :]) < 1e-7
    M.binary(x, x[::-1].copy(), y, 0, 1, 0.3)
    np.testing.assert_array_equal(y, np.maximum(x + x[::-1], 0))
    lg = rng.standard_normal((5, 1000)).astype(np.float32) * 4
    p = np.empty_like(lg)
    M.softmax(lg, p)
    assert _rel(p, torch.softmax(torch.from_numpy(lg), -1).numpy()) < 1e-6
    z = rng.standard_normal((2, 10, 9, 8)).astype(np.float32)
    cat = np.empty((2, 10, 9, 32), np.float32)
    M.concat([x, z], cat)
    np.testing.assert_array_equal(cat, np.concatenate([x, z], -1))
    pd = np.empty((2, 13, 11, 24), np.float32)
    M.zero_pad(x, pd, 2, 1)
    np.testing.assert_array_equal(pd, np.pad(x, ((0, 0), (2, 1), (1, 1), (0, 0))))


def test_resnet50_native_cpu_logits_match_oracle():
    """Config 1: whole ResNet-50 on the native path, logits within 1e-4 of the oracle."""
    g = R.build_resnet("resnet50")
    w = R.init_weights(g, seed=0)
    x = rng.standard_normal((2, 224, 224, 3)).astype(np.float32)
    ex = cpu_executor.CpuExecutor(g, w)
    assert {st.kind for st in ex.steps} <= {"conv", "maxpool", "gap", "dense"}
    probs = ex(x)
    feat = ReferenceExecutor(g, w).run({g.input: torch.from_numpy(x)}, outputs=["avg_pool"])["avg_pool"]
    want = feat.double().numpy() @ w["predictions/kernel"].astype(np.float64) + w["predictions/bias"]
    assert _rel(ex.logits(), want) < 1e-4
    assert (ex.logits().argmax(-1) == want.argmax(-1)).all()
    assert np.allclose(probs.sum(-1), 1.0, atol=1e-5)


@pytest.mark.parametrize("name", ["mobilenet_v2", "efficientnetb0", "densenet121", "inception_v3", "vgg16"])
def test_zoo_native_cpu_matches_oracle(name):
    g = zoo.build_model(name)
    w = R.init_weights(g, seed=1)
    x = rng.standard_normal((1,) + tuple(g.layers[g.input].out_shape)).astype(np.float32)
    y = cpu_executor.CpuExecutor(g, w)(x)
    yr = ReferenceExecutor(g, w)(torch.from_numpy(x)).numpy()
    assert _rel(y, yr) < 1e-4


def test_predict_and_stage_compute_use_the_native_path():
    """Model.predict(device="cpu") and a CPU StageCompute run CpuExecutor, not
    PyTorch ops; a sliced stage with a multi-tensor frontier (BASELINE config
    2's cut) composes to the unsliced forward."""
    m = resnet("resnet50")
    x = rng.standard_normal((1, 224, 224, 3)).astype(np.float32)
    y = m.predict(x, device="cpu")
    assert isinstance(m._executors["cpu"], cpu_executor.CpuExecutor)
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.graph.slicer import (
        partition, subgraph)
    parts = [subgraph(m.graph, s) for s in partition(m.graph, ["conv3_block1_1_conv"])]
    assert len(parts) == 2
    s0 = StageCompute(parts[0], m.weights, batch=1, device="cpu")
    s1 = StageCompute(parts[1], m.weights, batch=1, device="cpu")
    assert isinstance(s0.ex, cpu_executor.CpuExecutor) and isinstance(s1.ex, cpu_executor.CpuExecutor)
    mid, _ = s0.run_host([x], [False], 1)
    assert len(mid) == 2                            # conv3_block1_1_conv + conv2_block3_out
    feed = dict(zip(s0.outputs, mid))
    out, _ = s1.run_host([feed[n] for n in s1.inputs], [False] * len(s1.inputs), 1)
    assert _rel(out[0], y) < 1e-5
    # bf16 bit patterns from a GPU stage are widened on the way in
    bf = [(np.ascontiguousarray(feed[n]).view(np.uint32) >> 16).astype(np.uint16) for n in s1.inputs]
    out16, _ = s1.run_host(bf, [True] * len(bf), 1)
    assert _rel(out16[0], y) < 5e-2
