"""Model-level numerics on the MI355X: our fused HIP runtime vs the fp32
PyTorch oracle, whole-model and sliced."""
import numpy as np
import pytest
import torch

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.graph.slicer import partition, subgraph
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.resnet import build_resnet, init_weights
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops.reference import ReferenceExecutor
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.runtime.executor import SliceExecutor

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def r50():
    g = build_resnet("resnet50")
    w = init_weights(g, seed=0)
    return g, w


def _img(b, seed=0):
    gen = torch.Generator().manual_seed(seed)
    return torch.randn(b, 224, 224, 3, generator=gen)


def test_resnet50_full_vs_oracle(r50):
    g, w = r50
    x = _img(4)
    ref = ReferenceExecutor(g, w, device="cuda")
    want = ref(x.cuda())
    ex = SliceExecutor(g, w, batch=4, precision="bf16")
    got = ex(x.cuda()).float()
    torch.cuda.synchronize()
    # probabilities: compare top-1 and L1 distance of the distributions
    assert got.shape == (4, 1000)
    assert torch.allclose(got.sum(-1), torch.ones(4, device="cuda"), atol=1e-3)
    l1 = (got - want).abs().sum(-1).max().item()
    assert l1 < 0.1, f"softmax L1 distance {l1}"
    # pre-softmax features: compare the GAP vector (bf16 path vs fp32)
    feats_ref = ref.run({g.input: x.cuda()}, outputs=["avg_pool"])["avg_pool"]
    ex2 = SliceExecutor(g, w, batch=4, outputs=["avg_pool"], precision="bf16")
    feats = ex2(x.cuda()).float()
    rel = ((feats - feats_ref).norm() / feats_ref.norm()).item()
    assert rel < 3e-2, f"relative feature error {rel}"


@pytest.mark.parametrize("cuts", [["conv3_block1_1_conv"], ["conv4_block1_out"],
                                  ["pool1_pool", "conv3_block1_out", "conv4_block1_out"],
                                  ["conv1_pad", "conv2_block1_3_bn", "conv3_block2_add"]])
def test_sliced_equals_unsliced(r50, cuts):
    g, w = r50
    x = _img(2, seed=3).cuda()
    full = SliceExecutor(g, w, batch=2, precision="bf16")
    want = full(x).float().clone()
    slices = partition(g, cuts)
    vals = {g.input: x}
    for s in slices:
        sg = subgraph(g, s)
        ex = SliceExecutor(sg, w, batch=2, precision="bf16")
        outs = ex.run({n: vals[n] for n in s.inputs})
        vals = {k: v.clone() for k, v in outs.items()}
    got = vals[g.output].float()
    # same kernels, same rounding points except where a cut forces an unfused BN/add
    assert (got - want).abs().sum(-1).max().item() < 0.05


def test_graph_capture_replay(r50):
    g, w = r50
    ex = SliceExecutor(g, w, batch=8, precision="bf16")
    x = _img(8, seed=5).cuda()
    eager = ex(x).clone()
    ex.capture()
    ex.inputs[g.input].copy_(x)
    out = ex.forward()[g.output]
    torch.cuda.synchronize()
    assert torch.equal(out, eager)


@pytest.mark.parametrize("batch", [2, 32])
def test_resnet152_bf16_logits_vs_fp32_oracle(batch):
    """BASELINE config 5's model in bf16 (the 4-stage config runs bf16): pre-softmax
    logits against the fp32 PyTorch oracle (max error relative to the largest
    logit) and top-1 agreement, at a small and at the bench batch (the bench batch
    takes the pair / bottleneck / register-resident 3x3 kernels)."""
    g = build_resnet("resnet152")
    w = init_weights(g, seed=1)
    x = _img(batch, seed=11).cuda()
    ex = SliceExecutor(g, w, batch=batch, precision="bf16")
    ex(x)
    got = ex.logits().double()
    ref = ReferenceExecutor(g, w, device="cuda")
    feat = ref.run({g.input: x}, outputs=["avg_pool"])["avg_pool"].double()
    want = feat @ torch.from_numpy(w["predictions/kernel"]).double().cuda() \
        + torch.from_numpy(w["predictions/bias"]).double().cuda()
    torch.cuda.synchronize()
    rel = ((got - want).abs().max() / want.abs().max()).item()
    top1 = (got.argmax(-1) == want.argmax(-1)).float().mean().item()
    print(f"resnet152 bf16 bs={batch}: logits rel err {rel:.3e}, top-1 agreement {top1:.3f}")
    assert torch.isfinite(got).all() and rel < 5e-2, rel
    assert top1 >= 0.9, top1
