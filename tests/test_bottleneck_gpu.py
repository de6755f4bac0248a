"""Fused ResNet bottleneck kernel (csrc/kernels/bottleneck.hip) against a
PyTorch fp32 reference of the same three convs (intermediates rounded to bf16
like the unfused path), identity and projection shortcuts, and the whole
ResNet-50 with the fusion on vs off."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops import conv as C

pytestmark = pytest.mark.gpu


def _ref(x, k1, b1, k2, b2, k3, b3, kp=None, bp=None):
    def conv(t, k, b, pad=0):
        return F.conv2d(t, torch.from_numpy(k).permute(3, 2, 0, 1).cuda(), torch.from_numpy(b).cuda(), padding=pad)
    xt = x.float().permute(0, 3, 1, 2)
    y1 = conv(xt, k1, b1).relu().bfloat16().float()
    y2 = conv(y1, k2, b2, 1).relu().bfloat16().float()
    sc = xt if kp is None else conv(xt, kp, bp)
    return (conv(y2, k3, b3) + sc).relu().permute(0, 2, 3, 1)


@pytest.mark.parametrize("proj", [False, True])
@pytest.mark.parametrize("hw", [(56, 56), (16, 24), (8, 8)])
def test_bottleneck_matches_reference(proj, hw):
    torch.backends.cudnn.allow_tf32 = False
    rng = np.random.default_rng(int(proj) * 10 + hw[0])
    cin = 64 if proj else 256

    def w(*s):
        return (rng.standard_normal(s) / np.sqrt(np.prod(s[:3]))).astype(np.float32)
    k1, k2, k3 = w(1, 1, cin, 64), w(3, 3, 64, 64), w(1, 1, 64, 256)
    b1, b2, b3 = (rng.standard_normal(n).astype(np.float32) * 0.1 for n in (64, 64, 256))
    kp, bp = (w(1, 1, 64, 256), rng.standard_normal(256).astype(np.float32) * 0.1) if proj else (None, None)
    x = torch.randn(2, hw[0], hw[1], cin, device="cuda").to(torch.bfloat16)
    pb = C.pack_bottleneck(k1, b1, k2, b2, k3, b3, kp, bp)
    out = torch.empty(2, hw[0], hw[1], 256, device="cuda", dtype=torch.bfloat16)
    C.bottleneck_forward(x, pb, out)
    want = _ref(x, k1, b1, k2, b2, k3, b3, kp, bp)
    err = (out.float() - want).abs().max().item() / max(1.0, want.abs().max().item())
    assert err < 1.5e-2, f"rel err {err}"


def test_resnet50_fused_vs_unfused():
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models import resnet as R
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.runtime.executor import \
        SliceExecutor
    g = R.build_resnet("resnet50")
    w = R.init_weights(g, seed=0)
    x = torch.randn(8, 224, 224, 3, device="cuda")
    fused = SliceExecutor(g, w, batch=8, device="cuda", precision="bf16")
    assert sum(st.kind == "bottleneck" for st in fused.steps) == 3
    fused(x)
    lf = fused.logits().clone()
    os.environ["ADAPT_FUSED_BOTTLENECK"] = "0"
    try:
        plain = SliceExecutor(g, w, batch=8, device="cuda", precision="bf16")
    finally:
        os.environ.pop("ADAPT_FUSED_BOTTLENECK")
    assert not any(st.kind == "bottleneck" for st in plain.steps)
    plain(x)
    lp = plain.logits()
    rel = (lf - lp).abs().max().item() / lp.abs().max().item()
    assert rel < 3e-2, rel
