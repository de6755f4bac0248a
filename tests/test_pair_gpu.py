"""Fused 1x1 pair across a ResNet block boundary (csrc/kernels/pw_pair.hip):
y = relu(x.W3 + b3 + res), z = relu(y.W1 + b1) against an fp32 PyTorch
reference of the same two convs, for every compiled (CIN, CO, CM, BM)
instance, including a pixel count that is not a multiple of the tile."""
import importlib

import numpy as np
import pytest
import torch

PKG = "adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd"
conv = importlib.import_module(f"{PKG}.ops.conv")

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cin,co,cm,bm", sorted(conv.PAIR_CFGS))
@pytest.mark.parametrize("M", [25088, 6272, 1000, 17])
def test_pair_matches_two_convs(cin, co, cm, bm, M):
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    g = torch.Generator().manual_seed(cin + M)
    k3 = (torch.randn(1, 1, cin, co, generator=g) / cin ** 0.5).numpy()
    k1 = (torch.randn(1, 1, co, cm, generator=g) / co ** 0.5).numpy()
    b3 = (torch.randn(co, generator=g) * 0.1).numpy()
    b1 = (torch.randn(cm, generator=g) * 0.1).numpy()
    pp = conv.pack_pair(k3, b3, k1, b1, device="cuda")
    x = torch.randn(M, cin, generator=g).to("cuda", torch.bfloat16)
    res = torch.randn(M, co, generator=g).to("cuda", torch.bfloat16)
    y = torch.empty(M, co, device="cuda", dtype=torch.bfloat16)
    z = torch.empty(M, cm, device="cuda", dtype=torch.bfloat16)
    conv.pair_forward(x, res, pp, y, z, bm=bm)
    torch.cuda.synchronize()
    w3 = torch.from_numpy(np.ascontiguousarray(k3[0, 0])).cuda().to(torch.bfloat16).float()
    w1 = torch.from_numpy(np.ascontiguousarray(k1[0, 0])).cuda().to(torch.bfloat16).float()
    y_ref = torch.relu(x.float() @ w3 + torch.from_numpy(b3).cuda() + res.float())
    err_y = (y.float() - y_ref).abs().max().item()
    assert err_y <= 2e-2 * y_ref.abs().max().item() + 1e-2, f"y max err {err_y}"
    # z from the kernel's own (bf16-rounded) y: the second GEMM's numerics alone
    z_ref = torch.relu(y.float() @ w1 + torch.from_numpy(b1).cuda())
    err_z = (z.float() - z_ref).abs().max().item()
    assert err_z <= 2e-2 * z_ref.abs().max().item() + 1e-2, f"z max err {err_z}"


def test_pair_rejects_bad_shapes():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    k3 = np.zeros((1, 1, 128, 512), np.float32)
    k1 = np.zeros((1, 1, 512, 128), np.float32)
    pp = conv.pack_pair(k3, np.zeros(512, np.float32), k1, np.zeros(128, np.float32), device="cuda")
    x = torch.zeros(64, 128, device="cuda", dtype=torch.bfloat16)
    with pytest.raises(ValueError):
        conv.pair_forward(x, torch.zeros(64, 256, device="cuda", dtype=torch.bfloat16), pp,
                          torch.zeros(64, 512, device="cuda", dtype=torch.bfloat16),
                          torch.zeros(64, 128, device="cuda", dtype=torch.bfloat16))
    with pytest.raises(ValueError):
        conv.pair_forward(x, torch.zeros(64, 512, device="cuda", dtype=torch.bfloat16), pp,
                          torch.zeros(64, 512, device="cuda", dtype=torch.bfloat16),
                          torch.zeros(64, 128, device="cuda", dtype=torch.bfloat16), bm=48)


def test_resnet50_with_pairs_matches_unfused(monkeypatch):
    """Whole ResNet-50 with the pair fusion (default) against the plan without it
    (ADAPT_FUSED_PAIR=0) on the same weights and input: same logits up to bf16
    rounding (bit-identical at bs=32, where the unfused convs do not split K)."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    resnet = importlib.import_module(f"{PKG}.models.resnet")
    exe = importlib.import_module(f"{PKG}.runtime.executor")
    g = resnet.build_resnet("resnet50")
    w = resnet.init_weights(g, seed=0)
    x = torch.randn(4, 224, 224, 3, generator=torch.Generator().manual_seed(0)).cuda()
    outs = {}
    for flag in ("0", "1"):
        monkeypatch.setenv("ADAPT_FUSED_PAIR", flag)
        ex = exe.SliceExecutor(g, w, batch=4, device="cuda:0", precision="bf16")
        assert sum(s.kind == "pair" for s in ex.steps) == (3 if flag == "1" else 0)
        ex(x)
        outs[flag] = ex.logits().double().clone()
    torch.cuda.synchronize()
    rel = ((outs["1"] - outs["0"]).abs().max() / outs["0"].abs().max()).item()
    assert rel < 2e-2, f"pair-fused logits rel diff {rel}"
    assert (outs["1"].argmax(-1) == outs["0"].argmax(-1)).float().mean().item() >= 0.75
