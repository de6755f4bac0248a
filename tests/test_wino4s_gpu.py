"""fp32 Winograd F(4x4, 3x3) as transform + pure-MFMA GEMM (csrc/kernels/wino4s_f32.hip, cfgs 220-229).

Every config and split against a float64 `F.conv2d` of the same fp32 data (the reference computes in
Keras float32, `/root/reference/test/local_infer.py:22`; ResNet-50's 3x3s, `/root/reference/test/test.py:13`).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops import conv as C_

pytestmark = pytest.mark.gpu

CFGS = sorted(C_.WINO4S_F32_CFGS)


def _oracle(x, k, b, relu):
    y = F.conv2d(x.double().permute(0, 3, 1, 2), k.double().permute(3, 2, 0, 1), b.double(), padding=1)
    y = y.permute(0, 2, 3, 1)
    return torch.relu(y) if relu else y


def _run(B, H, W, C, N, cfg, ks, relu=1, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn((B, H, W, C), generator=g)
    k = torch.randn((3, 3, C, N), generator=g) / (3.0 * C ** 0.5)
    b = torch.randn(N, generator=g) * 0.1
    pc = C_.pack_conv_f32(k.numpy(), b.numpy(), 1, ((1, 1), (1, 1)), "cuda")
    assert pc.wino4s is not None
    out = torch.full((B, H, W, N), float("nan"), device="cuda")
    ctr = torch.zeros(1 << 14, dtype=torch.int32, device="cuda")
    for _ in range(2):                       # twice: the fused fixup must leave its counters zero
        C_.conv_forward_f32(x.cuda(), pc, out, relu=relu, cfg=cfg, ksplit=ks, counters=ctr)
    torch.cuda.synchronize()
    assert int(ctr.abs().sum()) == 0
    torch.cuda.synchronize()
    want = _oracle(x, k, b, relu)
    got = out.double().cpu()
    assert torch.isfinite(got).all()
    return ((got - want).abs().max() / want.abs().max()).item()


@pytest.mark.parametrize("cfg", CFGS)
def test_resnet_stage_shapes_whole_k(cfg):
    """The four ResNet-50 3x3 shapes at bs 2 (bs 32 runs in test_resnet_bs32_splits)."""
    for (H, C) in ((56, 64), (28, 128), (14, 256), (7, 512)):
        if not C_.kernels().wino4s_ok(cfg, C, C, 1):
            continue
        rel = _run(2, H, H, C, C, cfg, 1)
        assert rel < 3e-5, (cfg, H, C, rel)


@pytest.mark.parametrize("cfg", [220, 221, 223, 227, 228, 234, 236, 237])
@pytest.mark.parametrize("H,C,ks", [(56, 64, 1), (56, 64, 2), (56, 64, -2), (28, 128, 2), (28, 128, -2),
                                    (14, 256, 2), (14, 256, 4), (14, 256, -4), (7, 512, 4), (7, 512, 8),
                                    (7, 512, -8), (7, 512, -4)])
def test_resnet_bs32_splits(cfg, H, C, ks):
    if not C_.kernels().wino4s_ok(cfg, C, C, ks):
        pytest.skip("config / split not built for this shape")
    rel = _run(32, H, H, C, C, cfg, ks, seed=H)
    assert rel < 3e-5, rel


@pytest.mark.parametrize("B,H,W,C,N", [(1, 7, 7, 16, 16), (3, 13, 10, 32, 48), (1, 4, 4, 16, 32),
                                       (2, 9, 17, 48, 64), (5, 5, 6, 16, 16)])
def test_odd_maps_and_partial_tile_groups(B, H, W, C, N):
    """Edge tiles (H, W not multiples of 4), tile counts not multiples of 16, no ReLU."""
    for cfg in (220, 222, 225, 226):
        if not C_.kernels().wino4s_ok(cfg, C, N, 1):
            continue
        rel = _run(B, H, W, C, N, cfg, 1, relu=0, seed=B * H + W)
        assert rel < 3e-5, (cfg, rel)


@pytest.mark.parametrize("ks", [2, 4, 8])
def test_split_reduce_kernels_agree(ks, monkeypatch):
    """The split-count-templated reduce (default) and the generic one (ADAPT_W4S_REDUCE=0) give the same bits."""
    outs = []
    for mode in ("1", "0"):
        monkeypatch.setenv("ADAPT_W4S_REDUCE", mode)
        g = torch.Generator().manual_seed(ks)
        x = torch.randn((4, 7, 7, 512), generator=g).cuda()
        k = torch.randn((3, 3, 512, 512), generator=g) / 60.0
        pc = C_.pack_conv_f32(k.numpy(), np.zeros(512, np.float32), 1, ((1, 1), (1, 1)), "cuda")
        out = torch.full((4, 7, 7, 512), float("nan"), device="cuda")
        C_.conv_forward_f32(x, pc, out, relu=1, cfg=221, ksplit=ks)
        torch.cuda.synchronize()
        outs.append(out.cpu())
    assert torch.equal(outs[0], outs[1])


def test_rejects_residual_and_bad_split():
    pc = C_.pack_conv_f32(np.zeros((3, 3, 32, 32), np.float32), np.zeros(32, np.float32), 1, ((1, 1), (1, 1)),
                          "cuda")
    x = torch.zeros((1, 8, 8, 32), device="cuda")
    out = torch.zeros_like(x)
    with pytest.raises(ValueError):
        C_.conv_forward_f32(x, pc, out, residual=torch.zeros_like(x), cfg=220, ksplit=1)
    with pytest.raises(ValueError):
        C_.conv_forward_f32(x, pc, out, cfg=220, ksplit=4)          # 2 chunks cannot split 4 ways
    with pytest.raises(ValueError):
        C_.conv_forward_f32(x, pc, out, cfg=220, ksplit=-2)         # fused split-K without counters
