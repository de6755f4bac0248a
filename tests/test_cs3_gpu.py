"""Channel-split register-resident 3x3 conv (csrc/kernels/conv3x3_cs.hip): the
ResNet stage-4 (14x14, 256 -> 256) and stage-5 (7x7, 512 -> 512) shapes, BN folded,
against an fp32 PyTorch reference of the same conv, plus its shape checks and
its place in a ResNet-50 bf16 plan."""
import math

import pytest
import torch
import torch.nn.functional as F

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops import conv as C

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


@pytest.mark.parametrize("shape", [(14, 256), (7, 512)])
@pytest.mark.parametrize("B", [1, 5, 32])
@pytest.mark.parametrize("relu", [True, False])
def test_cs3_matches_torch(shape, B, relu):
    _need_gpu()
    hw, c = shape
    g = torch.Generator().manual_seed(B * 7 + c)
    x = torch.randn(B, hw, hw, c, generator=g).cuda().to(torch.bfloat16)
    kern = (torch.randn(3, 3, c, c, generator=g) / math.sqrt(9 * c)).numpy()
    bias = (torch.randn(c, generator=g) * 0.1).numpy()
    pc = C.pack_conv(kern, bias, 1, ((1, 1), (1, 1)), "cuda")
    assert C.cfg_supported(73, pc, False)
    out = torch.full((B, hw, hw, c), float("nan"), device="cuda", dtype=torch.bfloat16)
    C.conv_forward(x, pc, out, relu=relu, cfg=73)
    torch.cuda.synchronize()
    w = torch.from_numpy(kern).cuda().to(torch.bfloat16).float().permute(3, 2, 0, 1)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w, torch.from_numpy(bias).cuda(), padding=1).permute(0, 2, 3, 1)
    if relu:
        ref = ref.clamp_min(0)
    assert torch.isfinite(out.float()).all()
    err = (out.float() - ref).abs().max().item()
    assert err <= 1e-2 * ref.abs().max().item() + 1e-2, f"max err {err}"


def test_cs3_rejects_other_shapes():
    _need_gpu()
    pc = C.pack_conv(torch.zeros(3, 3, 256, 256).numpy(), torch.zeros(256).numpy(), 1, ((1, 1), (1, 1)), "cuda")
    x = torch.zeros(2, 28, 28, 256, device="cuda", dtype=torch.bfloat16)
    with pytest.raises(ValueError):
        C.conv_forward(x, pc, torch.empty_like(x), relu=True, cfg=73)
    pc2 = C.pack_conv(torch.zeros(3, 3, 128, 128).numpy(), torch.zeros(128).numpy(), 1, ((1, 1), (1, 1)), "cuda")
    assert not C.cfg_supported(73, pc2, False)
    pc3 = C.pack_conv(torch.zeros(3, 3, 256, 256).numpy(), torch.zeros(256).numpy(), 2, ((1, 1), (1, 1)), "cuda")
    assert not C.cfg_supported(73, pc3, False)
