"""3x3 conv with the filter resident in VGPRs (csrc/kernels/conv3x3_rr.hip), the
ResNet stage-3 shape (28x28, 128 -> 128, pad 1, BN folded, ReLU), against an fp32
PyTorch reference of the same conv, and the tile config's shape checks."""
import math

import pytest
import torch
import torch.nn.functional as F

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops import conv as C

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B", [1, 3, 32])
@pytest.mark.parametrize("relu", [True, False])
@pytest.mark.parametrize("cfg", sorted(C.RR3_CFGS))
def test_rr3_matches_torch(B, relu, cfg):
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    g = torch.Generator().manual_seed(B)
    x = torch.randn(B, 28, 28, 128, generator=g).cuda().to(torch.bfloat16)
    kern = (torch.randn(3, 3, 128, 128, generator=g) / math.sqrt(9 * 128)).numpy()
    bias = (torch.randn(128, generator=g) * 0.1).numpy()
    pc = C.pack_conv(kern, bias, 1, ((1, 1), (1, 1)), "cuda")
    assert C.cfg_supported(cfg, pc, False)
    out = torch.empty(B, 28, 28, 128, device="cuda", dtype=torch.bfloat16)
    C.conv_forward(x, pc, out, relu=relu, cfg=cfg)
    torch.cuda.synchronize()
    w = torch.from_numpy(kern).cuda().to(torch.bfloat16).float().permute(3, 2, 0, 1)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w, torch.from_numpy(bias).cuda(), padding=1).permute(0, 2, 3, 1)
    if relu:
        ref = ref.clamp_min(0)
    err = (out.float() - ref).abs().max().item()
    assert err <= 1e-2 * ref.abs().max().item() + 1e-2, f"max err {err}"


def test_rr3_rejects_other_shapes():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    kern = torch.zeros(3, 3, 128, 128).numpy()
    pc = C.pack_conv(kern, torch.zeros(128).numpy(), 1, ((1, 1), (1, 1)), "cuda")
    x = torch.zeros(2, 14, 14, 128, device="cuda", dtype=torch.bfloat16)
    with pytest.raises(ValueError):
        C.conv_forward(x, pc, torch.empty_like(x), relu=True, cfg=71)
    pc2 = C.pack_conv(torch.zeros(3, 3, 64, 64).numpy(), torch.zeros(64).numpy(), 1, ((1, 1), (1, 1)), "cuda")
    assert not C.cfg_supported(71, pc2, False)
