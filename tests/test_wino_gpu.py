"""fp32 Winograd F(2x2, 3x3) conv kernel (csrc/kernels/conv_wino_f32.hip, cfgs 80-85) against a
float64 CPU oracle of the same 3x3 / stride-1 / pad-1 conv (bias, optional residual, ReLU / ReLU6),
every config, whole-K and split-K, on even and odd maps (ResNet stages 2-5 shapes at small batch)."""
import numpy as np
import pytest
import torch

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops import conv as C

from test_fp32_gpu import _ref_conv

pytestmark = pytest.mark.gpu

SHAPES = [  # (B, H, W, Cin, Cout, residual, relu)
    (2, 56, 56, 64, 64, False, 1),
    (2, 28, 28, 128, 128, False, 1),
    (3, 14, 14, 256, 96, True, 2),
    (2, 7, 7, 512, 192, False, 1),
    (1, 9, 5, 32, 48, False, 0),
]


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("ksplit", [1, 2, 4])
def test_wino_f32_matches_fp64(shape, ksplit):
    B, H, W, Cin, Cout, has_res, relu = shape
    if ksplit > Cin // 16:
        pytest.skip("split-K beyond the 16-channel chunks")
    rng = np.random.default_rng(hash(shape) % 2**32)
    x = rng.standard_normal((B, H, W, Cin)).astype(np.float32)
    kern = (rng.standard_normal((3, 3, Cin, Cout)) / np.sqrt(9 * Cin)).astype(np.float32)
    bias = rng.standard_normal(Cout).astype(np.float32)
    pads = ((1, 1), (1, 1))
    res = rng.standard_normal((B, H, W, Cout)).astype(np.float32) if has_res else None
    want = _ref_conv(x, kern, bias, 1, pads, res, relu)
    pc = C.pack_conv_f32(kern, bias, 1, pads, "cuda")
    assert pc.wino is not None
    xd = torch.from_numpy(x).cuda()
    rd = None if res is None else torch.from_numpy(res).cuda()
    out = torch.empty((B, H, W, Cout), dtype=torch.float32, device="cuda")
    ran = 0
    for cfg in C.WINO_F32_CFGS:
        if not C.f32_cfg_supported(cfg, Cin, Cout, pc) or not C.wino_map_ok(cfg, H, W):
            continue
        out.fill_(float("nan"))
        C.conv_forward_f32(xd, pc, out, rd, relu=relu, cfg=cfg, ksplit=ksplit)
        got = out.cpu().numpy()
        err = np.abs(got - want).max() / max(1.0, np.abs(want).max())
        assert np.isfinite(got).all() and err < 2e-5, f"cfg {cfg} ksplit {ksplit}: rel err {err}"
        ran += 1
    assert ran > 0


def test_wino_f32_rejects_other_convs():
    kern = np.zeros((3, 3, 64, 64), np.float32)
    pc = C.pack_conv_f32(kern, np.zeros(64, np.float32), 2, ((0, 1), (0, 1)), "cuda")
    x = torch.zeros((1, 8, 8, 64), device="cuda")
    with pytest.raises(ValueError):
        C.conv_forward_f32(x, pc, torch.empty((1, 4, 4, 64), device="cuda"), cfg=80)
