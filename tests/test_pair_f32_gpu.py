"""fp32 fused 1x1 pair (csrc/kernels/pw_pair_f32.hip, ResNet stage 2: 64 -> 256 -> 64) against a
float64 CPU reference of the two convs (BN folded, residual, ReLU), both tile sizes, pixel counts
that are and are not tile multiples; and its place in the fp32 ResNet-50 plan."""
import numpy as np
import pytest
import torch

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops import conv as C

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("bm", [16, 32])
@pytest.mark.parametrize("B,H,W", [(2, 56, 56), (1, 9, 9), (3, 7, 5)])
@pytest.mark.parametrize("grid", [0, 3])
def test_pair_f32_matches_fp64(bm, B, H, W, grid):
    rng = np.random.default_rng(B * 100 + H + bm)
    x = rng.standard_normal((B, H, W, 64)).astype(np.float32)
    res = rng.standard_normal((B, H, W, 256)).astype(np.float32)
    k3 = (rng.standard_normal((1, 1, 64, 256)) / 8).astype(np.float32)
    b3 = rng.standard_normal(256).astype(np.float32) * 0.1
    k1 = (rng.standard_normal((1, 1, 256, 64)) / 16).astype(np.float32)
    b1 = rng.standard_normal(64).astype(np.float32) * 0.1
    pp = C.pack_pair_f32(k3, b3, k1, b1, "cuda")
    y = torch.full((B, H, W, 256), float("nan"), device="cuda")
    z = torch.full((B, H, W, 64), float("nan"), device="cuda")
    C.pair_f32_forward(torch.from_numpy(x).cuda(), torch.from_numpy(res).cuda(), pp, y, z, bm=bm, grid=grid)
    yw = np.maximum(x.astype(np.float64) @ k3[0, 0].astype(np.float64) + b3 + res, 0)
    zw = np.maximum(yw @ k1[0, 0].astype(np.float64) + b1, 0)
    for got, want, nm in ((y, yw, "y"), (z, zw, "z")):
        g = got.cpu().numpy()
        assert np.isfinite(g).all(), nm
        err = np.abs(g - want).max() / max(1.0, np.abs(want).max())
        assert err < 2e-5, f"{nm}: rel err {err}"


def test_pair_f32_rejects_other_shapes():
    with pytest.raises(ValueError):
        C.pack_pair_f32(np.zeros((1, 1, 128, 512)), np.zeros(512), np.zeros((1, 1, 512, 128)), np.zeros(128), "cuda")
