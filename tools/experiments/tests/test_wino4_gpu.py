"""fp32 Winograd F(4x4, 3x3) conv kernels (csrc/kernels/conv_wino4_f32.hip, cfg 200; the producer / consumer
form csrc/kernels/conv_wino4pc_f32.hip, cfg 210) against a float64
CPU oracle of the same 3x3 / stride-1 / pad-1 conv (bias, optional residual, ReLU / ReLU6), whole-K,
slab split-K and fused split-K, on the ResNet stage shapes at small batch and on odd maps (partial
tiles, tile groups straddling rows and images).  F(4x4) on fp32 must stay within 1e-4 of the fp64
oracle (the F(2x2) kernels measure ~1e-6): the transforms' integer coefficients grow the rounding
error by ~10x, which the measured error is printed against."""
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
    (2, 7, 7, 512, 128, False, 1),
    (1, 9, 13, 32, 32, True, 0),
    (5, 12, 7, 16, 64, False, 1),
]


def _case(shape, seed):
    B, H, W, Cin, Cout, has_res, relu = shape
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((B, H, W, Cin)).astype(np.float32)
    kern = (rng.standard_normal((3, 3, Cin, Cout)) / np.sqrt(9 * Cin)).astype(np.float32)
    bias = rng.standard_normal(Cout).astype(np.float32)
    res = rng.standard_normal((B, H, W, Cout)).astype(np.float32) if has_res else None
    return x, kern, bias, res


@pytest.mark.parametrize("cfg", [200, 210])
@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("ksplit", [1, 2, 4, -2, -4, -8])
def test_wino4_f32_matches_fp64(shape, ksplit, cfg):
    B, H, W, Cin, Cout, has_res, relu = shape
    if abs(ksplit) not in C.wino4_splits(Cin):
        pytest.skip("split-K needs an even chunk count per split")
    x, kern, bias, res = _case(shape, sum(shape[:5]) * 7 + abs(ksplit))
    pads = ((1, 1), (1, 1))
    want = _ref_conv(x, kern, bias, 1, pads, res, relu)
    pc = C.pack_conv_f32(kern, bias, 1, pads, "cuda")
    assert pc.wino4 is not None
    xd = torch.from_numpy(x).cuda()
    rd = None if res is None else torch.from_numpy(res).cuda()
    out = torch.empty((B, H, W, Cout), dtype=torch.float32, device="cuda")
    ctr = torch.zeros(C.wino4_blocks(B, H, W, Cout), dtype=torch.int32, device="cuda") if ksplit < 0 else None
    for rep in range(2 if ksplit < 0 else 1):        # the second launch checks the counters came back zero
        out.fill_(float("nan"))
        C.conv_forward_f32(xd, pc, out, rd, relu=relu, cfg=cfg, ksplit=ksplit, counters=ctr)
        got = out.cpu().numpy()
        err = np.abs(got - want).max() / max(1.0, np.abs(want).max())
        print(f"F(4x4) cfg {cfg} {shape} ksplit {ksplit}: rel err {err:.2e}")
        assert np.isfinite(got).all() and err < 1e-4, f"ksplit {ksplit} rep {rep}: rel err {err}"
    if ctr is not None:
        assert int(ctr.abs().sum()) == 0, "fused split-K left arrival counters non-zero"


@pytest.mark.parametrize("cfg", [200, 210])
def test_wino4_fused_split_matches_slab_split(cfg):
    """The fused fixup adds the same slabs in the same (split) order as splitk_reduce_f32."""
    B, H, W, Cin, Cout = 4, 14, 14, 256, 256
    x, kern, bias, _ = _case((B, H, W, Cin, Cout, False, 1), 5)
    pc = C.pack_conv_f32(kern, bias, 1, ((1, 1), (1, 1)), "cuda")
    xd = torch.from_numpy(x).cuda()
    a = torch.empty((B, H, W, Cout), device="cuda")
    b = torch.empty_like(a)
    ctr = torch.zeros(C.wino4_blocks(B, H, W, Cout), dtype=torch.int32, device="cuda")
    C.conv_forward_f32(xd, pc, a, relu=1, cfg=cfg, ksplit=4)
    C.conv_forward_f32(xd, pc, b, relu=1, cfg=cfg, ksplit=-4, counters=ctr)
    assert torch.equal(a, b)


def test_wino4_error_against_f2x2():
    """F(4x4)'s fp32 error on the stage-5 shape (K = 4608), printed next to F(2x2)'s."""
    B, H, W, Cin, Cout = 8, 7, 7, 512, 512
    x, kern, bias, _ = _case((B, H, W, Cin, Cout, False, 0), 3)
    want = _ref_conv(x, kern, bias, 1, ((1, 1), (1, 1)), None, 0)
    pc = C.pack_conv_f32(kern, bias, 1, ((1, 1), (1, 1)), "cuda")
    xd = torch.from_numpy(x).cuda()
    out = torch.empty((B, H, W, Cout), device="cuda")
    errs = {}
    for cfg, ks in ((200, 1), (210, 1), (118, 1)):
        C.conv_forward_f32(xd, pc, out, cfg=cfg, ksplit=ks)
        errs[cfg] = np.abs(out.cpu().numpy() - want).max() / np.abs(want).max()
    print(f"stage-5 3x3 rel err vs fp64: F(4x4) {errs[200]:.2e} / pc {errs[210]:.2e}, F(2x2) {errs[118]:.2e}")
    assert errs[200] < 1e-4 and errs[210] < 1e-4


def test_wino4_rejects_bad_splits_and_maps():
    kern = np.zeros((3, 3, 64, 64), np.float32)
    pc = C.pack_conv_f32(kern, np.zeros(64, np.float32), 1, ((1, 1), (1, 1)), "cuda")
    x = torch.zeros((1, 8, 8, 64), device="cuda")
    out = torch.empty((1, 8, 8, 64), device="cuda")
    with pytest.raises(ValueError):
        C.conv_forward_f32(x, pc, out, cfg=200, ksplit=8)      # 8 chunks / 8 splits: odd per split
    with pytest.raises(ValueError):
        C.conv_forward_f32(torch.zeros((1, 4, 4, 64), device="cuda"), pc, torch.empty((1, 4, 4, 64), device="cuda"),
                           cfg=200)                            # one tile per row
