"""fp32 big-tile 1x1 GEMM (csrc/kernels/gemm_f32s.hip, cfg ids 300+) against a float64 CPU oracle of the same
1x1 conv (bias, optional residual, ReLU / ReLU6; stride 1 and 2; dual output of merged sibling convs), whole-K
tiles and stream-K over 256 blocks (the fused, deterministic fixup), on the ResNet-50 1x1 shapes at small batch
and on maps whose pixel count is not a tile multiple."""
import numpy as np
import pytest
import torch

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops import conv as C

from test_fp32_gpu import _ref_conv

pytestmark = pytest.mark.gpu

SHAPES = [  # (B, H, W, Cin, Cout, stride, residual, relu)
    (32, 14, 14, 1024, 256, 1, False, 1),     # the 256-tile shape of cfg 307
    (32, 7, 7, 512, 2048, 1, True, 1),        # ... and of cfg 308
    (32, 7, 7, 2048, 512, 1, False, 1),       # ... and of cfg 309
    (2, 14, 14, 1024, 256, 1, False, 1),
    (2, 7, 7, 2048, 512, 1, False, 1),
    (3, 14, 14, 256, 1024, 1, True, 1),
    (1, 28, 28, 512, 128, 1, False, 2),
    (2, 28, 28, 512, 1024, 2, False, 0),
    (5, 7, 9, 64, 48, 1, True, 0),
]


def _case(shape, seed):
    B, H, W, Cin, Cout, stride, has_res, relu = shape
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((B, H, W, Cin)).astype(np.float32)
    kern = (rng.standard_normal((1, 1, Cin, Cout)) / np.sqrt(Cin)).astype(np.float32)
    bias = rng.standard_normal(Cout).astype(np.float32)
    OH, OW = (H - 1) // stride + 1, (W - 1) // stride + 1
    res = rng.standard_normal((B, OH, OW, Cout)).astype(np.float32) if has_res else None
    return x, kern, bias, res, OH, OW


def _units(cfg, M, N, Cin):
    return C.f32s_tiles(cfg, M, N) * (Cin // 32)


@pytest.mark.parametrize("cfg", sorted(C.F32S_CFGS))
@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("ksplit", [1, -1])
def test_gemm_f32s_matches_fp64(shape, cfg, ksplit):
    B, H, W, Cin, Cout, stride, has_res, relu = shape
    x, kern, bias, res, OH, OW = _case(shape, sum(shape[:5]) + cfg)
    M = B * OH * OW
    units = _units(cfg, M, Cout, Cin)
    if ksplit < 0 and cfg in C.F32S_TM:
        pytest.skip("owned-row tiles run whole K only")
    if ksplit < 0:
        per = units // 256
        if per < 1 or -(-(Cin // 32) // per) + 1 > 16:
            pytest.skip("stream-K needs >= 256 (tile, chunk) units and <= 16 blocks per tile")
    want = _ref_conv(x, kern, bias, stride, ((0, 0), (0, 0)), res, relu)
    pc = C.pack_conv_f32(kern, bias, stride, ((0, 0), (0, 0)), "cuda")
    xd = torch.from_numpy(x).cuda()
    rd = None if res is None else torch.from_numpy(res).cuda()
    out = torch.empty((B, OH, OW, Cout), dtype=torch.float32, device="cuda")
    ctr = torch.zeros(C.f32s_tiles(cfg, M, Cout), dtype=torch.int32, device="cuda") if ksplit < 0 else None
    for rep in range(2 if ksplit < 0 else 1):          # the second launch checks the counters came back zero
        out.fill_(float("nan"))
        C.conv_forward_f32(xd, pc, out, rd, relu=relu, cfg=cfg, ksplit=ksplit, counters=ctr)
        got = out.cpu().numpy()
        err = np.abs(got - want).max() / max(1.0, np.abs(want).max())
        assert np.isfinite(got).all() and err < 2e-5, f"cfg {cfg} ksplit {ksplit} rep {rep}: rel err {err}"
    if ctr is not None:
        assert int(ctr.abs().sum()) == 0


@pytest.mark.parametrize("cfg", [300, 302])
def test_gemm_f32s_dual_output(cfg):
    """Merged sibling convs (runtime/plan.py merge_siblings): columns [0, ns) -> out with relu, the rest -> out2
    with relu2, both from one GEMM."""
    B, H, W, Cin, n1, n2 = 2, 28, 28, 256, 128, 512
    rng = np.random.default_rng(9)
    x = rng.standard_normal((B, H, W, Cin)).astype(np.float32)
    k = (rng.standard_normal((1, 1, Cin, n1 + n2)) / np.sqrt(Cin)).astype(np.float32)
    b = rng.standard_normal(n1 + n2).astype(np.float32)
    want = _ref_conv(x, k, b, 2, ((0, 0), (0, 0)), None, 0)
    pc = C.pack_conv_f32(k, b, 2, ((0, 0), (0, 0)), "cuda")
    pc.n_split = n1
    OH, OW = H // 2, W // 2
    out = torch.empty((B, OH, OW, n1), device="cuda")
    out2 = torch.empty((B, OH, OW, n2), device="cuda")
    C.conv_forward_f32(torch.from_numpy(x).cuda(), pc, out, relu=1, cfg=cfg, out2=out2, relu2=0)
    np.testing.assert_allclose(out.cpu().numpy(), np.maximum(want[..., :n1], 0), rtol=2e-5, atol=2e-5)
    np.testing.assert_allclose(out2.cpu().numpy(), want[..., n1:], rtol=2e-5, atol=2e-5)


def test_gemm_f32s_stream_k_is_deterministic():
    """The fixup adds the partial tiles in block order whoever arrives last: two launches are bit-identical."""
    B, H, W, Cin, Cout = 32, 14, 14, 1024, 256
    x, kern, bias, _, _, _ = _case((B, H, W, Cin, Cout, 1, False, 1), 4)
    pc = C.pack_conv_f32(kern, bias, 1, ((0, 0), (0, 0)), "cuda")
    xd = torch.from_numpy(x).cuda()
    ctr = torch.zeros(C.f32s_tiles(300, B * H * W, Cout), dtype=torch.int32, device="cuda")
    a = torch.empty((B, H, W, Cout), device="cuda")
    b = torch.empty_like(a)
    C.conv_forward_f32(xd, pc, a, relu=1, cfg=300, ksplit=-1, counters=ctr)
    C.conv_forward_f32(xd, pc, b, relu=1, cfg=300, ksplit=-1, counters=ctr)
    assert torch.equal(a, b)
    want = _ref_conv(x, kern, bias, 1, ((0, 0), (0, 0)), None, 1)
    assert np.abs(a.cpu().numpy() - want).max() / np.abs(want).max() < 2e-5
