"""fp32 persistent pointwise conv (csrc/kernels/pw_f32.hip, cfgs 120 / 121: filter slice register-resident,
persistent pixel tiles) against a float64 CPU reference: the ResNet-50 `_out` shapes with residual + ReLU,
a pixel count that is not a tile multiple, and no-residual / no-activation; the K-split tail configs
125 / 126 on the batch-32 shapes whose tiles leave a partial last round."""
import numpy as np
import pytest
import torch

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops import conv as C

pytestmark = pytest.mark.gpu

SHAPES = [  # B, H, W, K, N, residual, relu
    (2, 14, 14, 256, 1024, True, 1),
    (2, 28, 28, 128, 512, True, 1),
    (2, 7, 7, 512, 2048, True, 1),
    (2, 56, 56, 64, 256, True, 1),
    (1, 5, 3, 256, 512, False, 0),
    (2, 14, 14, 1024, 256, False, 1),          # K groups (partials meet in LDS)
    (1, 3, 5, 1024, 192, True, 0),
]


def _tail_scratch(cfg, M, K, N, n_split):
    """Skip a tail config when the launch has no partial last round to split (nothing else to pass)."""
    if cfg not in C.PW_F32_TAIL:
        return {}
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops._lib import kernels
    if kernels().pw_f32_fpw(K, N, n_split, C.PW_F32_CFGS[cfg]) <= 0:
        pytest.skip("no pointwise instance")
    tail, parts = kernels().pw_f32_tail_plan(M, K, N, n_split, C.PW_F32_CFGS[cfg])
    if not tail:
        pytest.skip("no partial last tile round (or one fragment per wave): nothing to split")
    assert parts >= 2
    return {}


TAIL_SHAPES = [  # B, H, W, K, N, residual, relu: 6 1/8 tiles per slot, 3 1/16, a ragged last tile
    (32, 28, 28, 128, 512, True, 1),
    (32, 28, 28, 512, 128, False, 1),
    (32, 14, 14, 256, 1024, True, 1),
    (32, 14, 14, 1024, 256, False, 1),
    (8, 56, 56, 64, 256, True, 1),
    (5, 30, 31, 512, 128, True, 0),
]


@pytest.mark.parametrize("shape", TAIL_SHAPES)
@pytest.mark.parametrize("cfg", sorted(C.PW_F32_TAIL))
def test_pw_f32_tail_split(shape, cfg):
    """The left-over tile round split by output fragment over idle waves: fp64 parity, and two launches
    bit-identical."""
    B, H, W, K, N, has_res, relu = shape
    rng = np.random.default_rng(K * 3 + N + cfg)
    x = torch.from_numpy(rng.standard_normal((B, H, W, K)).astype(np.float32)).cuda()
    kern = (rng.standard_normal((1, 1, K, N)) / np.sqrt(K)).astype(np.float32)
    bias = rng.standard_normal(N).astype(np.float32)
    res = torch.from_numpy(rng.standard_normal((B, H, W, N)).astype(np.float32)).cuda() if has_res else None
    pc = C.pack_conv_f32(kern, bias, 1, ((0, 0), (0, 0)), "cuda")
    if not C.f32_cfg_supported(cfg, K, N, pc):
        pytest.skip("no pointwise instance for this K / N")
    extra = _tail_scratch(cfg, B * H * W, K, N, 0)
    outs = []
    for _ in range(2):
        out = torch.full((B, H, W, N), float("nan"), device="cuda")
        C.conv_forward_f32(x, pc, out, res, relu=relu, cfg=cfg, **extra)
        outs.append(out.cpu())
    assert torch.equal(outs[0], outs[1])
    want = x.double().cpu().numpy().reshape(-1, K) @ kern[0, 0].astype(np.float64) + bias
    if res is not None:
        want = want + res.double().cpu().numpy().reshape(-1, N)
    if relu:
        want = np.maximum(want, 0)
    got = outs[0].numpy().reshape(-1, N)
    assert np.isfinite(got).all()
    err = np.abs(got - want).max() / max(1.0, np.abs(want).max())
    assert err < 2e-5, f"cfg {cfg}: rel err {err}"


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("cfg", sorted(C.PW_F32_CFGS))
def test_pw_f32_matches_fp64(shape, cfg):
    B, H, W, K, N, has_res, relu = shape
    rng = np.random.default_rng(K + N + cfg)
    x = rng.standard_normal((B, H, W, K)).astype(np.float32)
    kern = (rng.standard_normal((1, 1, K, N)) / np.sqrt(K)).astype(np.float32)
    bias = rng.standard_normal(N).astype(np.float32)
    res = rng.standard_normal((B, H, W, N)).astype(np.float32) if has_res else None
    pc = C.pack_conv_f32(kern, bias, 1, ((0, 0), (0, 0)), "cuda")
    if not C.f32_cfg_supported(cfg, K, N, pc):
        pytest.skip("tile size not built for this K")
    out = torch.full((B, H, W, N), float("nan"), device="cuda")
    extra = _tail_scratch(cfg, B * H * W, K, N, 0)
    C.conv_forward_f32(torch.from_numpy(x).cuda(), pc, out, None if res is None else torch.from_numpy(res).cuda(),
                       relu=relu, cfg=cfg, **extra)
    want = x.astype(np.float64) @ kern[0, 0].astype(np.float64) + bias
    if res is not None:
        want = want + res
    if relu:
        want = np.maximum(want, 0)
    got = out.cpu().numpy()
    assert np.isfinite(got).all()
    err = np.abs(got - want).max() / max(1.0, np.abs(want).max())
    assert err < 2e-5, f"cfg {cfg}: rel err {err}"


@pytest.mark.parametrize("cfg", [120, 122, 123, 125, 126])
@pytest.mark.parametrize("B,H,K,N0,N1", [(2, 56, 256, 512, 128), (2, 28, 512, 1024, 256), (1, 9, 256, 512, 128),
                                         (32, 56, 256, 512, 128), (32, 28, 512, 1024, 256)])
def test_pw_f32_strided_dual_output(cfg, B, H, K, N0, N1):
    """Merged sibling stride-2 1x1 convs (the ResNet projection shortcut + block-1 `_1` conv): one pointwise
    launch, columns >= N0 to the second output with their own activation."""
    rng = np.random.default_rng(B + H + K)
    x = rng.standard_normal((B, H, H, K)).astype(np.float32)
    kern = (rng.standard_normal((1, 1, K, N0 + N1)) / np.sqrt(K)).astype(np.float32)
    bias = rng.standard_normal(N0 + N1).astype(np.float32)
    pc = C.pack_conv_f32(kern, bias, 2, ((0, 0), (0, 0)), "cuda")
    pc.n_split = N0
    if not C.f32_cfg_supported(cfg, K, N0 + N1, pc):
        pytest.skip("no pointwise instance for this split")
    OH = (H - 1) // 2 + 1
    out = torch.full((B, OH, OH, N0), float("nan"), device="cuda")
    out2 = torch.full((B, OH, OH, N1), float("nan"), device="cuda")
    extra = _tail_scratch(cfg, B * OH * OH, K, N0 + N1, N0)
    C.conv_forward_f32(torch.from_numpy(x).cuda(), pc, out, relu=0, cfg=cfg, out2=out2, relu2=1, **extra)
    want = x[:, ::2, ::2, :].astype(np.float64) @ kern[0, 0].astype(np.float64) + bias
    for got, w in ((out, want[..., :N0]), (out2, np.maximum(want[..., N0:], 0))):
        g = got.cpu().numpy()
        assert np.isfinite(g).all()
        assert np.abs(g - w).max() / max(1.0, np.abs(w).max()) < 2e-5
