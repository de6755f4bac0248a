"""Channel-sliced persistent pointwise conv (csrc/kernels/pw_slice.hip, cfg ids 74-79) against a float64 oracle
of the same bf16 1x1 conv (bias, optional residual, ReLU) and against the implicit-GEMM path on the same packed
weights: the ResNet-50 stage-3/4/5 1x1 shapes it takes at bs=32 and ragged pixel counts."""
import numpy as np
import pytest
import torch

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops import conv as C

pytestmark = pytest.mark.gpu

SHAPES = [  # (M, K, N, residual)
    (25088, 128, 512, True),      # stage-3 _out
    (6272, 256, 1024, True),      # stage-4 _out
    (6272, 1024, 256, False),     # stage-4 _1
    (1568, 512, 2048, True),      # stage-5 _out
    (25088, 512, 128, False),     # stage-3 _1
    (777, 256, 512, True),        # ragged last tile
    (100, 1024, 128, False),
]


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("cfg", sorted(C.PS_CFGS))
@pytest.mark.parametrize("relu", [1, 0])
def test_pw_slice_matches_oracle(shape, cfg, relu):
    M, K, N, res = shape
    rng = np.random.default_rng(M + K + N + cfg)
    kern = (rng.standard_normal((1, 1, K, N)) / np.sqrt(K)).astype(np.float32)
    bias = rng.standard_normal(N).astype(np.float32)
    pc = C.pack_conv(kern, bias, 1, ((0, 0), (0, 0)), "cuda")
    if not C.ps_supported(pc, cfg):
        pytest.skip(f"cfg {cfg} does not take K={K}, N={N}")
    x = torch.from_numpy(rng.standard_normal((M, K)).astype(np.float32)).cuda().to(torch.bfloat16)
    r = torch.from_numpy(rng.standard_normal((M, N)).astype(np.float32)).cuda().to(torch.bfloat16) if res else None
    out = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device="cuda")
    C.ps_forward(x, pc, out, r, relu=relu, cfg=cfg, blocks=256)
    w = pc.w.double()[:N, :K]
    want = x.double() @ w.T + pc.bias.double()
    if res:
        want = want + r.double()
    if relu:
        want = want.clamp_min(0)
    got = out.double()
    assert torch.isfinite(got).all()
    err = (got - want).abs().max().item() / want.abs().max().item()
    assert err < 1e-2, err
    ref = torch.empty_like(out)
    C.conv_forward(x.view(1, 1, M, K), pc, ref.view(1, 1, M, N), None if r is None else r.view(1, 1, M, N),
                   relu=relu)
    assert (out.float() - ref.float()).abs().max().item() <= 2 * 2 ** -7 * max(1.0, ref.float().abs().max().item())


@pytest.mark.parametrize("blocks", [1, 7, 64, 1000])
def test_pw_slice_any_grid(blocks):
    """Walkers = blocks / slices, at least one and at most the tile count: every grid covers every tile."""
    M, K, N = 1000, 256, 1024
    rng = np.random.default_rng(blocks)
    pc = C.pack_conv((rng.standard_normal((1, 1, K, N)) / 16).astype(np.float32),
                     rng.standard_normal(N).astype(np.float32), 1, ((0, 0), (0, 0)), "cuda")
    x = torch.from_numpy(rng.standard_normal((M, K)).astype(np.float32)).cuda().to(torch.bfloat16)
    out = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device="cuda")
    C.ps_forward(x, pc, out, None, relu=0, cfg=74, blocks=blocks)
    want = x.double() @ pc.w.double()[:N, :K].T + pc.bias.double()
    assert (out.double() - want).abs().max().item() / want.abs().max().item() < 1e-2
