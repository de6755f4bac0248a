"""Persistent pointwise conv (csrc/kernels/pw_wide.hip) against a float64 oracle
and against the implicit-GEMM path on the same packed weights."""
import numpy as np
import pytest
import torch

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops import conv as C

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("K,N,M", [(128, 512, 25088), (128, 512, 1000), (64, 256, 777)])
@pytest.mark.parametrize("cfg", sorted(C.PW_CFGS))
@pytest.mark.parametrize("res,relu", [(True, 1), (False, 0)])
def test_pw_matches_oracle(K, N, M, cfg, res, relu):
    rng = np.random.default_rng(K + N + M)
    kern = (rng.standard_normal((1, 1, K, N)) / np.sqrt(K)).astype(np.float32)
    bias = rng.standard_normal(N).astype(np.float32)
    pc = C.pack_conv(kern, bias, 1, ((0, 0), (0, 0)), "cuda")
    assert C.pw_supported(pc)
    x = torch.from_numpy(rng.standard_normal((M, K)).astype(np.float32)).cuda().to(torch.bfloat16)
    r = torch.from_numpy(rng.standard_normal((M, N)).astype(np.float32)).cuda().to(torch.bfloat16) if res else None
    out = torch.empty((M, N), dtype=torch.bfloat16, device="cuda")
    C.pw_forward(x, pc, out, r, relu=relu, cfg=cfg, blocks=64)
    w = pc.w.double()[:N, :K]
    want = x.double() @ w.T + pc.bias.double()
    if res:
        want = want + r.double()
    if relu:
        want = want.clamp_min(0)
    err = (out.double() - want).abs().max().item() / want.abs().max().item()
    assert err < 1e-2, err
    ref = torch.empty_like(out)
    C.conv_forward(x.view(1, 1, M, K), pc, ref.view(1, 1, M, N), None if r is None else r.view(1, 1, M, N),
                   relu=relu)
    assert (out.float() - ref.float()).abs().max().item() <= 2 * 2 ** -7 * max(1.0, ref.float().abs().max().item())
