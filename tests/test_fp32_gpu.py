"""fp32 execution path (csrc/kernels/conv_f32.hip) against fp32/fp64 oracles.

The reference computes in Keras float32 (`src/node.py:177`,
`test/local_infer.py:22`); `SliceExecutor(precision="fp32")` runs every conv /
GEMM on the fp32 matrix cores (v_mfma_f32_16x16x4_f32) with fp32 activations.
Kernel checks compare with a float64 CPU oracle; the model check compares the
pre-softmax logits of ResNet-50 with the fp32 CPU oracle at rel <= 1e-4.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops import conv as C
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops import eltwise as E

pytestmark = pytest.mark.gpu


def _ref_conv(x, k, b, stride, pads, res=None, relu=0):
    """float64 CPU oracle: NHWC x, HWIO k."""
    (pt, pb), (pl, pr) = pads
    xt = torch.from_numpy(x).double().permute(0, 3, 1, 2)
    xt = F.pad(xt, (pl, pr, pt, pb))
    y = F.conv2d(xt, torch.from_numpy(k).double().permute(3, 2, 0, 1), torch.from_numpy(b).double(), stride=stride)
    y = y.permute(0, 2, 3, 1)
    if res is not None:
        y = y + torch.from_numpy(res).double()
    if relu == 1:
        y = y.clamp_min(0)
    elif relu == 2:
        y = y.clamp(0, 6)
    return y.numpy()


SHAPES = [  # (B, H, W, Cin, Cout, k, stride, pad, residual, relu)
    (2, 56, 56, 3, 64, 7, 2, 3, False, 1),          # stem: 3-channel gather path
    (2, 28, 28, 64, 256, 1, 1, 0, True, 1),         # 1x1 + residual + ReLU (pure GEMM path)
    (2, 28, 28, 64, 64, 3, 1, 1, False, 1),         # 3x3 halo
    (2, 28, 28, 128, 256, 1, 2, 0, False, 0),       # strided projection shortcut
    (4, 7, 7, 512, 2048, 1, 1, 0, True, 1),         # small-M stage-5 shape
    (3, 14, 14, 256, 96, 3, 1, 1, False, 2),        # ReLU6, N not a tile multiple
]


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("ksplit", [1, 4, -1, -2])
def test_conv_f32_matches_fp64(shape, ksplit):
    """Every fp32 tile config; ksplit > 1 split-K slabs, ksplit < 0 stream-K (v2 configs)."""
    B, H, W, Cin, Cout, k, s, pad, has_res, relu = shape
    rng = np.random.default_rng(hash(shape) % 2**32)
    x = rng.standard_normal((B, H, W, Cin)).astype(np.float32)
    kern = (rng.standard_normal((k, k, Cin, Cout)) / np.sqrt(k * k * Cin)).astype(np.float32)
    bias = rng.standard_normal(Cout).astype(np.float32)
    pads = ((pad, pad), (pad, pad))
    OH = (H + 2 * pad - k) // s + 1
    OW = (W + 2 * pad - k) // s + 1
    res = rng.standard_normal((B, OH, OW, Cout)).astype(np.float32) if has_res else None
    want = _ref_conv(x, kern, bias, s, pads, res, relu)
    pc = C.pack_conv_f32(kern, bias, s, pads, "cuda")
    out = torch.empty((B, OH, OW, Cout), dtype=torch.float32, device="cuda")
    M = B * OH * OW
    for cfg in C.F32_TILES:
        if not C.f32_cfg_supported(cfg, Cin, Cout) or (ksplit < 0 and cfg not in C.F32G_CFGS):
            continue
        ctr = None
        if ksplit < 0:
            ctr = torch.zeros(C.f32_sk_plan(M, Cout, pc.Kpad, cfg, -ksplit)[0], dtype=torch.int32, device="cuda")
        out.fill_(float("nan"))
        for _rep in range(2 if ksplit < 0 else 1):       # stream-K counters must come back zeroed
            C.conv_forward_f32(torch.from_numpy(x).cuda(), pc, out,
                               None if res is None else torch.from_numpy(res).cuda(),
                               relu=relu, cfg=cfg, ksplit=ksplit, counters=ctr)
        if ctr is not None:
            assert int(ctr.abs().sum()) == 0, f"cfg {cfg}: stream-K counters not reset"
        got = out.cpu().numpy()
        err = np.abs(got - want).max() / max(1.0, np.abs(want).max())
        assert err < 2e-5, f"cfg {cfg} ksplit {ksplit}: rel err {err}"


def test_dense_f32_split_k():
    rng = np.random.default_rng(0)
    x = rng.standard_normal((32, 2048)).astype(np.float32)
    w = (rng.standard_normal((2048, 1000)) / 45).astype(np.float32)
    b = rng.standard_normal(1000).astype(np.float32)
    pc = C.pack_conv_f32(w.reshape(1, 1, 2048, 1000), b, 1, ((0, 0), (0, 0)), "cuda")
    out = torch.empty((32, 1000), dtype=torch.float32, device="cuda")
    C.conv_forward_f32(torch.from_numpy(x).cuda(), pc, out, cfg=3, ksplit=16)
    want = x.astype(np.float64) @ w.astype(np.float64) + b
    assert np.abs(out.cpu().numpy() - want).max() / np.abs(want).max() < 2e-5


@pytest.mark.parametrize("M,K,N", [(32, 2048, 1000), (1, 2048, 1000), (5, 1280, 1000), (17, 4096, 10), (32, 96, 130)])
def test_dense_small_f32_head(M, K, N):
    """fp32 small-M head (head.hip dense_partial_f32_kernel + finish): logits against fp64, softmax
    probabilities of those logits."""
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops import eltwise as E
    rng = np.random.default_rng(M * 7 + K)
    x = rng.standard_normal((M, K)).astype(np.float32)
    w = (rng.standard_normal((K, N)) / np.sqrt(K)).astype(np.float32)
    b = rng.standard_normal(N).astype(np.float32)
    pc = C.pack_conv_f32(w.reshape(1, 1, K, N), b, 1, ((0, 0), (0, 0)), "cuda")
    part = torch.empty(E.dense_small_f32_scratch(M, N, pc.Kpad), dtype=torch.float32, device="cuda")
    logits = torch.full((M, N), float("nan"), device="cuda")
    probs = torch.full((M, N), float("nan"), device="cuda")
    E.dense_small_f32(torch.from_numpy(x).cuda(), pc, part, logits=logits, probs=probs)
    want = x.astype(np.float64) @ w.astype(np.float64) + b
    got = logits.cpu().numpy()
    assert np.abs(got - want).max() / np.abs(want).max() < 2e-5
    e = np.exp(want - want.max(1, keepdims=True))
    assert np.abs(probs.cpu().numpy() - e / e.sum(1, keepdims=True)).max() < 1e-5


def test_f32_layers():
    rng = np.random.default_rng(1)
    x = torch.from_numpy(rng.standard_normal((2, 15, 15, 64)).astype(np.float32))
    y = torch.empty((2, 8, 8, 64), device="cuda")
    E.maxpool_f32(x.cuda(), y, 3, 2, 1, 1, pad_zero=False)
    want = F.max_pool2d(F.pad(x.permute(0, 3, 1, 2), (1, 1, 1, 1), value=float("-inf")), 3, 2).permute(0, 2, 3, 1)
    assert torch.equal(y.cpu(), want)
    g = torch.empty((2, 64), device="cuda")
    E.gap_f32(x.cuda(), g)
    assert torch.allclose(g.cpu(), x.mean(dim=(1, 2)), rtol=1e-6, atol=1e-6)
    a, b2 = x.cuda(), torch.from_numpy(rng.standard_normal((2, 15, 15, 64)).astype(np.float32)).cuda()
    o = torch.empty_like(a)
    E.eltwise_f32(a, o, b=b2, relu=1)
    assert torch.allclose(o, (a + b2).clamp_min(0))
    sc, sh = torch.rand(64, device="cuda"), torch.rand(64, device="cuda")
    E.eltwise_f32(a, o, scale=sc, shift=sh)
    assert torch.allclose(o, a * sc + sh, rtol=1e-6, atol=1e-6)
    p = torch.empty((2, 17, 17, 64), device="cuda")
    E.pad_f32(a, p, 1, 1)
    assert torch.equal(p.cpu(), F.pad(x.permute(0, 3, 1, 2), (1, 1, 1, 1)).permute(0, 2, 3, 1))


@pytest.mark.parametrize("shape", [(2, 56, 56, 96), (3, 33, 40, 1160), (1, 112, 112, 32)])
def test_gap_f32_large_map_sliced(shape):
    """Maps of >= GAP_LARGE_HW pixels take the two-pass sliced kernel (C/4 > 256 exercises the channel groups)."""
    x = torch.from_numpy(np.random.default_rng(4).standard_normal(shape).astype(np.float32))
    B, H, W, Cc = shape
    assert H * W >= E.GAP_LARGE_HW
    g = torch.empty((B, Cc), device="cuda")
    E.gap_f32(x.cuda(), g)
    torch.cuda.synchronize()
    want = x.double().mean(dim=(1, 2))
    assert torch.allclose(g.cpu().double(), want, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("C", [8, 6])             # 4-channel vector kernels / scalar fallback
@pytest.mark.parametrize("k,stride", [(3, 1), (5, 2), (2, 1)])
def test_f32_dwconv_avgpool_vector_and_scalar(C, k, stride):
    rng = np.random.default_rng(7)
    x = torch.from_numpy(rng.standard_normal((2, 13, 11, C)).astype(np.float32))
    w = torch.from_numpy(rng.standard_normal((k, k, C)).astype(np.float32))
    bias = torch.from_numpy(rng.standard_normal(C).astype(np.float32))
    p = k // 2
    OH, OW = (13 + 2 * p - k) // stride + 1, (11 + 2 * p - k) // stride + 1
    xt = F.pad(x.permute(0, 3, 1, 2).double(), (p, p, p, p))
    for act, fn in ((1, lambda t: t.clamp_min(0)), (3, lambda t: t * torch.sigmoid(t))):
        y = torch.empty((2, OH, OW, C), device="cuda")
        E.dwconv_f32(x.cuda(), w.cuda(), bias.cuda(), y, stride, ((p, p), (p, p)), act=act)
        want = F.conv2d(xt, w.double().permute(2, 0, 1).unsqueeze(1), bias.double(), stride=stride, groups=C)
        assert torch.allclose(y.cpu().double(), fn(want).permute(0, 2, 3, 1), rtol=1e-5, atol=1e-5)
    y = torch.empty((2, OH, OW, C), device="cuda")
    E.avgpool_f32(x.cuda(), y, k, stride, ((p, p), (p, p)))
    want = F.avg_pool2d(xt, k, stride, count_include_pad=False) if p == 0 else \
        F.avg_pool2d(x.permute(0, 3, 1, 2).double(), k, stride, padding=p, count_include_pad=False)
    assert torch.allclose(y.cpu().double(), want.permute(0, 2, 3, 1), rtol=1e-5, atol=1e-6)
    a = x.cuda()
    se = torch.from_numpy(rng.standard_normal((2, C)).astype(np.float32)).cuda()
    o = torch.empty_like(a)
    E.binary_f32(a, se, o, "mul")
    assert torch.allclose(o, a * se[:, None, None, :], rtol=1e-6, atol=1e-6)
    sc, sh = torch.rand(C, device="cuda"), torch.rand(C, device="cuda")
    E.affine_act_f32(a, o, sc, sh, act=3)
    t = a * sc + sh
    assert torch.allclose(o, t * torch.sigmoid(t), rtol=1e-5, atol=1e-5)
    cat = torch.empty((2, 13, 11, 2 * C), device="cuda")
    E.concat_f32([a, o], cat)
    assert torch.equal(cat, torch.cat([a, o], dim=-1))


def _oracle_logits(g, w, x):
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops.reference import \
        ReferenceExecutor
    feat = ReferenceExecutor(g, w, device="cpu").run({g.input: torch.from_numpy(x)}, outputs=["avg_pool"])["avg_pool"]
    return feat.double().numpy() @ w["predictions/kernel"].astype(np.float64) + w["predictions/bias"]


@pytest.mark.parametrize("depth", ["resnet50", "resnet152"])
def test_resnet_fp32_logits_match_oracle(depth):
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models import resnet as R
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.runtime.executor import \
        SliceExecutor
    g = R.build_resnet(depth)
    w = R.init_weights(g, seed=0)
    x = np.random.default_rng(2).standard_normal((2, 224, 224, 3)).astype(np.float32)
    ex = SliceExecutor(g, w, batch=2, device="cuda:0", precision="fp32")
    ex.capture()
    probs = ex(torch.from_numpy(x).cuda())
    logits = ex.logits().double().cpu().numpy()
    want = _oracle_logits(g, w, x)
    rel = np.abs(logits - want).max() / np.abs(want).max()
    assert rel <= 1e-4, f"{depth} fp32 logits rel err {rel}"
    assert (logits.argmax(-1) == want.argmax(-1)).all()
    sm = np.exp(want - want.max(-1, keepdims=True))
    sm /= sm.sum(-1, keepdims=True)
    assert np.abs(probs.double().cpu().numpy() - sm).max() < 1e-5


def test_resnet50_bf16_logits_and_top1():
    """The bf16 fast path against the same fp32 oracle: logits within a bf16
    budget, top-1 equal wherever the oracle's top-2 margin exceeds that budget."""
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models import resnet as R
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.runtime.executor import \
        SliceExecutor
    g = R.build_resnet("resnet50")
    w = R.init_weights(g, seed=0)
    x = np.random.default_rng(3).standard_normal((8, 224, 224, 3)).astype(np.float32)
    ex = SliceExecutor(g, w, batch=8, device="cuda:0", precision="bf16")
    ex(torch.from_numpy(x).cuda())
    logits = ex.logits().double().cpu().numpy()
    want = _oracle_logits(g, w, x)
    scale = np.abs(want).max()
    rel = np.abs(logits - want).max() / scale
    assert rel <= 5e-2, f"bf16 logits rel err {rel}"
    top2 = np.sort(want, -1)[:, -2:]
    clear = (top2[:, 1] - top2[:, 0]) > 2 * rel * scale
    assert (logits.argmax(-1) == want.argmax(-1))[clear].all()


@pytest.mark.parametrize("name", ["mobilenet_v2", "densenet121", "efficientnetb0", "inception_v3"])
def test_other_families_fp32_logits_match_oracle(name):
    """fp32 execution of the other Keras application families (depthwise conv,
    average pool, concat, swish / sigmoid, squeeze-excite multiply, rescaling /
    normalization layers on the fp32 kernels): logits vs the fp32 CPU oracle."""
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.resnet import \
        init_weights
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.zoo import \
        build_model
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops.reference import \
        ReferenceExecutor
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.runtime.executor import \
        SliceExecutor
    g = build_model(name)
    w = init_weights(g, seed=0)
    shape = tuple(g.layers[g.input].out_shape)
    x = np.random.default_rng(5).uniform(0, 255, (2,) + shape).astype(np.float32)
    ex = SliceExecutor(g, w, batch=2, device="cuda:0", precision="fp32")
    probs = ex(torch.from_numpy(x).cuda())
    logits = ex.logits().double().cpu().numpy()
    feat_name = g.layers[g.output].inputs[0]
    feat = ReferenceExecutor(g, w, device="cpu").run({g.input: torch.from_numpy(x)}, outputs=[feat_name])[feat_name]
    want = feat.double().reshape(2, -1).numpy() @ w[f"{g.output}/kernel"].astype(np.float64) + w[f"{g.output}/bias"]
    rel = np.abs(logits - want).max() / np.abs(want).max()
    assert rel <= 1e-3, f"{name} fp32 logits rel err {rel}"
    assert (logits.argmax(-1) == want.argmax(-1)).all()
    assert torch.isfinite(probs).all()


@pytest.mark.parametrize("variant", [0, 1, 2, 5, 6])
@pytest.mark.parametrize("B,H", [(2, 224), (1, 64), (3, 112)])
def test_stem_f32_fused_matches_fp64(B, H, variant):
    """csrc/kernels/stem_f32.hip: 7x7/s2 conv (+bias, ReLU) + 3x3/s2 max-pool in one launch vs a float64 oracle."""
    rng = np.random.default_rng(H + B)
    x = rng.standard_normal((B, H, H, 3)).astype(np.float32)
    kern = (rng.standard_normal((7, 7, 3, 64)) / np.sqrt(147)).astype(np.float32)
    bias = (0.1 * rng.standard_normal(64)).astype(np.float32)
    pads = ((3, 3), (3, 3))
    conv = _ref_conv(x, kern, bias, 2, pads, None, 1)                    # B, OH, OW, 64
    t = torch.from_numpy(conv).permute(0, 3, 1, 2)
    want = F.max_pool2d(F.pad(t, (1, 1, 1, 1)), 3, 2).permute(0, 2, 3, 1).numpy()
    ps = C.pack_stem_f32(kern, bias, pads, "cuda")
    out = torch.full(want.shape, float("nan"), dtype=torch.float32, device="cuda")
    C.stem_f32_forward(torch.from_numpy(x).cuda(), ps, out, variant=variant)
    got = out.cpu().numpy()
    err = np.abs(got - want).max() / max(1.0, np.abs(want).max())
    assert np.isfinite(got).all() and err < 2e-5, f"rel err {err}"


def test_resnet50_fp32_plan_uses_fused_stem_and_v2_convs():
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.resnet import (
        build_resnet, init_weights)
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.runtime.executor import (
        SliceExecutor)
    g = build_resnet("resnet50")
    ex = SliceExecutor(g, init_weights(g, 0), 32, device="cuda", precision="fp32")
    kinds = [st.kind for st in ex.steps]
    assert kinds[0] == "stem_f32" and "maxpool" not in kinds
    v2 = [c for i, (c, _) in ex.cfg.items() if c in C.F32G_CFGS]
    print(f"fp32 plan: {len(ex.steps)} steps, {len(v2)} of {len(ex.cfg)} GEMMs on the v2 LDS-DMA kernel")
    # the round-3 kernels are on the tuned bs=32 plan, not silently replaced by a generic path
    assert kinds.count("pair") == 2                                    # pw_pair_f32.hip, stage 2
    assert sum(1 for st in ex.steps if st.kind == "conv" and st.p.get("out2")) == 4     # merged siblings
    cfgs = {c for c, _ in ex.cfg.values()}
    assert cfgs & set(C.WINO_F32_CFGS), "no Winograd config on the fp32 3x3 convs"
    assert cfgs & set(C.PW_F32_CFGS), "no persistent pointwise config on the fp32 1x1 convs"
    # every 3x3 runs a Winograd kernel: F(2x2) fused (stages 2-3) or the F(4x4) transform + GEMM pipeline
    # (stages 4-5, wino4s_f32.hip, the whole-model A/B winner of round 6)
    wino3x3 = [i for i, st in enumerate(ex.steps) if st.kind == "conv" and st.p.get("kernel") == (3, 3)]
    wino = set(C.WINO_F32_CFGS) | set(C.WINO4S_F32_CFGS)
    assert wino3x3 and all(ex.cfg[i][0] in wino for i in wino3x3)
    assert sum(1 for i in wino3x3 if ex.cfg[i][0] in C.WINO4S_F32_CFGS) == 12     # 3 stage-2 + 6 stage-4 + 3 stage-5
