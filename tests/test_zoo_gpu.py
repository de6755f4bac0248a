"""MI355X numerics for the layers beyond ResNet (csrc/kernels/layers.hip:
depthwise conv, average pool, channel concat; ReLU6 in every fused epilogue)
and for whole VGG16 / MobileNetV2 / DenseNet121 / Keras-JSON graphs through
the HIP runtime, each against the plain PyTorch fp32 reference."""
import importlib
import json

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
PKG = "adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd"


@pytest.fixture(scope="module")
def ops():
    return importlib.import_module(f"{PKG}.ops.eltwise"), importlib.import_module(f"{PKG}.ops.conv")


@pytest.mark.parametrize("B,H,W,C,k,s,pads,act", [
    (2, 56, 56, 32, 3, 1, ((1, 1), (1, 1)), 2), (2, 112, 112, 96, 3, 2, ((0, 1), (0, 1)), 2),
    (3, 14, 14, 576, 3, 1, ((1, 1), (1, 1)), 0), (1, 7, 9, 40, 3, 2, ((1, 1), (1, 1)), 1),
    (2, 10, 10, 16, 5, 1, ((2, 2), (2, 2)), 2),
    # large stride-1 maps take the register-blocked 3x3 kernel (OW tail of 2 in the last case)
    (16, 112, 112, 32, 3, 1, ((1, 1), (1, 1)), 2), (64, 30, 30, 96, 3, 1, ((1, 1), (1, 1)), 1)])
def test_dwconv_vs_torch(ops, B, H, W, C, k, s, pads, act):
    E, _ = ops
    torch.manual_seed(0)
    x = torch.randn(B, H, W, C, device="cuda").to(torch.bfloat16)
    w = torch.randn(k, k, C, device="cuda") * 0.3
    b = torch.randn(C, device="cuda") * 0.1
    (pt, pb), (pl, pr) = pads
    OH, OW = (H + pt + pb - k) // s + 1, (W + pl + pr - k) // s + 1
    out = torch.empty(B, OH, OW, C, device="cuda", dtype=torch.bfloat16)
    E.dwconv(x, w.contiguous(), b, out, s, pads, act=act)
    xr = F.pad(x.float().permute(0, 3, 1, 2), (pl, pr, pt, pb))
    ref = F.conv2d(xr, w.permute(2, 0, 1).unsqueeze(1), b, stride=s, groups=C).permute(0, 2, 3, 1)
    if act:
        ref = torch.relu(ref)
    if act == 2:
        ref = ref.clamp(max=6.0)
    torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("k,s,pads", [(2, 2, ((0, 0), (0, 0))), (3, 1, ((1, 1), (1, 1))), (3, 2, ((0, 1), (0, 1)))])
def test_avgpool_vs_torch(ops, k, s, pads):
    E, _ = ops
    x = torch.randn(2, 28, 28, 64, device="cuda").to(torch.bfloat16)
    (pt, pb), (pl, pr) = pads
    OH, OW = (28 + pt + pb - k) // s + 1, (28 + pl + pr - k) // s + 1
    out = torch.empty(2, OH, OW, 64, device="cuda", dtype=torch.bfloat16)
    E.avgpool(x, out, k, s, pads)
    xr = x.float().permute(0, 3, 1, 2)
    num = F.avg_pool2d(F.pad(xr, (pl, pr, pt, pb)), k, s, divisor_override=1)
    den = F.avg_pool2d(F.pad(torch.ones_like(xr[:, :1]), (pl, pr, pt, pb)), k, s, divisor_override=1)
    torch.testing.assert_close(out.float(), (num / den).permute(0, 2, 3, 1), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("chans", [(64, 32), (96, 32, 32), (16, 24), (20, 12, 5)])
def test_concat_vs_torch(ops, chans):
    E, _ = ops
    pad8 = lambda c: (c + 7) // 8 * 8  # noqa: E731
    xs, real = [], []
    for c in chans:
        t = torch.randn(2, 7, 9, c, device="cuda").to(torch.bfloat16)
        real.append(t)
        xs.append(F.pad(t, (0, pad8(c) - c)).contiguous())
    total = sum(chans)
    out = torch.full((2, 7, 9, pad8(total)), 7.0, device="cuda", dtype=torch.bfloat16)
    E.concat(xs, list(chans), out, total)
    torch.testing.assert_close(out[..., :total], torch.cat(real, -1))
    assert (out[..., total:] == 0).all()


def test_relu6_in_conv_epilogue_and_eltwise(ops):
    E, C = ops
    torch.manual_seed(1)
    x = (torch.randn(2, 14, 14, 64, device="cuda") * 4).to(torch.bfloat16)
    kern = (torch.randn(1, 1, 64, 128) / 2).numpy()
    pc = C.pack_conv(kern, torch.zeros(128).numpy(), 1, ((0, 0), (0, 0)), "cuda")
    out = torch.empty(2, 14, 14, 128, device="cuda", dtype=torch.bfloat16)
    C.conv_forward(x, pc, out, relu=2)
    ref = (x.float().reshape(-1, 64) @ torch.from_numpy(kern[0, 0]).cuda().to(torch.bfloat16).float())
    torch.testing.assert_close(out.float().reshape(-1, 128), ref.clamp(0, 6), rtol=2e-2, atol=3e-2)
    y = torch.empty_like(x)
    E.relu(x, y, mode=2)
    torch.testing.assert_close(y.float(), x.float().clamp(0, 6))
    sc, sh = torch.full((64,), 2.0, device="cuda"), torch.ones(64, device="cuda")
    E.bn_act(x, sc, sh, y, relu=2)
    torch.testing.assert_close(y.float(), (x.float() * 2 + 1).clamp(0, 6), rtol=1e-2, atol=2e-2)


def _model_check(g, w, batch, feat, size, rel_tol=3e-2):
    ex_mod = importlib.import_module(f"{PKG}.runtime.executor")
    ref_mod = importlib.import_module(f"{PKG}.ops.reference")
    gen = torch.Generator().manual_seed(0)
    x = torch.randn(batch, *size, generator=gen).cuda()
    ref = ref_mod.ReferenceExecutor(g, w, device="cuda").run({g.input: x}, outputs=[feat, g.output])
    ex = ex_mod.SliceExecutor(g, w, batch=batch, outputs=[feat, g.output], precision="bf16")
    ex.capture()
    got = ex.run({g.input: x})
    torch.cuda.synchronize()
    f, fr = got[feat].float().reshape(batch, -1), ref[feat].float().reshape(batch, -1)
    rel = ((f - fr).norm() / fr.norm()).item()
    assert rel < rel_tol, f"{feat}: relative error {rel}"
    p = got[g.output].float()
    assert torch.allclose(p.sum(-1), torch.ones(batch, device="cuda"), atol=1e-3)
    assert (p - ref[g.output]).abs().sum(-1).max().item() < 0.1


@pytest.mark.parametrize("name,batch,feat", [("vgg16", 2, "fc2"), ("mobilenet_v2", 4, "global_average_pooling2d"),
                                             ("densenet121", 2, "avg_pool"), ("inception_v3", 2, "avg_pool")])
def test_zoo_model_vs_oracle(name, batch, feat):
    zoo = importlib.import_module(f"{PKG}.models.zoo")
    res = importlib.import_module(f"{PKG}.models.resnet")
    g = zoo.build_model(name)
    size = (299, 299, 3) if name == "inception_v3" else (224, 224, 3)
    _model_check(g, res.init_weights(g, 0), batch, feat, size, rel_tol=5e-2)


def test_keras_json_model_vs_oracle():
    kj = importlib.import_module(f"{PKG}.graph.keras_json")
    res = importlib.import_module(f"{PKG}.models.resnet")
    zoo = importlib.import_module(f"{PKG}.models.zoo")
    # MobileNetV2 through the Keras JSON bridge: export, re-import, run on the HIP runtime
    g = kj.from_keras_json(kj.to_keras_json(zoo.build_model("mobilenet_v2", input_shape=(96, 96, 3), classes=10)))
    assert json.loads(g.to_json())["layers"][0]["op"] == "input"
    _model_check(g, res.init_weights(g, 1), 4, "out_relu", (96, 96, 3), rel_tol=5e-2)


ACT_NAMES = ["relu", "relu6", "swish", "sigmoid", "tanh", "hard_sigmoid", "hard_swish", "gelu", "elu", "selu",
             "softplus", "leaky_relu"]


@pytest.mark.parametrize("fn", ACT_NAMES)
def test_act_kernel_vs_keras_definition(ops, fn):
    E, _ = ops
    ref_mod = importlib.import_module(f"{PKG}.ops.reference")
    x = (torch.randn(4, 9, 7, 24, device="cuda") * 3).to(torch.bfloat16)
    out = torch.empty_like(x)
    E.act(x, out, E.ACT_MODES[fn], alpha=0.2)
    ref = ref_mod._act(x.float(), fn, 0.2)
    torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("fn", ["add", "sub", "mul", "max", "min", "avg"])
@pytest.mark.parametrize("bcast", [False, True])
def test_binary_kernel(ops, fn, bcast):
    E, _ = ops
    a = torch.randn(3, 5, 6, 32, device="cuda").to(torch.bfloat16)
    b = torch.randn(3, 1, 1, 32, device="cuda").to(torch.bfloat16) if bcast else torch.randn_like(a)
    out = torch.empty_like(a)
    E.binary(a, b, out, fn, act_mode=E.ACT_MODES["swish"] if fn == "mul" else 0)
    af, bf = a.float(), b.float()
    ref = {"add": af + bf, "sub": af - bf, "mul": af * bf, "max": torch.maximum(af, bf),
           "min": torch.minimum(af, bf), "avg": 0.5 * (af + bf)}[fn]
    if fn == "mul":
        ref = ref * torch.sigmoid(ref)
    torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=2e-2)


def test_gmp_kernel(ops):
    E, _ = ops
    x = torch.randn(4, 7, 7, 1040, device="cuda").to(torch.bfloat16)
    out = torch.empty(4, 1040, device="cuda", dtype=torch.bfloat16)
    E.gmp(x, out)
    torch.testing.assert_close(out, x.amax(dim=(1, 2)))


def test_efficientnet_b0_vs_oracle():
    zoo = importlib.import_module(f"{PKG}.models.zoo")
    res = importlib.import_module(f"{PKG}.models.resnet")
    g = zoo.build_model("efficientnetb0")
    _model_check(g, res.init_weights(g, 0), 4, "avg_pool", (224, 224, 3), rel_tol=5e-2)


def test_keras_json_se_model_vs_oracle():
    kj = importlib.import_module(f"{PKG}.graph.keras_json")
    res = importlib.import_module(f"{PKG}.models.resnet")
    from tests.test_model_zoo import _se_keras
    g = kj.from_keras_json(_se_keras())
    _model_check(g, res.init_weights(g, 2), 4, "gelu", (12, 12, 3), rel_tol=5e-2)


@pytest.mark.parametrize("B,H,W,C", [(32, 112, 112, 32), (4, 56, 56, 144), (3, 33, 37, 2056), (2, 7, 7, 2048)])
def test_gap_large_and_small_maps(ops, B, H, W, C):
    E, _ = ops
    x = torch.randn(B, H, W, C, device="cuda").to(torch.bfloat16)
    out = torch.empty(B, C, device="cuda", dtype=torch.bfloat16)
    need = E.gap_scratch_elems(B, H * W, C)
    scratch = torch.empty(max(need, 1), device="cuda", dtype=torch.float32)
    E.gap(x, out=out, scratch=scratch)
    torch.testing.assert_close(out.float(), x.float().mean(dim=(1, 2)), rtol=1e-2, atol=1e-2)
    assert (need > 0) == (H * W >= E.GAP_LARGE_HW)


def test_dense_with_non_relu_activation_chain():
    """Dense(swish) -> Dense(sigmoid) -> Dense(softmax) (bf16 hidden activations, post-activation steps)."""
    kj = importlib.import_module(f"{PKG}.graph.keras_json")
    res = importlib.import_module(f"{PKG}.models.resnet")

    def L(cls, name, inbound, **cfg):
        cfg["name"] = name
        return {"class_name": cls, "config": cfg, "name": name,
                "inbound_nodes": [[[i, 0, 0, {}] for i in inbound]] if inbound else []}
    layers = [L("InputLayer", "img", [], batch_input_shape=[None, 4, 4, 8]),
              L("Flatten", "fl", ["img"]),
              L("Dense", "h1", ["fl"], units=64, activation="swish"),
              L("Dense", "h2", ["h1"], units=32, activation="sigmoid"),
              L("Dense", "predictions", ["h2"], units=16, activation="softmax")]
    js = json.dumps({"class_name": "Functional", "config": {"name": "mlp", "layers": layers,
                                                            "input_layers": [["img", 0, 0]],
                                                            "output_layers": [["predictions", 0, 0]]}})
    g = kj.from_keras_json(js)
    _model_check(g, res.init_weights(g, 5), 4, "h2", (4, 4, 8), rel_tol=5e-2)
