"""Numerics of every gfx950 kernel against a plain PyTorch fp32 reference
(SURVEY §4 item 2).  Runs only on the MI355X box (`-m gpu`)."""
import importlib
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

PKG = "adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd"

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ops():
    import importlib
    conv = importlib.import_module(f"{PKG}.ops.conv")
    E = importlib.import_module(f"{PKG}.ops.eltwise")
    lib = importlib.import_module(f"{PKG}.ops._lib")
    lib.kernels()   # must load the in-tree HIP library
    return conv, E


def _ref_conv(x_nhwc, k_hwio, bias, stride, pads, residual=None, relu=False):
    x = x_nhwc.float().permute(0, 3, 1, 2)
    (pt, pb), (pl, pr) = pads
    x = F.pad(x, (pl, pr, pt, pb))
    w = k_hwio.float().permute(3, 2, 0, 1)
    y = F.conv2d(x, w, bias.float(), stride=stride).permute(0, 2, 3, 1)
    if residual is not None:
        y = y + residual.float()
    if relu:
        y = torch.relu(y)
    return y


CONV_CASES = [
    # B, H, W, Cin, Cout, k, stride, pad
    (2, 56, 56, 64, 64, 1, 1, 0),
    (2, 56, 56, 64, 256, 1, 1, 0),
    (2, 56, 56, 64, 64, 3, 1, 1),
    (2, 56, 56, 256, 128, 1, 2, 0),
    (2, 28, 28, 128, 128, 3, 1, 1),
    (4, 7, 7, 512, 512, 3, 1, 1),
    (2, 14, 14, 256, 256, 3, 1, 1),
    (3, 13, 11, 128, 64, 3, 1, 1),     # odd spatial sizes for the halo tiles
    (2, 14, 14, 1024, 2048, 1, 2, 0),
    (2, 224, 224, 8, 64, 7, 2, 3),     # stem (input padded to 8 channels)
    (3, 9, 11, 24, 40, 3, 2, 1),       # odd sizes, M/N tails
]


conv_ops = importlib.import_module(f"{PKG}.ops.conv")
ALL_CFGS = sorted(conv_ops.CFG_TILES)


@pytest.mark.parametrize("case", CONV_CASES)
@pytest.mark.parametrize("cfg", [None] + ALL_CFGS)
def test_conv_vs_torch(ops, case, cfg):
    conv, _ = ops
    B, H, W, Cin, Cout, k, s, p = case
    torch.manual_seed(0)
    dev = "cuda"
    x = torch.randn(B, H, W, Cin, device=dev).to(torch.bfloat16)
    kern = (torch.randn(k, k, Cin, Cout) / math.sqrt(k * k * Cin)).numpy()
    bias = (torch.randn(Cout) * 0.1).numpy()
    pc = conv.pack_conv(kern, bias, s, ((p, p), (p, p)), dev)
    OH, OW = pc.out_hw(H, W)
    res = torch.randn(B, OH, OW, Cout, device=dev).to(torch.bfloat16)
    out = torch.empty(B, OH, OW, Cout, device=dev, dtype=torch.bfloat16)
    ks = 1
    ws = None
    halo = cfg in conv.HALO_PATCH
    if cfg is not None and pc.Kpad // 64 >= 4 and not halo:
        ks = 2 if cfg % 2 == 0 else 3
        ws = torch.empty(ks * B * OH * OW * Cout, device=dev, dtype=torch.float32)
    pure = k == 1 and s == 1 and p == 0
    if cfg is not None and (not conv.cfg_supported(cfg, pc, pure) or (halo and conv.halo_rows(cfg, pc, H, W) < 1)):
        with pytest.raises(ValueError):
            conv.conv_forward(x, pc, out, residual=res, relu=True, cfg=cfg, ksplit=ks, workspace=ws)
        return
    conv.conv_forward(x, pc, out, residual=res, relu=True, cfg=cfg, ksplit=ks, workspace=ws)
    torch.cuda.synchronize()
    wq = torch.from_numpy(kern).to(dev).to(torch.bfloat16).float()      # kernel sees bf16 weights
    ref = _ref_conv(x, wq, torch.from_numpy(bias).to(dev), s, ((p, p), (p, p)), res, True)
    err = (out.float() - ref).abs().max().item()
    scale = ref.abs().max().item() + 1e-6
    assert err <= 2e-2 * scale + 1e-2, f"max err {err} (scale {scale})"


@pytest.mark.parametrize("B,H,W,pool", [(4, 224, 224, True), (3, 224, 224, False), (2, 64, 48, True),
                                         (2, 37, 29, True), (1, 21, 30, False), (3, 230, 218, True)])
@pytest.mark.parametrize("version", ["v6", "v4", "v3", "v2", "v1"])
def test_stem_vs_torch(ops, B, H, W, pool, version, monkeypatch):
    """Fused fp32-image -> conv1(7x7/s2)+BN+ReLU [-> 3x3/s2 max-pool] vs F.conv2d/F.max_pool2d
    (v2 = row-group kernel with the conv-row ring; v3 = v2 with the whole patch requested up front;
    v1 = one pool row per block; v4 = 8 waves, pool of step k-1 beside the conv of step k)."""
    monkeypatch.setenv("ADAPT_STEM_V1", {"v1": "1", "v2": "0", "v3": "3", "v4": "4", "v6": "6"}[version])
    conv, _ = ops
    dev = "cuda"
    torch.manual_seed(1)
    x = torch.randn(B, H, W, 3, device=dev) * 40.0          # caffe-preprocessed pixel scale
    kern = (torch.randn(7, 7, 3, 64) / math.sqrt(147) / 40.0).numpy()
    bias = (torch.randn(64) * 0.1).numpy()
    ps = conv.pack_stem(kern, bias, ((3, 3), (3, 3)), dev)
    OH, OW = ps.out_hw(H, W)
    if pool:
        PH, PW = (OH - 1) // 2 + 1, (OW - 1) // 2 + 1
        out = torch.empty(B, PH, PW, 64, device=dev, dtype=torch.bfloat16)
    else:
        out = torch.empty(B, OH, OW, 64, device=dev, dtype=torch.bfloat16)
    conv.stem_forward(x, ps, out, pool=pool)
    torch.cuda.synchronize()
    xq = x.to(torch.bfloat16).float()                       # kernel stages the image as bf16
    wq = torch.from_numpy(kern).to(dev).to(torch.bfloat16).float()
    ref = _ref_conv(xq, wq, torch.from_numpy(bias).to(dev), 2, ((3, 3), (3, 3)), None, True)
    if pool:
        r = F.pad(ref.permute(0, 3, 1, 2), (1, 1, 1, 1))    # ZeroPadding2D(1) then MaxPool2D(3, 2)
        ref = F.max_pool2d(r, 3, 2).permute(0, 2, 3, 1)
    assert out.shape == ref.shape
    err = (out.float() - ref).abs().max().item()
    scale = ref.abs().max().item() + 1e-6
    assert err <= 2e-2 * scale + 1e-2, f"max err {err} (scale {scale})"


@pytest.mark.parametrize("B,H,W", [(32, 224, 224), (3, 230, 218)])
def test_stem_versions_bitwise_equal(ops, B, H, W, monkeypatch):
    """v1 - v4 and v6 of the pooled bf16 stem do the same sums in the same order: bit-identical outputs."""
    conv, _ = ops
    torch.manual_seed(2)
    x = torch.randn(B, H, W, 3, device="cuda") * 40.0
    kern = (torch.randn(7, 7, 3, 64) / math.sqrt(147) / 40.0).numpy()
    ps = conv.pack_stem(kern, (torch.randn(64) * 0.1).numpy(), ((3, 3), (3, 3)), "cuda")
    OH, OW = ps.out_hw(H, W)
    outs = []
    for ver in ("1", "0", "3", "4", "6"):
        monkeypatch.setenv("ADAPT_STEM_V1", ver)
        out = torch.full((B, (OH - 1) // 2 + 1, (OW - 1) // 2 + 1, 64), float("nan"), device="cuda",
                         dtype=torch.bfloat16)
        conv.stem_forward(x, ps, out, pool=True)
        outs.append(out.cpu())
    assert all(torch.equal(outs[0], o) for o in outs[1:])


V2_CFGS = [c for c in ALL_CFGS if c >= 6 and c not in conv_ops.HALO_PATCH]


@pytest.mark.parametrize("case", [c for c in CONV_CASES if c[3] % 64 == 0])
@pytest.mark.parametrize("cfg", V2_CFGS)
@pytest.mark.parametrize("mult", [1, 2])
def test_conv_stream_k(ops, case, cfg, mult):
    """Stream-K (ksplit < 0): partial tiles published by one block and combined by
    the last arriver must match torch, be bitwise reproducible and leave the
    tile counters at zero."""
    conv, _ = ops
    B, H, W, Cin, Cout, k, s, p = case
    torch.manual_seed(0)
    dev = "cuda"
    x = torch.randn(B, H, W, Cin, device=dev).to(torch.bfloat16)
    kern = (torch.randn(k, k, Cin, Cout) / math.sqrt(k * k * Cin)).numpy()
    bias = (torch.randn(Cout) * 0.1).numpy()
    pc = conv.pack_conv(kern, bias, s, ((p, p), (p, p)), dev)
    OH, OW = pc.out_hw(H, W)
    M = B * OH * OW
    res = torch.randn(B, OH, OW, Cout, device=dev).to(torch.bfloat16)
    out = torch.empty(B, OH, OW, Cout, device=dev, dtype=torch.bfloat16)
    tiles, grid, iters, need = conv.sk_plan(M, Cout, pc.Kpad, cfg, mult)
    ws = torch.empty(need, device=dev, dtype=torch.float32)
    ctr = torch.zeros(tiles, device=dev, dtype=torch.int32)
    conv.conv_forward(x, pc, out, residual=res, relu=True, cfg=cfg, ksplit=-mult, workspace=ws, counters=ctr)
    torch.cuda.synchronize()
    assert int(ctr.abs().sum()) == 0
    out2 = torch.empty_like(out)
    conv.conv_forward(x, pc, out2, residual=res, relu=True, cfg=cfg, ksplit=-mult, workspace=ws, counters=ctr)
    torch.cuda.synchronize()
    assert torch.equal(out, out2)
    wq = torch.from_numpy(kern).to(dev).to(torch.bfloat16).float()
    ref = _ref_conv(x, wq, torch.from_numpy(bias).to(dev), s, ((p, p), (p, p)), res, True)
    err = (out.float() - ref).abs().max().item()
    scale = ref.abs().max().item() + 1e-6
    assert err <= 2e-2 * scale + 1e-2, f"max err {err} (scale {scale}) grid {grid} iters {iters}"


def test_conv_f32_out_dense(ops):
    conv, _ = ops
    dev = "cuda"
    B, K, N = 32, 2048, 1000
    x = torch.randn(B, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(K, N) / math.sqrt(K)).numpy()
    b = torch.randn(N).numpy()
    pc = conv.pack_conv(w.reshape(1, 1, K, N), b, 1, ((0, 0), (0, 0)), dev)
    out = torch.empty(B, N, device=dev, dtype=torch.float32)
    conv.conv_forward(x, pc, out)
    ref = x.float() @ torch.from_numpy(w).to(dev).to(torch.bfloat16).float() + torch.from_numpy(b).to(dev)
    assert torch.allclose(out, ref, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("M,K,N", [(32, 2048, 1000), (1, 2048, 1000), (7, 512, 10), (20, 1000, 37), (4, 512, 1500)])
def test_dense_small_head(ops, M, K, N):
    """Small-M classifier GEMM (+bias, + softmax) of csrc/kernels/head.hip vs torch fp32."""
    conv, E = ops
    dev = "cuda"
    torch.manual_seed(3)
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(K, N) / math.sqrt(K)).numpy()
    b = (torch.randn(N) * 0.1).numpy()
    pc = conv.pack_conv(w.reshape(1, 1, K, N), b, 1, ((0, 0), (0, 0)), dev)
    part = torch.empty(E.dense_small_scratch(M, N, K), device=dev)
    logits = torch.empty(M, N, device=dev)
    probs = torch.empty(M, N, device=dev)
    E.dense_small(x, pc, part, logits=logits, probs=probs)
    torch.cuda.synchronize()
    ref = x.float() @ torch.from_numpy(w).to(dev).to(torch.bfloat16).float() + torch.from_numpy(b).to(dev)
    assert torch.allclose(logits, ref, atol=2e-2, rtol=2e-2)
    assert torch.allclose(probs, torch.softmax(ref, -1), atol=1e-3, rtol=2e-2)


@pytest.mark.parametrize("B,H,W,C", [(32, 7, 7, 2048), (3, 5, 9, 64), (2, 1, 1, 520)])
def test_gap(ops, B, H, W, C):
    _, E = ops
    x = torch.randn(B, H, W, C, device="cuda").to(torch.bfloat16)
    y = torch.empty(B, C, device="cuda", dtype=torch.bfloat16)
    y32 = torch.empty(B, C, device="cuda")
    E.gap(x, out=y, out32=y32)
    torch.cuda.synchronize()
    ref = x.float().mean(dim=(1, 2))
    assert torch.allclose(y32, ref, atol=1e-3, rtol=1e-3)
    assert torch.allclose(y.float(), ref, atol=1e-2, rtol=1e-2)


def test_eltwise(ops):
    _, E = ops
    dev = "cuda"
    torch.manual_seed(1)
    x = torch.randn(2, 9, 10, 64, device=dev).to(torch.bfloat16)
    y = torch.randn(2, 9, 10, 64, device=dev).to(torch.bfloat16)
    out = torch.empty_like(x)
    E.relu(x, out)
    assert torch.equal(out, torch.relu(x))
    E.add_act(x, y, out, relu=True)
    assert torch.allclose(out.float(), torch.relu(x.float() + y.float()), atol=1e-2, rtol=1e-2)
    sc = torch.rand(64, device=dev) + 0.5
    sh = torch.randn(64, device=dev)
    E.bn_act(x, sc, sh, out, relu=False)
    assert torch.allclose(out.float(), x.float() * sc + sh, atol=2e-2, rtol=1e-2)
    # maxpool with Keras zero-pad semantics
    xp = torch.randn(2, 112, 112, 64, device=dev).to(torch.bfloat16)
    mp = torch.empty(2, 56, 56, 64, device=dev, dtype=torch.bfloat16)
    E.maxpool(xp, mp, 3, 2, 1, 1, True)
    ref = F.max_pool2d(F.pad(xp.float().permute(0, 3, 1, 2), (1, 1, 1, 1)), 3, 2).permute(0, 2, 3, 1)
    assert torch.equal(mp.float(), ref)
    # gap
    g = torch.empty(2, 64, device=dev, dtype=torch.bfloat16)
    g32 = torch.empty(2, 64, device=dev, dtype=torch.float32)
    E.gap(xp, g, g32)
    assert torch.allclose(g32, xp.float().mean(dim=(1, 2)), atol=1e-3, rtol=1e-3)
    # softmax
    lg = torch.randn(4, 1000, device=dev) * 5
    pr = torch.empty_like(lg)
    E.softmax_rows(lg, pr)
    assert torch.allclose(pr, torch.softmax(lg, -1), atol=1e-5, rtol=1e-4)
    # input pack + pad
    img = torch.randn(2, 5, 6, 3, device=dev)
    pk = torch.empty(2, 5, 6, 8, device=dev, dtype=torch.bfloat16)
    E.input_pack(img, pk)
    assert torch.equal(pk[..., :3], img.to(torch.bfloat16)) and pk[..., 3:].abs().sum().item() == 0
    pd = torch.empty(2, 11, 12, 64, device=dev, dtype=torch.bfloat16)
    E.pad(x, pd, 1, 1)
    assert torch.equal(pd, F.pad(x, (0, 0, 1, 1, 1, 1)))


@pytest.mark.parametrize("n_elems", [1, 7, 513, 100_000, 3_211_264])
def test_gpu_lz4_roundtrip_and_host_interop(ops, n_elems):
    import importlib
    gl = importlib.import_module(f"{PKG}.codec.gpu_lz4")
    rt = importlib.import_module(f"{PKG}.native").runtime()
    torch.manual_seed(n_elems)
    # post-ReLU bf16 activations: ~half zeros, the case the side-stream codec targets
    x = torch.relu(torch.randn(n_elems, device="cuda")).to(torch.bfloat16)
    codec = gl.GpuLZ4(x.numel() * 2 + 4096)
    codec.compress(x)
    frame = codec.frame_bytes()
    host = rt.lz4_decompress(frame)                       # standard LZ4 frame
    assert host == x.view(torch.uint8).cpu().numpy().tobytes()
    y = torch.empty_like(x)
    codec.decompress(frame, y)
    torch.cuda.synchronize()
    assert torch.equal(y.view(torch.int16), x.view(torch.int16))
    if n_elems >= 100_000:
        assert len(frame) <= x.numel() * 2 + 16 + 4 * (x.numel() * 2 // 1024 + 1)   # never worse than stored
    # a host-produced frame (4 MiB blocks) takes the host path
    z = torch.empty_like(x)
    codec.decompress(rt.lz4_compress(x.view(torch.uint8).cpu().numpy()), z)
    assert torch.equal(z.view(torch.int16), x.view(torch.int16))


@pytest.mark.parametrize("n_elems,dtype", [(1, torch.bfloat16), (4097, torch.bfloat16), (3_211_264, torch.bfloat16),
                                           (100_003, torch.float32)])
def test_gpu_zvc_matches_host_codec(ops, n_elems, dtype):
    import importlib
    gz = importlib.import_module(f"{PKG}.codec.gpu_zvc")
    rt = importlib.import_module(f"{PKG}.native").runtime()
    torch.manual_seed(n_elems)
    x = torch.relu(torch.randn(n_elems, device="cuda")).to(dtype)
    esz = x.element_size()
    codec = gz.GpuZVC(n_elems, esz)
    codec.compress(x)
    s = codec.stream_bytes()
    raw = x.view(torch.uint8).cpu().numpy()
    assert s == rt.zvc_compress(raw, esz)                 # byte-identical to the host encoder
    assert rt.zvc_decompress(s) == raw.tobytes()
    y = torch.empty_like(x)
    codec.decompress(s, y)
    torch.cuda.synchronize()
    assert torch.equal(y.view(torch.uint8), x.view(torch.uint8))
    if n_elems > 4096:
        assert len(s) < 0.65 * x.numel() * esz            # ~half zeros removed


@pytest.mark.parametrize("cfg", [None, 3, 4, 20, 22, 23, 28])
@pytest.mark.parametrize("ks", [1, 2, -1])
@pytest.mark.parametrize("shape", [(2, 14, 14, 256, 512, 128, 2), (2, 9, 11, 64, 256, 64, 1)])
def test_conv_dual_output_matches_two_convs(ops, cfg, ks, shape):
    """Sibling 1x1 convs packed along N (runtime/plan.py merge_siblings): columns
    [0, n_split) -> out (no ReLU), the rest -> out2 (ReLU), for plain, split-K and
    stream-K launches, equal to the two convs run separately."""
    conv, _ = ops
    if ks < 0 and (cfg is None or cfg in conv.V1_CFGS):
        pytest.skip("stream-K is a v2-config mode")
    B, H, W, Cin, N0, N1, s = shape
    dev = "cuda"
    torch.manual_seed(4)
    x = torch.randn(B, H, W, Cin, device=dev).to(torch.bfloat16)
    k0 = (torch.randn(1, 1, Cin, N0) / math.sqrt(Cin)).numpy()
    k1 = (torch.randn(1, 1, Cin, N1) / math.sqrt(Cin)).numpy()
    b0, b1 = (torch.randn(N0) * 0.1).numpy(), (torch.randn(N1) * 0.1).numpy()
    pads = ((0, 0), (0, 0))
    pc0, pc1 = conv.pack_conv(k0, b0, s, pads, dev), conv.pack_conv(k1, b1, s, pads, dev)
    pcd = conv.pack_conv(np.concatenate([k0, k1], -1), np.concatenate([b0, b1]), s, pads, dev)
    pcd.n_split = N0
    OH, OW = pc0.out_hw(H, W)
    M = B * OH * OW
    r0 = torch.empty(B, OH, OW, N0, device=dev, dtype=torch.bfloat16)
    r1 = torch.empty(B, OH, OW, N1, device=dev, dtype=torch.bfloat16)
    conv.conv_forward(x, pc0, r0, relu=False)
    conv.conv_forward(x, pc1, r1, relu=True)
    o0, o1 = torch.full_like(r0, 7.0), torch.full_like(r1, 7.0)
    ws = ctr = None
    if cfg is not None:
        need = conv.workspace_elems(M, N0 + N1, pcd.Kpad, cfg, ks)
        ws = torch.empty(max(need, 1), device=dev, dtype=torch.float32)
        if ks < 0:
            ctr = torch.zeros(conv.sk_plan(M, N0 + N1, pcd.Kpad, cfg, -ks)[0], device=dev, dtype=torch.int32)
    if cfg is not None and ks > 1 and pcd.Kpad // 64 // ks < 1:
        pytest.skip("K too short to split")
    conv.conv_forward(x, pcd, o0, relu=False, cfg=cfg, ksplit=ks, workspace=ws, counters=ctr, out2=o1, relu2=True)
    torch.cuda.synchronize()
    for got, want in ((o0, r0), (o1, r1)):
        err = (got.float() - want.float()).abs().max().item()
        assert err <= 2e-2 * (want.float().abs().max().item() + 1e-6) + 1e-2, err
    assert (o1.float() >= 0).all()
