"""GPU wire codecs of the collective data plane (codec/wire.py over
csrc/kernels/lz4_gpu.hip and zvc_gpu.hip): encode on a side stream, decode
straight from the device buffer, bit-exact, and interoperable with the host
codecs.  Runs on the MI355X box only."""
import importlib

import pytest
import torch

PKG = "adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd"

pytestmark = pytest.mark.gpu


def _inputs(n):
    g = torch.Generator(device="cuda").manual_seed(n)
    relu = torch.relu(torch.randn(n, device="cuda", generator=g)).to(torch.bfloat16)
    zeros = torch.zeros(n, device="cuda", dtype=torch.bfloat16)
    # short-period repeats: overlapping LZ4 matches (offset < 64) and long runs
    period = torch.arange(n, device="cuda").remainder(7).to(torch.bfloat16)
    mixed = relu.clone()
    mixed[: n // 2] = 0
    rnd = torch.randint(-32768, 32767, (n,), device="cuda", dtype=torch.int16, generator=g).view(torch.bfloat16)
    return {"relu": relu, "zeros": zeros, "period7": period, "half_zero": mixed, "random_bits": rnd}


@pytest.fixture(scope="module")
def mods():
    importlib.import_module(f"{PKG}.ops._lib").kernels()
    return importlib.import_module(f"{PKG}.codec.wire"), importlib.import_module(f"{PKG}.native").runtime()


@pytest.mark.parametrize("kind", ["lz4", "zvc"])
@pytest.mark.parametrize("n", [1, 1000, 1025, 65_536, 1_605_632])
def test_wire_roundtrip_bit_exact(mods, kind, n):
    wire, rt = mods
    for name, x in _inputs(n).items():
        enc = wire.WireCodec(kind, x)
        dec = wire.WireCodec(kind, x)
        enc.encode(x)
        nb = enc.nbytes()
        dec.wire[:nb].copy_(enc.wire[:nb])                 # what the link moves
        y = torch.full_like(x, 3.0)
        dec.decode(nb, y)
        torch.cuda.synchronize()
        dec.check()
        assert torch.equal(y.view(torch.int16), x.view(torch.int16)), (kind, name, n)
        raw = x.view(torch.uint8).cpu().numpy().tobytes()
        body = enc.frame().tobytes()
        if kind == "lz4":
            assert rt.lz4_decompress(body) == raw, name      # standard LZ4 frame
        else:
            assert body == rt.zvc_compress(x.view(torch.uint8).cpu().numpy(), 2), name   # byte-identical to host
        if n >= 65_536 and kind == "lz4" and name in ("zeros", "period7"):
            assert nb < len(raw) / 20, (kind, name, nb)      # long runs / repeats compress hard
        if n >= 65_536 and kind == "zvc" and name == "zeros":
            assert nb < len(raw) / 10, (kind, name, nb)      # masks only
        if n >= 65_536 and name == "random_bits" and kind == "lz4":
            assert nb <= len(raw) + enc.head + 64 + 4 * (len(raw) // 2048 + 1)   # stored raw, never expands


def test_gpu_lz4_decoder_reads_host_frames_with_gpu_blocks(mods):
    """Host-parsed offsets path (codec/gpu_lz4.GpuLZ4.decompress) on the v2 encoder's frames."""
    gl = importlib.import_module(f"{PKG}.codec.gpu_lz4")
    for name, x in _inputs(300_001).items():
        c = gl.GpuLZ4(x.numel() * 2 + 4096)
        c.compress(x)
        frame = c.frame_bytes()
        y = torch.empty_like(x)
        c.decompress(frame, y)
        torch.cuda.synchronize()
        assert torch.equal(y.view(torch.int16), x.view(torch.int16)), name


@pytest.mark.parametrize("shape", [(13,), (6, 10), (3, 9, 10), (4, 7, 7, 64), (2, 3, 5, 6, 8)])
def test_gpu_zfp_bitexact_with_host_and_lossless(shape):
    """GPU zfp (csrc/kernels/zfp_gpu.hip) writes the host codec's v2 container
    byte for byte (chunk_blocks=1) and decodes losslessly, specials included."""
    import numpy as np
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.codec.gpu_zfp import GpuZFP
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.native import runtime
    rng = np.random.default_rng(len(shape))
    a = rng.standard_normal(shape).astype(np.float32).reshape(-1)
    a[:5] = [np.inf, -np.inf, -0.0, 1e-42, np.nan]
    a[5:50] = np.maximum(a[5:50], 0)
    a = a.reshape(shape)
    t = torch.from_numpy(a).cuda()
    z = GpuZFP(shape)
    z.compress(t)
    c = z.container()
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.codec import zfp_shape
    host = runtime().zfp_compress(a.reshape(zfp_shape(shape)), 4, 1)      # the fold both ends derive
    assert c == host
    out = torch.empty_like(t)
    z.decompress(c, out)
    torch.cuda.synchronize()
    assert out.cpu().numpy().tobytes() == a.tobytes()


def test_gpu_zfp_wire_codec_round_trip_and_host_interop(mods):
    wire, rt = mods
    t = torch.randn(8, 14, 14, 32, device="cuda").relu()
    enc, dec = wire.WireCodec("zfp", t), wire.WireCodec("zfp", t)
    enc.encode(t)
    n = enc.nbytes()
    dec.wire[:n].copy_(enc.wire[:n])
    out = torch.empty_like(t)
    dec.decode(n, out)
    torch.cuda.synchronize()
    assert torch.equal(out, t)
    host = wire.WireCodec("zfp", t.cpu())
    host.wire[:n].copy_(enc.wire[:n].cpu())
    o2 = torch.empty_like(t.cpu())
    host.decode(n, o2)
    assert torch.equal(o2, t.cpu())
