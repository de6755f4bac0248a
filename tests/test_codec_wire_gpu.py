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
