#!/usr/bin/env python3
"""Activation-compression measurements on real ResNet-50 bs=32 frontier
tensors: GPU LZ4 (side stream) vs host LZ4 vs host zfp+lz4 (the reference's
codec), compression ratio and throughput, and how much a side-stream encode
slows the overlapped next forward.  --precision fp32 (default: the shipped
DEFER precision) measures fp32 frontiers; the host LZ4 of byte-shuffled fp32
(4 byte planes per 16 KiB block) is reported beside the plain host LZ4.

    python tools/codec_bench.py [--batch 32] [--precision fp32|bf16] [--json out.json]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd import codec as C  # noqa: E402
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.codec.gpu_lz4 import GpuLZ4  # noqa: E402
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.codec.gpu_zfp import GpuZFP  # noqa: E402
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.codec.gpu_zvc import GpuZVC  # noqa: E402
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.resnet import build_resnet, init_weights  # noqa: E402
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.native import runtime  # noqa: E402
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.runtime.executor import SliceExecutor  # noqa: E402

# the single-tensor cut frontiers, plus the two tensors of BASELINE config 2's multi-tensor cut
# (part_at=['conv3_block1_1_conv']: conv3_block1_1_conv and conv2_block3_out cross it)
CUTS = ["pool1_pool", "conv2_block3_out", "conv3_block4_out", "conv4_block6_out", "conv5_block3_out",
        "conv3_block1_1_conv"]


def gpu_time(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--precision", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    prec = a.precision
    esz = 4 if prec == "fp32" else 2
    g = build_resnet("resnet50")
    w = init_weights(g, 0)
    ex = SliceExecutor(g, w, a.batch, outputs=CUTS + [g.output], precision=prec)
    x = torch.randn(a.batch, 224, 224, 3, device="cuda")
    outs = ex.run({g.input: x})
    torch.cuda.synchronize()
    rt = runtime()
    rows = []
    full = SliceExecutor(g, w, a.batch, precision=prec)
    full.capture()
    t_fwd = gpu_time(lambda: full.forward(0), reps=20)
    for name in CUTS:
        t = outs[name].contiguous()
        nbytes = t.numel() * esz
        codec = GpuLZ4(nbytes)
        codec.compress(t)
        frame = codec.frame_bytes()
        t_gpu = gpu_time(lambda: (codec.compress(t), codec.done.synchronize()), reps=10)
        host = t.view(torch.uint8).cpu().numpy().reshape(-1) if prec == "fp32" else \
            t.view(torch.int16).cpu().numpy().view(np.uint16)
        t0 = time.perf_counter()
        hf = rt.lz4_compress(host)
        t_host = time.perf_counter() - t0
        shuf_ratio = None
        if prec == "fp32" and host.size % (4 * 4096) == 0:
            planes = host.reshape(-1, 4096, 4).transpose(0, 2, 1).copy().reshape(-1)   # 16 KiB blocks
            shuf_ratio = nbytes / len(rt.lz4_compress(planes))
        f32 = t.float().cpu().numpy()
        t0 = time.perf_counter()
        zf = C.encode(f32, "zfp+lz4")
        t_zfp = time.perf_counter() - t0
        # the reference's zfp (reversible) on the GPU side stream, fp32 activations
        t32 = t.float().contiguous()
        gz = GpuZFP(tuple(t32.shape))
        gz.compress(t32)
        zc_bytes = gz.container()
        exact = zc_bytes == rt.zfp_compress(f32.reshape(C.zfp_shape(f32.shape)), 8, 1)   # the shared fold
        t_gzfp = gpu_time(lambda: (gz.compress(t32), gz.done.synchronize()), reps=5)
        back = torch.empty_like(t32)
        t_gzfp_dec = gpu_time(lambda: gz.decompress(zc_bytes, back), reps=3)
        if not torch.equal(back, t32):
            raise RuntimeError(f"GPU zfp round trip mismatch on {name}")
        t0 = time.perf_counter()
        rt.zfp_compress(f32.reshape(C.zfp_shape(f32.shape)), 8)
        t_hzfp = time.perf_counter() - t0
        zc = GpuZVC(t.numel(), esz)
        zc.compress(t)
        zs = zc.stream_bytes()
        t_zvc = gpu_time(lambda: (zc.compress(t), zc.done.synchronize()), reps=20)
        out_t = torch.empty_like(t)
        t_zvc_dec = gpu_time(lambda: zc.decompress(zs, out_t), reps=5)
        # overlap: forward on the compute stream while the side stream encodes
        def both():
            zc.compress(t)
            full.forward(0)
        t_both = gpu_time(both, reps=10)
        rows.append({"tensor": name, "shape": list(t.shape), "mbytes": nbytes / 1e6,
                     "gpu_zvc_ratio": nbytes / len(zs), "gpu_zvc_GBps": nbytes / t_zvc / 1e9,
                     "gpu_zvc_dec_GBps_incl_h2d": nbytes / t_zvc_dec / 1e9,
                     "gpu_lz4_ratio": nbytes / len(frame), "gpu_lz4_GBps": nbytes / t_gpu / 1e9,
                     "host_lz4_ratio": nbytes / len(hf), "host_lz4_GBps": nbytes / t_host / 1e9,
                     "host_lz4_byteshuffled_ratio": shuf_ratio, "precision": prec,
                     "zeros": float((t == 0).float().mean()),
                     "zfp_lz4_ratio_vs_frontier": nbytes / len(zf), "zfp_lz4_GBps": f32.nbytes / t_zfp / 1e9,
                     "gpu_zfp_ratio_fp32": f32.nbytes / len(zc_bytes), "gpu_zfp_GBps": f32.nbytes / t_gzfp / 1e9,
                     "gpu_zfp_dec_GBps_incl_h2d": f32.nbytes / t_gzfp_dec / 1e9,
                     "gpu_zfp_bitexact_with_host": bool(exact), "host_zfp_GBps": f32.nbytes / t_hzfp / 1e9,
                     "fwd_ms": t_fwd * 1e3, "fwd_plus_side_encode_ms": t_both * 1e3})
    for r in rows:
        print(f"{r['tensor']:18s} {r['mbytes']:7.1f} MB | GPU zvc x{r['gpu_zvc_ratio']:.2f} {r['gpu_zvc_GBps']:7.1f} GB/s"
              f" | GPU lz4 x{r['gpu_lz4_ratio']:.2f} {r['gpu_lz4_GBps']:7.1f} GB/s"
              f" | host lz4 x{r['host_lz4_ratio']:.2f} {r['host_lz4_GBps']:5.2f} GB/s"
              f" | shuffled host lz4 x{(r['host_lz4_byteshuffled_ratio'] or 0):.2f}"
              f" | zfp+lz4 x{r['zfp_lz4_ratio_vs_frontier']:.2f} {r['zfp_lz4_GBps']:5.2f} GB/s"
              f" | GPU zfp(fp32) x{r['gpu_zfp_ratio_fp32']:.2f} {r['gpu_zfp_GBps']:6.1f} GB/s"
              f" (host {r['host_zfp_GBps']:.2f}, exact={r['gpu_zfp_bitexact_with_host']})"
              f" | fwd {r['fwd_ms']:.3f} ms, fwd||encode {r['fwd_plus_side_encode_ms']:.3f} ms")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
