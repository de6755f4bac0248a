"""Compressed pipeline data plane on the GPU (BASELINE config 3 protocol):
two stage processes share the box's one MI355X over the host-staged gloo
rehearsal backend (RCCL refuses two ranks on one device); stage outputs are
encoded by the GPU codecs on a side stream and decoded on the device by the
next stage.  The codecs are lossless and the cut sits on a block output, so
the pipeline's predictions equal the unsliced model's bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

PKG = "adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd"
B = 4
STEPS = 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, codec, port, outdir):
    import importlib
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        resnet = importlib.import_module(f"{PKG}.models.resnet")
        runner = importlib.import_module(f"{PKG}.parallel.runner")
        g = resnet.build_resnet("resnet50")
        w = resnet.init_weights(g, seed=0)
        job = runner.PipelineJob(g, w, world, rank, dev, B, world, ["conv4_block1_out"], host_staged=True, codec=codec,
                                 precision="bf16")
        x = torch.randn((B, 224, 224, 3), generator=torch.Generator(device=dev).manual_seed(5), device=dev)
        job.set_synthetic_input(x)
        job.set_total_steps(STEPS)
        for _ in range(STEPS):
            job.step()
        job.finish()
        torch.cuda.synchronize()
        if rank == 0:
            np.save(os.path.join(outdir, "ratio.npy"), np.array([job.link.ratio]))
        if rank == world - 1:
            got = job.ex.output_buf(job.slice.outputs[0], 0).float().cpu().numpy()
            ex = importlib.import_module(f"{PKG}.runtime.executor").SliceExecutor(g, w, B, device=dev, precision="bf16")
            want = ex(x).float().cpu().numpy()
            np.save(os.path.join(outdir, "got.npy"), got)
            np.save(os.path.join(outdir, "want.npy"), want)
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("codec", ["lz4", "zvc"])
def test_compressed_pipeline_gpu_matches_unsliced(tmp_path, codec):
    mp.start_processes(_worker, args=(2, codec, _free_port(), str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    got, want = np.load(tmp_path / "got.npy"), np.load(tmp_path / "want.npy")
    assert got.shape == (B, 1000)
    np.testing.assert_array_equal(got, want)
    ratio = float(np.load(tmp_path / "ratio.npy")[0])
    assert ratio > (1.0 if codec == "zvc" else 0.95)
