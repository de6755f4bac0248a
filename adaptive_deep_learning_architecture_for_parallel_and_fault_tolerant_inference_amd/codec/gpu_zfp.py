"""GPU reversible zfp codec on a side HIP stream (csrc/kernels/zfp_gpu.hip).

The reference runs zfp (reversible) + LZ4 on every hop on the CPU
(`src/dispatcher.py:92-98`, `src/node.py:122-125`).  `GpuZFP(shape)` encodes a
float32 device tensor into the host codec's version-2 container with one
block per chunk: the device produces the word-count table + payload, the
header (shape, chunk_blocks = 1) is fixed per shape and prepended on the host.
`runtime().zfp_decompress` reads the result, and bytes match
`runtime().zfp_compress(a, chunk_blocks=1)` exactly; `decompress()` decodes
such a container on the device.
"""
from __future__ import annotations

import struct
from typing import Optional, Sequence

import numpy as np
import torch

from ..ops._lib import kernels


from . import zfp_shape  # noqa: E402  (shared with the host codec: the same folding at both ends)


def header(shape: Sequence[int]) -> bytes:
    zs = zfp_shape(shape)
    h = struct.pack("<IBBBB", 0x50465A41, 2, 0, len(zs), 0)        # "AZFP", version 2, float32
    h += b"".join(struct.pack("<Q", v) for v in zs) + struct.pack("<Q", 1)
    return h


class GpuZFP:
    def __init__(self, shape: Sequence[int], device="cuda"):
        self.K = kernels()
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.shape = tuple(int(v) for v in shape)
        self.zshape = list(zfp_shape(self.shape))
        self.nblocks = int(self.K.zfp_gpu_nblocks(self.zshape))
        maxw = int(self.K.zfp_gpu_maxw(len(self.zshape)))
        self.scratch = torch.empty(self.nblocks * maxw, dtype=torch.int64, device=self.device)
        self.offs = torch.empty(self.nblocks, dtype=torch.int64, device=self.device)
        self.out = torch.empty(self.nblocks * (1 + maxw), dtype=torch.int64, device=self.device)
        self.total = torch.zeros(1, dtype=torch.int64, device=self.device)
        self.total_host = torch.zeros(1, dtype=torch.int64, pin_memory=True)
        self.stream = torch.cuda.Stream(device=self.device)
        self.done = torch.cuda.Event()
        self.hdr = header(self.shape)

    def compress(self, t: torch.Tensor, after: Optional[torch.cuda.Event] = None) -> torch.cuda.Event:
        if t.dtype != torch.float32 or not t.is_contiguous() or tuple(t.shape) != self.shape:
            raise ValueError(f"GpuZFP: contiguous float32 tensor of shape {self.shape} required")
        ev = after
        if ev is None:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
        self.stream.wait_event(ev)
        with torch.cuda.stream(self.stream):
            self.K.zfp_gpu_compress(t.data_ptr(), self.zshape, self.scratch.data_ptr(), self.offs.data_ptr(),
                                    self.out.data_ptr(), self.total.data_ptr(), int(self.stream.cuda_stream))
            self.total_host.copy_(self.total, non_blocking=True)
            self.done.record(self.stream)
        t.record_stream(self.stream)
        return self.done

    def container(self) -> bytes:
        """Wait for the last compress() and return the full container bytes."""
        self.done.synchronize()
        nw = self.nblocks + int(self.total_host.item())
        body = self.out[:nw].cpu().numpy().tobytes()
        return self.hdr + struct.pack("<Q", self.nblocks) + body

    def decompress(self, buf, out: torch.Tensor) -> torch.Tensor:
        """Decode a chunk_blocks=1 container (host bytes) into `out` on the current stream."""
        from ..native import runtime
        dt, shape, off, cb = runtime().zfp_info(buf)
        if dt != 0 or cb != 1 or tuple(shape) != tuple(self.zshape):
            raise ValueError(f"GpuZFP.decompress: needs a float32 chunk_blocks=1 container of {self.zshape}")
        if out.dtype != torch.float32 or out.numel() != int(np.prod(self.shape)) or not out.is_contiguous():
            raise ValueError("GpuZFP.decompress: contiguous float32 output of the codec's size required")
        (nchunks,) = struct.unpack_from("<Q", buf, off)
        if nchunks != self.nblocks:
            raise ValueError("GpuZFP.decompress: block count mismatch")
        body = np.frombuffer(memoryview(buf)[off + 8:], dtype=np.int64)
        dev = torch.from_numpy(body.copy()).to(self.device)
        self.K.zfp_gpu_decompress(dev.data_ptr(), self.zshape, self.offs.data_ptr(), self.total.data_ptr(),
                                  out.data_ptr(), int(torch.cuda.current_stream(self.device).cuda_stream))
        return out
