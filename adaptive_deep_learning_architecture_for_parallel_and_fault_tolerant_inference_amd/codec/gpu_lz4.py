"""GPU LZ4 activation codec on a side HIP stream (csrc/kernels/lz4_gpu.hip).

`GpuLZ4(max_bytes, device)` owns its scratch buffers.  `compress(t)` enqueues
the encoder on the codec's own stream after an event recorded on the caller's
(compute) stream, so the encode of micro-batch t overlaps the compute of t+1;
`frame_bytes()` then copies only the compressed bytes to host.  Frames are
standard LZ4 frames (1 KiB independent blocks): any LZ4 decoder reads them;
`decompress()` decodes on the GPU from a host or device frame whose blocks
are at most 1 KiB, and uses the host codec otherwise.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from ..native import runtime
from ..ops._lib import kernels


class GpuLZ4:
    def __init__(self, max_bytes: int, device="cuda"):
        K = kernels()
        self.K = K
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.chunk = K.lz4_gpu_chunk()
        self.max_bytes = int(max_bytes)
        nch = (self.max_bytes + self.chunk - 1) // self.chunk
        self.scratch = torch.empty(max(1, K.lz4_gpu_scratch_bytes(self.max_bytes)), dtype=torch.uint8, device=self.device)
        self.sizes = torch.empty(max(1, nch), dtype=torch.int32, device=self.device)
        self.offs = torch.empty(max(1, nch), dtype=torch.int32, device=self.device)
        self.frame = torch.empty(K.lz4_gpu_max_frame(self.max_bytes), dtype=torch.uint8, device=self.device)
        self.total = torch.zeros(1, dtype=torch.int64, device=self.device)
        self.total_host = torch.zeros(1, dtype=torch.int64, pin_memory=True)
        self.err = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.stream = torch.cuda.Stream(device=self.device)
        self.done = torch.cuda.Event()
        self._n = 0
        self._host: Optional[torch.Tensor] = None     # persistent pinned D2H buffer (frame_view)
        self._stage: Optional[torch.Tensor] = None    # persistent pinned H2D staging (decompress)
        self._dframe: Optional[torch.Tensor] = None
        self._h2d_done: Optional[torch.cuda.Event] = None

    def compress(self, t: torch.Tensor, after: Optional[torch.cuda.Event] = None) -> torch.cuda.Event:
        """Enqueue compression of `t` (any dtype, contiguous) on the side stream."""
        if not t.is_contiguous() or t.device != self.device:
            raise ValueError("GpuLZ4.compress: contiguous tensor on the codec's device required")
        n = t.numel() * t.element_size()
        if n == 0 or n > self.max_bytes:
            raise ValueError(f"GpuLZ4.compress: {n} bytes outside (0, {self.max_bytes}]")
        ev = after
        if ev is None:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
        self.stream.wait_event(ev)
        with torch.cuda.stream(self.stream):
            self.K.lz4_gpu_compress(t.data_ptr(), n, self.scratch.data_ptr(), self.sizes.data_ptr(),
                                    self.offs.data_ptr(), self.frame.data_ptr(), self.total.data_ptr(),
                                    int(self.stream.cuda_stream))
            self.total_host.copy_(self.total, non_blocking=True)
            self.done.record(self.stream)
        t.record_stream(self.stream)
        self._n = n
        return self.done

    def frame_view(self) -> memoryview:
        """Wait for the last compress() and return its LZ4 frame as a view of a
        persistent pinned host buffer (valid until the next frame_view call)."""
        self.done.synchronize()
        tot = int(self.total_host.item())
        if self._host is None:
            self._host = torch.empty(self.frame.numel(), dtype=torch.uint8, pin_memory=True)
        with torch.cuda.stream(self.stream):
            self._host[:tot].copy_(self.frame[:tot], non_blocking=True)
        self.stream.synchronize()
        return memoryview(self._host.numpy())[:tot]

    def frame_bytes(self) -> bytes:
        """Wait for the last compress() and return its LZ4 frame."""
        return bytes(self.frame_view())

    def _to_device(self, raw) -> torch.Tensor:
        nb = len(raw)
        if self._stage is None or self._stage.numel() < nb:
            cap = max(nb, self.frame.numel())
            self._stage = torch.empty(cap, dtype=torch.uint8, pin_memory=True)
            self._dframe = torch.empty(cap, dtype=torch.uint8, device=self.device)
        if self._h2d_done is not None:
            self._h2d_done.synchronize()
        self._stage.numpy()[:nb] = np.frombuffer(raw, dtype=np.uint8)
        self._dframe[:nb].copy_(self._stage[:nb], non_blocking=True)
        self._h2d_done = torch.cuda.Event()
        self._h2d_done.record(torch.cuda.current_stream(self.device))
        return self._dframe

    def decompress(self, frame, out: torch.Tensor) -> torch.Tensor:
        """Decode an LZ4 frame (bytes, or a uint8 device tensor) into `out` (on the
        current stream).  GPU path for 1 KiB-block frames; host codec otherwise."""
        n = out.numel() * out.element_size()
        raw = frame if isinstance(frame, (bytes, bytearray, memoryview)) else frame.cpu().numpy().tobytes()
        content, bmax, indep, offs, words = runtime().lz4_frame_blocks(raw)
        if content not in (0, n):
            raise ValueError(f"frame holds {content} bytes, destination {n}")
        if not indep or len(offs) != (n + self.chunk - 1) // self.chunk or \
                any(((w & 0x7FFFFFFF) > self.chunk + self.chunk // 255 + 16) for w in words[:1]):
            data = np.frombuffer(runtime().lz4_decompress(raw), dtype=np.uint8)
            out.view(torch.uint8).reshape(-1).copy_(torch.from_numpy(data.copy()))
            return out
        dev_frame = self._to_device(raw) if not isinstance(frame, torch.Tensor) else frame
        d_offs = torch.from_numpy(offs.astype(np.int32)).to(self.device)
        d_words = torch.from_numpy(words.astype(np.int64).astype(np.uint32).view(np.int32)).to(self.device)
        self.err.zero_()
        self.K.lz4_gpu_decompress(dev_frame.data_ptr(), d_offs.data_ptr(), d_words.data_ptr(), len(offs),
                                  out.data_ptr(), n, self.err.data_ptr(), int(torch.cuda.current_stream(self.device).cuda_stream))
        if int(self.err.item()) != 0:
            raise RuntimeError(f"GPU LZ4 decode error flags {int(self.err.item())}")
        return out
