"""GPU zero-value compression (ZVC) on a side HIP stream (csrc/kernels/zvc_gpu.hip).

The activation codec for MI355X stage boundaries: post-ReLU bf16 tensors are
~half exact zeros, which ZVC (64-bit non-zero mask per 64 elements + packed
values) removes at memory speed, where byte-LZ4 finds few 4-byte matches
(tools/codec_bench.py).  Streams are byte-identical between the GPU codec
and the host codec (`_runtime.zvc_*`), so a CPU peer can decode them.

Usage mirrors `GpuLZ4`: `compress(t)` enqueues on the codec's own stream
behind an event of the producer stream (overlapping the next micro-batch's
compute); `stream_bytes()` returns the compressed bytes; `decompress(buf,
out)` decodes host bytes or a device stream on the current stream.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from ..native import runtime
from ..ops._lib import kernels


class GpuZVC:
    def __init__(self, max_elems: int, elem_bytes: int = 2, device="cuda"):
        if elem_bytes not in (2, 4):
            raise ValueError("elem_bytes must be 2 (bf16/fp16) or 4 (fp32)")
        K = kernels()
        self.K = K
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.esz = elem_bytes
        self.max_elems = int(max_elems)
        nseg = (self.max_elems + K.zvc_seg() - 1) // K.zvc_seg()
        self.scratch = torch.empty(K.zvc_scratch_bytes(self.max_elems, self.esz), dtype=torch.uint8, device=self.device)
        self.sizes = torch.empty(max(1, nseg), dtype=torch.int32, device=self.device)
        self.offs = torch.empty(max(1, nseg), dtype=torch.int32, device=self.device)
        self.out = torch.empty(K.zvc_max_stream(self.max_elems, self.esz), dtype=torch.uint8, device=self.device)
        self.total = torch.zeros(1, dtype=torch.int64, device=self.device)
        self.total_host = torch.zeros(1, dtype=torch.int64, pin_memory=True)
        self.stream = torch.cuda.Stream(device=self.device)
        self.done = torch.cuda.Event()
        self._host: Optional[torch.Tensor] = None     # persistent pinned D2H buffer (stream_view)
        self._stage: Optional[torch.Tensor] = None    # persistent pinned H2D staging (decompress)
        self._dstream: Optional[torch.Tensor] = None
        self._h2d_done: Optional[torch.cuda.Event] = None

    def compress(self, t: torch.Tensor, after: Optional[torch.cuda.Event] = None) -> torch.cuda.Event:
        if not t.is_contiguous() or t.device != self.device or t.element_size() != self.esz:
            raise ValueError(f"GpuZVC.compress: contiguous {self.esz}-byte tensor on {self.device} required")
        n = t.numel()
        if n == 0 or n > self.max_elems:
            raise ValueError(f"GpuZVC.compress: {n} elements outside (0, {self.max_elems}]")
        ev = after
        if ev is None:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
        self.stream.wait_event(ev)
        with torch.cuda.stream(self.stream):
            self.K.zvc_gpu_compress(t.data_ptr(), n, self.esz, self.scratch.data_ptr(), self.sizes.data_ptr(),
                                    self.offs.data_ptr(), self.out.data_ptr(), self.total.data_ptr(),
                                    int(self.stream.cuda_stream))
            self.total_host.copy_(self.total, non_blocking=True)
            self.done.record(self.stream)
        t.record_stream(self.stream)
        return self.done

    def stream_view(self) -> memoryview:
        """Wait for the last compress() and return its stream as a view of a
        persistent pinned host buffer (valid until the next stream_view call)."""
        self.done.synchronize()
        tot = int(self.total_host.item())
        if self._host is None:
            self._host = torch.empty(self.out.numel(), dtype=torch.uint8, pin_memory=True)
        with torch.cuda.stream(self.stream):
            self._host[:tot].copy_(self.out[:tot], non_blocking=True)
        self.stream.synchronize()
        return memoryview(self._host.numpy())[:tot]

    def stream_bytes(self) -> bytes:
        return bytes(self.stream_view())

    def _to_device(self, raw) -> torch.Tensor:
        """Host stream -> device copy through a reused pinned staging buffer
        (one host memcpy + an async DMA on the current stream)."""
        nb = len(raw)
        if self._stage is None or self._stage.numel() < nb:
            cap = max(nb, self.out.numel())
            self._stage = torch.empty(cap, dtype=torch.uint8, pin_memory=True)
            self._dstream = torch.empty(cap, dtype=torch.uint8, device=self.device)
        if self._h2d_done is not None:
            self._h2d_done.synchronize()            # the previous DMA has left the staging buffer
        self._stage.numpy()[:nb] = np.frombuffer(raw, dtype=np.uint8)
        self._dstream[:nb].copy_(self._stage[:nb], non_blocking=True)
        self._h2d_done = torch.cuda.Event()
        self._h2d_done.record(torch.cuda.current_stream(self.device))
        return self._dstream

    def decompress(self, buf, out: torch.Tensor) -> torch.Tensor:
        raw = buf if isinstance(buf, (bytes, bytearray, memoryview)) else buf.cpu().numpy().tobytes()
        n, esz, nseg, offs = runtime().zvc_info(raw)
        if n != out.numel() or esz != out.element_size():
            raise ValueError(f"ZVC stream holds {n} x {esz} B, destination {out.numel()} x {out.element_size()} B")
        dev = self._to_device(raw) if not isinstance(buf, torch.Tensor) else buf
        d_offs = torch.from_numpy(offs.astype(np.uint32).view(np.int32)).to(self.device)
        self.K.zvc_gpu_decompress(dev.data_ptr(), d_offs.data_ptr(), int(nseg), int(n), int(esz), out.data_ptr(),
                                  int(torch.cuda.current_stream(self.device).cuda_stream))
        return out
