"""Wire codecs for the collective data plane (RCCL / gloo stage links).

The reference compresses every activation it forwards (zfp + LZ4 on the CPU,
`src/dispatcher.py:92-98`, `src/node.py:178`).  On the pipeline's
point-to-point links (parallel/pipeline.py) a frontier tensor instead becomes
ONE contiguous device byte buffer, ``wire``, that travels as a single
``send``/``recv`` and is decoded straight from device memory on the receiver:

* ``lz4``  ``wire = [u32 block sizes (nchunks) | pad to 16 | LZ4 frame]``;
           the frame is a standard LZ4 frame (csrc/kernels/lz4_gpu.hip); the
           size table lets the receiver find the blocks with a device scan
           (`lz4_gpu_decompress_dev`) instead of walking the frame on the host.
* ``zvc``  ``wire = AZVC stream`` (csrc/kernels/zvc_gpu.hip); the stream holds
           its own segment-size table (`zvc_gpu_decompress_dev`).
* ``zfp``  float32 tensors only (the reference's zfp): ``wire = [u64 word count
           per 4^d block | payload words]``, i.e. the host zfp container
           (chunk_blocks = 1) without its fixed header (csrc/kernels/zfp_gpu.hip).

GPU encodes run on a side HIP stream behind an event of the producer stream
(BASELINE config 3: compression overlapped with the next micro-batch's
compute); `nbytes()` waits for that encode only.  CPU tensors use the host
codecs (csrc/runtime) with the same stream formats — the CPU rehearsal of the
same protocol.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from ..native import runtime

KINDS = ("lz4", "zvc", "zfp")


class WireCodec:
    """Encoder/decoder of one frontier tensor (fixed shape and dtype)."""

    def __init__(self, kind: str, like: torch.Tensor, stream: Optional["torch.cuda.Stream"] = None):
        if kind not in KINDS:
            raise ValueError(f"wire codec must be one of {KINDS}, got {kind!r}")
        self.kind = kind
        self.device = like.device
        self.gpu = like.device.type == "cuda"
        self.esz = like.element_size()
        self.numel = like.numel()
        self.n = self.numel * self.esz
        if kind == "zvc" and self.esz not in (2, 4):
            raise ValueError("zvc needs 2- or 4-byte elements")
        if kind == "zfp" and like.dtype != torch.float32:
            raise ValueError("zfp wire codec needs float32 tensors (zfp has no bf16 mode)")
        self.shape = tuple(like.shape)
        if self.n == 0:
            raise ValueError("empty tensor")
        self._nbytes: Optional[int] = None
        self.head = 0
        if not self.gpu:
            # zfp's worst case on small blocks (1-D/2-D tensors) nearly doubles the bytes
            cap = 2 * self.n + 8 * self.numel + 4096 if kind == "zfp" else self.n + self.n // 8 + 4096
            self.wire = torch.empty(cap, dtype=torch.uint8)
            return
        from ..ops._lib import kernels
        K = self.K = kernels()
        self.stream = stream if stream is not None else torch.cuda.Stream(device=self.device)
        dev = self.device
        if kind == "zfp":
            from .gpu_zfp import GpuZFP
            self.zfp = GpuZFP(self.shape, dev)
            self.zfp.stream = self.stream
            self.wire = self.zfp.out.view(torch.uint8)
            self.total_host = self.zfp.total_host
            self.done = self.zfp.done
            self.err = torch.zeros(1, dtype=torch.int32, device=dev)
            return
        if kind == "lz4":
            ch = K.lz4_gpu_chunk()
            self.nidx = (self.n + ch - 1) // ch
            self.head = ((4 * self.nidx + 15) // 16) * 16
            cap = self.head + K.lz4_gpu_max_frame(self.n)
            self.scratch = torch.empty(K.lz4_gpu_scratch_bytes(self.n), dtype=torch.uint8, device=dev)
            self.sizes = None                          # the size table lives at the head of `wire`
        else:
            seg = K.zvc_seg()
            self.nidx = (self.numel + seg - 1) // seg
            self.head = 0
            cap = K.zvc_max_stream(self.numel, self.esz)
            self.scratch = torch.empty(K.zvc_scratch_bytes(self.numel, self.esz), dtype=torch.uint8, device=dev)
            self.sizes = torch.empty(self.nidx, dtype=torch.int32, device=dev)
        self.enc_offs = torch.empty(self.nidx, dtype=torch.int32, device=dev)
        self.dec_offs = torch.empty(self.nidx, dtype=torch.int32, device=dev)
        self.wire = torch.empty(cap, dtype=torch.uint8, device=dev)
        self.err = torch.zeros(1, dtype=torch.int32, device=dev)
        self.total = torch.zeros(1, dtype=torch.int64, device=dev)
        self.total_host = torch.zeros(1, dtype=torch.int64, pin_memory=True)
        self.done = torch.cuda.Event()

    # ------------------------------------------------------------ encode
    def encode(self, t: torch.Tensor, after: Optional["torch.cuda.Event"] = None):
        """Compress `t` into `wire`.  GPU: enqueued on the codec stream behind
        `after` (default: the current stream's tail); returns the done event."""
        if t.numel() != self.numel or t.element_size() != self.esz or not t.is_contiguous() or t.device != self.device:
            raise ValueError("WireCodec.encode: tensor does not match the codec's shape/dtype/device")
        self._nbytes = None
        if not self.gpu:
            raw = t.view(torch.uint8).reshape(-1).numpy()
            rt = runtime()
            if self.kind == "zfp":
                from .gpu_zfp import header, zfp_shape
                b = rt.zfp_compress(t.numpy().reshape(zfp_shape(self.shape)), 4, 1)[len(header(self.shape)) + 8:]
            else:
                b = rt.lz4_compress(raw) if self.kind == "lz4" else rt.zvc_compress(raw, self.esz)
            if len(b) > self.wire.numel():
                raise RuntimeError("host codec output exceeds the wire buffer")
            self.wire[:len(b)].copy_(torch.frombuffer(bytearray(b), dtype=torch.uint8))
            self._nbytes = len(b)
            return None
        ev = after
        if ev is None:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
        if self.kind == "zfp":
            return self.zfp.compress(t, after=ev)
        self.stream.wait_event(ev)
        s = int(self.stream.cuda_stream)
        w = self.wire.data_ptr()
        with torch.cuda.stream(self.stream):
            if self.kind == "lz4":
                self.K.lz4_gpu_compress(t.data_ptr(), self.n, self.scratch.data_ptr(), w, self.enc_offs.data_ptr(),
                                        w + self.head, self.total.data_ptr(), s)
            else:
                self.K.zvc_gpu_compress(t.data_ptr(), self.numel, self.esz, self.scratch.data_ptr(),
                                        self.sizes.data_ptr(), self.enc_offs.data_ptr(), w, self.total.data_ptr(), s)
            self.total_host.copy_(self.total, non_blocking=True)
            self.done.record(self.stream)
        return self.done

    def nbytes(self) -> int:
        """Message length of the last encode (waits for that encode only)."""
        if self._nbytes is None:
            self.done.synchronize()
            if self.kind == "zfp":
                self._nbytes = 8 * (self.zfp.nblocks + int(self.total_host.item()))
            else:
                self._nbytes = self.head + int(self.total_host.item())
        return self._nbytes

    # ------------------------------------------------------------ decode
    def decode(self, nbytes: int, out: torch.Tensor, stream: Optional["torch.cuda.Stream"] = None) -> torch.Tensor:
        """`wire[:nbytes]` (as received) -> `out`.  GPU: on `stream` (default current)."""
        if out.numel() != self.numel or out.element_size() != self.esz or not out.is_contiguous():
            raise ValueError("WireCodec.decode: destination does not match the codec")
        if nbytes <= self.head or nbytes > self.wire.numel():
            raise ValueError(f"WireCodec.decode: bad message length {nbytes}")
        if not self.gpu:
            data = self.wire[:nbytes].numpy().tobytes()
            rt = runtime()
            if self.kind == "zfp":
                import struct
                from .gpu_zfp import header, zfp_shape
                nb = int(np.prod([(v + 3) // 4 for v in zfp_shape(self.shape)]))
                raw = rt.zfp_decompress(header(self.shape) + struct.pack("<Q", nb) + data, 4).tobytes()
            else:
                raw = rt.lz4_decompress(data) if self.kind == "lz4" else rt.zvc_decompress(data)
            if len(raw) != self.n:
                raise RuntimeError(f"decoded {len(raw)} bytes, expected {self.n}")
            out.view(torch.uint8).reshape(-1).copy_(torch.frombuffer(bytearray(raw), dtype=torch.uint8))
            return out
        s = int((stream if stream is not None else torch.cuda.current_stream(self.device)).cuda_stream)
        w = self.wire.data_ptr()
        if self.kind == "zfp":
            z = self.zfp
            self.K.zfp_gpu_decompress(w, z.zshape, z.offs.data_ptr(), z.total.data_ptr(), out.data_ptr(), s)
        elif self.kind == "lz4":
            self.K.lz4_gpu_decompress_dev(w + self.head, w, self.nidx, self.dec_offs.data_ptr(), out.data_ptr(), self.n,
                                          self.err.data_ptr(), s)
        else:
            self.K.zvc_gpu_decompress_dev(w, self.nidx, self.numel, self.esz, out.data_ptr(), self.dec_offs.data_ptr(), s)
        return out

    def check(self) -> None:
        """Raise if any LZ4 block failed to decode since construction (syncs)."""
        if self.gpu and self.kind == "lz4" and int(self.err.item()) != 0:
            raise RuntimeError(f"GPU LZ4 wire decode error flags {int(self.err.item())}")

    def frame(self) -> np.ndarray:
        """Host copy of the last encoded message's codec stream (LZ4 frame /
        AZVC stream without the wire's size table): any standard decoder reads it."""
        n = self.nbytes()
        return self.wire[self.head:n].cpu().numpy()
