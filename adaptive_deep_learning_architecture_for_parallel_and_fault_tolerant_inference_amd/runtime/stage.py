"""Stage compute wrapper used by `Node`: one slice, one device, fixed batch.

GPU (``cuda:N``): `SliceExecutor` (our HIP kernels, hipGraph-captured).
CPU: `CpuExecutor` (runtime/cpu_executor.py: the compiled fp32 plan on the
native OpenMP ops of csrc/cpu) — the CPU path of BASELINE.json config 1 and
of the CPU-only integration tests.  PyTorch's own ops are not on either path.

Host-side arrays in/out are numpy; bfloat16 tensors travel as uint16 bit
patterns with a flag (numpy has no bf16).  Device-resident paths (RCCL links)
use `device_inputs()` / `device_outputs()` directly and never touch the host.

`submit()` is the pipelined GPU path of a TCP stage: H2D of micro-batch t
(straight from a page-locked shared-memory slot when the dispatcher is on
the same host), the ingest kernel (uint8 images -> preprocessed fp32), the
graph replay and the D2H of the outputs are all enqueued on the stream and
only an event comes back, so the host receives t+1 and sends t-1 while t
computes (two buffer sets alternate).  Uploads from page-locked memory run on
a copy stream of their own, so the H2D of t+1 overlaps the replay of t: set
j's upload waits for the event that retired set j's previous replay, and the
replay waits for the upload's event.  Each buffer set also has a compute
stream of its own (ingest, replay and output copies of set j run on stream j),
so micro-batches t and t+1 overlap on the GPU the way `bench.py --streams 2`
does (ADAPT_STAGE_STREAMS=1 keeps one stream).  Results still leave in order:
the send thread waits for the events in FIFO order.  `run_host()` is the
synchronous form.
"""
from __future__ import annotations

import warnings
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..graph.ir import Graph


def to_torch(a: np.ndarray, is_bf16: bool, device) -> torch.Tensor:
    """Host array -> tensor on `device`.  Read-only arrays (zero-copy views of a
    received frame) are only read: straight into a device copy, or copied once
    on the host when the tensor stays on the CPU."""
    a = np.ascontiguousarray(a)
    if not a.flags.writeable:
        if torch.device(device).type == "cpu":
            a = a.copy()
        else:
            with warnings.catch_warnings():
                warnings.simplefilter("ignore", UserWarning)
                t = torch.from_numpy(a)
            if is_bf16:
                t = t.view(torch.bfloat16)
            return t.to(device, non_blocking=False)
    t = torch.from_numpy(a)
    if is_bf16:
        t = t.view(torch.bfloat16)
    return t.to(device, non_blocking=False)


def _readonly_tensor(a: np.ndarray) -> torch.Tensor:
    """A CPU tensor over a read-only array (a received frame or a shm slot), no copy."""
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", UserWarning)
        return torch.from_numpy(np.ascontiguousarray(a))


def to_numpy(t: torch.Tensor) -> Tuple[np.ndarray, bool]:
    t = t.detach()
    if t.dtype == torch.bfloat16:
        return t.cpu().contiguous().view(torch.int16).numpy().view(np.uint16), True
    return t.cpu().contiguous().numpy(), False


class StageCompute:
    def __init__(self, g: Graph, weights: Dict[str, np.ndarray], batch: int, device: str = "cpu",
                 outputs: Optional[Sequence[str]] = None, graph_capture: bool = True, num_sets: int = 1,
                 host_ring: int = 8, capture_mode: str = "global", precision: str = "fp32",
                 preprocess: str = "none", streams: int = 2):
        self.g = g
        self.preprocess = preprocess          # uint8 image inputs: Keras preprocess_input mode (ops/eltwise.py)
        self._u8: Dict[Tuple[str, int], torch.Tensor] = {}
        self._tick = 0
        self.batch = batch
        self.device = torch.device(device)
        self.inputs = list(g.input_names)
        self.outputs = list(outputs or g.output_names)
        self.gpu = self.device.type == "cuda"
        self.host_ring = max(2, int(host_ring))
        self._pinned: List[Dict[str, torch.Tensor]] = []
        self._pin_next = 0
        self._h2d = None                      # copy stream for page-locked uploads (created on first use)
        self._set_free: List[Optional[torch.cuda.Event]] = []   # set j's last replay has retired
        self._uploads: List[torch.cuda.Event] = []              # this micro-batch's side-stream uploads
        self._cstreams: List = []                                # per-set compute streams (created on first use)
        self.multi_stream = False
        if self.gpu:
            import os
            from .executor import SliceExecutor
            # concurrent sets: set j replays on its own stream (submit), so the sets must not
            # share the executor's internal arena and scratch
            self.multi_stream = (num_sets > 1 and int(streams) > 1
                                 and os.environ.get("ADAPT_STAGE_STREAMS", "") != "1")
            self.ex = SliceExecutor(g, weights, batch, device=self.device, outputs=self.outputs, num_sets=num_sets,
                                    precision=precision, private_sets=self.multi_stream)
            if graph_capture:
                self.ex.capture(mode=capture_mode)
        else:
            from .cpu_executor import CpuExecutor
            self.ex = CpuExecutor(g, weights, outputs=self.outputs)

    def _pad(self, t: torch.Tensor, count: int) -> torch.Tensor:
        if t.shape[0] == self.batch:
            return t
        pad = torch.zeros((self.batch - t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        return torch.cat([t, pad])

    def _upload(self, dst: torch.Tensor, src, rows: int, j: int) -> None:
        """dst[:rows] <- src (page-locked host memory, or a device link slot), zero-fill dst[rows:]: on the copy
        stream, after set j's previous replay; the replay of this set waits for it."""
        cur = torch.cuda.current_stream(self.device)
        if self._h2d is None:
            from ..ops._lib import private_stream
            self._h2d = private_stream(self.device)
        if len(self._set_free) <= j:
            self._set_free.extend([None] * (j + 1 - len(self._set_free)))
        with torch.cuda.stream(self._h2d):
            if self._set_free[j] is not None:
                self._h2d.wait_event(self._set_free[j])
            else:
                self._h2d.wait_stream(cur)          # first use: after whatever set the buffer up
            if isinstance(src, torch.Tensor):
                dst[:rows].copy_(src, non_blocking=True)
            else:                                   # a device link slot (DevArray): device to device
                from ..ops._lib import kernels, stream_handle
                kernels().memcpy_async(int(dst.data_ptr()), src.ptr, src.nbytes, stream_handle(self._h2d))
            if rows < dst.shape[0]:
                dst[rows:].zero_()
            ev = torch.cuda.Event()
            ev.record(self._h2d)
        self._uploads.append(ev)

    def _feed(self, name: str, a: np.ndarray, is_bf16: bool, count: int, j: int) -> None:
        """Host array -> input buffer `name` of set j (page-locked sources through the
        copy stream, `_upload`; the rest on the current stream)."""
        from ..ops import eltwise as E
        from ..transport.shm import DevArray
        dst = self.ex.input_buf(name, j)
        if isinstance(a, DevArray):
            want = np.dtype(np.uint16) if dst.dtype == torch.bfloat16 else np.dtype(np.float32)
            if (a.dtype != want or is_bf16 != (dst.dtype == torch.bfloat16)
                    or tuple(a.shape[1:]) != tuple(dst.shape[1:]) or a.shape[0] > dst.shape[0]):
                raise ValueError(f"device link tensor {a.shape} {a.dtype} does not match input {name} "
                                 f"{tuple(dst.shape)} {dst.dtype}")
            self._upload(dst, a, a.shape[0], j)
            return
        if a.dtype == np.uint8 and dst.dtype == torch.float32 and tuple(a.shape[1:]) == tuple(dst.shape[1:]):
            key = (name, j)
            u8 = self._u8.get(key)
            if u8 is None:
                u8 = self._u8[key] = torch.zeros(tuple(dst.shape), dtype=torch.uint8, device=self.device)
            src = _readonly_tensor(a)
            if src.is_pinned():             # a registered shm slot; it outlives the request
                self._upload(u8, src, a.shape[0], j)
                self._wait_uploads()
            else:
                u8[: a.shape[0]].copy_(src)
                if a.shape[0] < dst.shape[0]:
                    u8[a.shape[0]:].zero_()
            E.ingest_u8(u8, dst, self.preprocess)
            return
        want = np.uint16 if dst.dtype == torch.bfloat16 else (np.float32 if dst.dtype == torch.float32 else None)
        if (want is not None and a.dtype == want and is_bf16 == (dst.dtype == torch.bfloat16)
                and tuple(a.shape[1:]) == tuple(dst.shape[1:]) and a.shape[0] <= dst.shape[0]):
            # same layout: one copy straight into the input buffer, async when `a` is
            # page-locked (a registered shared-memory link slot, released at the event)
            src = _readonly_tensor(a)
            if is_bf16:
                src = src.view(torch.bfloat16)
            if src.is_pinned():             # a registered shared-memory link slot, released at the event
                self._upload(dst, src, a.shape[0], j)
                return
            dst[: a.shape[0]].copy_(src)
            if a.shape[0] < dst.shape[0]:
                dst[a.shape[0]:].zero_()
            return
        t = to_torch(a, is_bf16, self.device)
        if t.dtype != dst.dtype:
            t = t.to(dst.dtype)
        if t.shape[-1] != dst.shape[-1]:          # channel padding (e.g. 3 -> 8)
            t = torch.nn.functional.pad(t, (0, dst.shape[-1] - t.shape[-1]))
        t = self._pad(t, count)
        dst.copy_(t)

    def submit(self, arrays: Sequence[np.ndarray], bf16_flags: Sequence[bool], count: int, out_slots=None):
        """Enqueue one micro-batch (GPU): returns (event, [(array, bf16)]) whose host
        arrays are valid once the event has completed.  `out_slots(shape, dtype)`
        -> (host tensor, handle): copy the first `count` rows of each output into
        that tensor (a same-host link slot) and return the handle instead."""
        if len(arrays) != len(self.inputs):
            raise ValueError(f"stage expects {len(self.inputs)} inputs, got {len(arrays)}")
        j = self._tick % self.ex.num_sets
        self._tick += 1
        if self.multi_stream:
            if not self._cstreams:
                from ..ops._lib import private_stream
                cur = torch.cuda.current_stream(self.device)
                self._cstreams = [private_stream(self.device) for _ in range(self.ex.num_sets)]
                for cs in self._cstreams:
                    cs.wait_stream(cur)             # after whatever set the buffers up
            with torch.cuda.stream(self._cstreams[j]):
                return self._submit(j, arrays, bf16_flags, count, out_slots)
        return self._submit(j, arrays, bf16_flags, count, out_slots)

    def _submit(self, j: int, arrays, bf16_flags, count: int, out_slots):
        for name, a, b in zip(self.inputs, arrays, bf16_flags):
            self._feed(name, a, b, count, j)
        self._wait_uploads()
        outs = self.ex.forward(j)
        if self._h2d is not None:
            # set j's buffers may be overwritten once this replay has retired
            free = torch.cuda.Event()
            free.record(torch.cuda.current_stream(self.device))
            if len(self._set_free) <= j:
                self._set_free.extend([None] * (j + 1 - len(self._set_free)))
            self._set_free[j] = free
        if out_slots is not None:
            res = []
            for o in self.outputs:
                src = outs[o][:count]
                host, handle = out_slots(tuple(src.shape), src.dtype)
                host.copy_(src, non_blocking=True)
                res.append((handle, src.dtype == torch.bfloat16))
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
            return ev, res
        if not self._pinned:
            for _ in range(self.host_ring):
                self._pinned.append({o: torch.empty(tuple(outs[o].shape), dtype=outs[o].dtype, pin_memory=True)
                                     for o in self.outputs})
        slot = self._pinned[self._pin_next]
        self._pin_next = (self._pin_next + 1) % self.host_ring
        for o in self.outputs:
            slot[o].copy_(outs[o], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        res = []
        for o in self.outputs:
            h = slot[o][:count]
            if h.dtype == torch.bfloat16:
                res.append((h.view(torch.int16).numpy().view(np.uint16), True))
            else:
                res.append((h.numpy(), False))
        return ev, res

    def _wait_uploads(self) -> None:
        cur = torch.cuda.current_stream(self.device)
        for ev in self._uploads:
            cur.wait_event(ev)
        self._uploads.clear()

    def run_host(self, arrays: Sequence[np.ndarray], bf16_flags: Sequence[bool], count: int
                 ) -> Tuple[List[np.ndarray], List[bool]]:
        if len(arrays) != len(self.inputs):
            raise ValueError(f"stage expects {len(self.inputs)} inputs, got {len(arrays)}")
        if self.gpu:
            ev, res = self.submit(arrays, bf16_flags, count)
            ev.synchronize()
            return [r[0] for r in res], [r[1] for r in res]
        feed = {}
        for name, a, b in zip(self.inputs, arrays, bf16_flags):
            if a.dtype == np.uint8 and self.preprocess != "none":
                from ..ops.eltwise import preprocess_ref
                a = preprocess_ref(a, self.preprocess)
            a = np.asarray(a)
            if b:                                   # bf16 bit patterns from a GPU stage -> fp32
                a = (np.ascontiguousarray(a).view(np.uint16).astype(np.uint32) << 16).view(np.float32)
            a = np.asarray(a, np.float32)
            true_c = self.g.layers[name].out_shape[-1] if self.g.layers[name].out_shape else None
            if true_c and a.ndim == 4 and a.shape[-1] != true_c:
                a = a[..., :true_c]
            feed[name] = np.ascontiguousarray(a)
        outs = self.ex.run(feed, outputs=self.outputs)
        return [np.asarray(outs[o][:count], np.float32) for o in self.outputs], [False] * len(self.outputs)
