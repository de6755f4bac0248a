"""Stage compute wrapper used by `Node`: one slice, one device, fixed batch.

GPU (``cuda:N``): `SliceExecutor` (our HIP kernels, hipGraph-captured).
CPU: the fp32 oracle (`ops.reference`) — the "CPU plumbing path" of
BASELINE.json config 1 and of the CPU-only integration tests.

Host-side arrays in/out are numpy; bfloat16 tensors travel as uint16 bit
patterns with a flag (numpy has no bf16).  Device-resident paths (RCCL links)
use `device_inputs()` / `device_outputs()` directly and never touch the host.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..graph.ir import Graph


def to_torch(a: np.ndarray, is_bf16: bool, device) -> torch.Tensor:
    t = torch.from_numpy(np.ascontiguousarray(a))
    if is_bf16:
        t = t.view(torch.bfloat16)
    return t.to(device, non_blocking=False)


def to_numpy(t: torch.Tensor) -> Tuple[np.ndarray, bool]:
    t = t.detach()
    if t.dtype == torch.bfloat16:
        return t.cpu().contiguous().view(torch.int16).numpy().view(np.uint16), True
    return t.cpu().contiguous().numpy(), False


class StageCompute:
    def __init__(self, g: Graph, weights: Dict[str, np.ndarray], batch: int, device: str = "cpu",
                 outputs: Optional[Sequence[str]] = None, graph_capture: bool = True, num_sets: int = 1):
        self.g = g
        self.batch = batch
        self.device = torch.device(device)
        self.inputs = list(g.input_names)
        self.outputs = list(outputs or g.output_names)
        self.gpu = self.device.type == "cuda"
        if self.gpu:
            from .executor import SliceExecutor
            self.ex = SliceExecutor(g, weights, batch, device=self.device, outputs=self.outputs, num_sets=num_sets)
            if graph_capture:
                self.ex.capture()
        else:
            from ..ops.reference import ReferenceExecutor
            self.ex = ReferenceExecutor(g, weights, device="cpu")

    def _pad(self, t: torch.Tensor, count: int) -> torch.Tensor:
        if t.shape[0] == self.batch:
            return t
        pad = torch.zeros((self.batch - t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        return torch.cat([t, pad])

    def run_host(self, arrays: Sequence[np.ndarray], bf16_flags: Sequence[bool], count: int
                 ) -> Tuple[List[np.ndarray], List[bool]]:
        if len(arrays) != len(self.inputs):
            raise ValueError(f"stage expects {len(self.inputs)} inputs, got {len(arrays)}")
        if self.gpu:
            for name, a, b in zip(self.inputs, arrays, bf16_flags):
                dst = self.ex.input_buf(name)
                t = to_torch(a, b, self.device)
                if t.dtype != dst.dtype:
                    t = t.to(dst.dtype)
                if t.shape[-1] != dst.shape[-1]:          # channel padding (e.g. 3 -> 8)
                    t = torch.nn.functional.pad(t, (0, dst.shape[-1] - t.shape[-1]))
                t = self._pad(t, count)
                dst.copy_(t)
            outs = self.ex.forward(0)
            res = [to_numpy(outs[o][:count]) for o in self.outputs]
            torch.cuda.current_stream(self.device).synchronize()
        else:
            feed = {}
            for name, a, b in zip(self.inputs, arrays, bf16_flags):
                t = to_torch(a, b, "cpu").float()
                true_c = self.g.layers[name].out_shape[-1] if self.g.layers[name].out_shape else None
                if true_c and t.dim() == 4 and t.shape[-1] != true_c:
                    t = t[..., :true_c]
                feed[name] = t
            outs = self.ex.run(feed, outputs=self.outputs)
            res = [(outs[o][:count].float().numpy(), False) for o in self.outputs]
        return [r[0] for r in res], [r[1] for r in res]
