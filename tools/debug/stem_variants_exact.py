"""Bitwise comparison of the fp32 stem variants 2 / 5 / 6 (bs 32, 224x224): count and location of differing outputs."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops import conv as C  # noqa: E402

rng = np.random.default_rng(0)
x = torch.from_numpy(rng.standard_normal((32, 224, 224, 3)).astype(np.float32)).cuda()
kern = (rng.standard_normal((7, 7, 3, 64)) / np.sqrt(147)).astype(np.float32)
ps = C.pack_stem_f32(kern, (0.1 * rng.standard_normal(64)).astype(np.float32), ((3, 3), (3, 3)), "cuda")
outs = {}
for v in (2, 5, 6):
    o = torch.full((32, 56, 56, 64), float("nan"), device="cuda")
    C.stem_f32_forward(x, ps, o, variant=v)
    outs[v] = o.cpu().numpy()
for v in (5, 6):
    ne = outs[v] != outs[2]
    print(v, "differing:", int(ne.sum()), "max abs", float(np.abs(outs[v] - outs[2]).max()))
    if ne.any():
        idx = np.argwhere(ne)
        print("  rows", sorted(set(idx[:, 1].tolist()))[:20], "cols", sorted(set(idx[:, 2].tolist()))[:20],
              "chans", sorted(set(idx[:, 3].tolist()))[:20], "imgs", sorted(set(idx[:, 0].tolist()))[:10])
        for b, r, c, ch in idx[:5]:
            print("   ", (b, r, c, ch), outs[2][b, r, c, ch], outs[v][b, r, c, ch])
