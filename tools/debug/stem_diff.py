"""Debug: stem v2 vs v1 mismatch map (pool rows / columns / channels)."""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops import conv as C  # noqa: E402

torch.manual_seed(1)
B = 2
x = torch.randn(B, 224, 224, 3, device="cuda") * 40
k = (torch.randn(7, 7, 3, 64) / math.sqrt(147) / 40).numpy()
b = (torch.randn(64) * 0.1).numpy()
ps = C.pack_stem(k, b, ((3, 3), (3, 3)), "cuda")
o2 = torch.empty(B, 56, 56, 64, device="cuda", dtype=torch.bfloat16)
o1 = torch.empty_like(o2)
C.stem_forward(x, ps, o2, pool=True)
os.environ["ADAPT_STEM_V1"] = "1"
C.stem_forward(x, ps, o1, pool=True)
torch.cuda.synchronize()
d = (o1.float() - o2.float()).abs()
print("max diff", d.max().item(), "frac bad", (d > 1e-3).float().mean().item())
bad_rows = (d > 1e-3).any(-1).any(-1).any(0).nonzero().flatten().tolist()
print("bad pool rows", bad_rows)
bad_cols = (d > 1e-3).any(-1).any(1).any(0).nonzero().flatten().tolist()
print("bad pool cols", bad_cols[:60])
bad_ch = (d > 1e-3).any(0).any(0).any(0).nonzero().flatten().tolist()
print("bad channels", bad_ch)
print("v1 row0", o1[0, 0, :4, :4].float().tolist())
print("v2 row0", o2[0, 0, :4, :4].float().tolist())
