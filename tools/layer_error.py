#!/usr/bin/env python3
"""Per-layer numerics of the HIP runtime against the fp32 oracle for any
model family: the executor is asked to emit every checked tensor (the plan
then keeps those fusion boundaries), and each is compared to the reference.

    python tools/layer_error.py --model mobilenet_v2 --batch 4 [--every 1]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.resnet import init_weights  # noqa: E402
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.zoo import build_model  # noqa: E402
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops.reference import ReferenceExecutor  # noqa: E402
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.runtime.executor import SliceExecutor  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="mobilenet_v2")
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--size", type=int, default=224)
    ap.add_argument("--ops", default="relu,add,bn,concat,gap,dense,maxpool,avgpool",
                    help="layer ops whose outputs are checked")
    a = ap.parse_args()
    g = build_model(a.model, input_shape=(a.size, a.size, 3))
    w = init_weights(g, 0)
    ops = set(a.ops.split(","))
    names = [n for n in g.order if g.layers[n].op in ops]
    x = torch.randn(a.batch, a.size, a.size, 3, generator=torch.Generator().manual_seed(0)).cuda()
    ref = ReferenceExecutor(g, w, device="cuda").run({g.input: x}, outputs=names)
    ex = SliceExecutor(g, w, batch=a.batch, outputs=names, precision="bf16")
    got = ex.run({g.input: x})
    torch.cuda.synchronize()
    for n in names:
        r = ref[n].float().reshape(a.batch, -1)
        o = got[n].float().reshape(a.batch, -1)[:, :r.shape[1]] if got[n].dim() == 2 else \
            got[n].float()[..., :ref[n].shape[-1]].reshape(a.batch, -1)
        rel = ((o - r).norm() / (r.norm() + 1e-12)).item()
        print(f"{n:36s} {g.layers[n].op:8s} rms {r.pow(2).mean().sqrt().item():9.4f}  rel {rel:.4f}", flush=True)


if __name__ == "__main__":
    main()
