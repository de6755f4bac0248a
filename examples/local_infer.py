#!/usr/bin/env python3
"""The reference's single-device baseline (`test/local_infer.py:1-29`):
`model.predict(x)` repeated, req/s.  Here `Model.predict` runs the slice
executor (our HIP kernels, one hipGraph) on a GPU, or the fp32 oracle on CPU.

    python examples/local_infer.py [--device cuda] [--batch 1] [--requests 10]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.model import resnet  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default=None)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--requests", type=int, default=10)
    ap.add_argument("--model", default="resnet50")
    a = ap.parse_args()
    model = resnet(a.model, seed=0)
    x = np.random.default_rng(0).standard_normal((a.batch, 224, 224, 3)).astype(np.float32)
    model.predict(x, device=a.device)               # build + capture (the reference's first call traces)
    start = time.time()
    for _ in range(a.requests):
        res = model.predict(x, device=a.device)
    run = time.time() - start
    print(res.shape)
    print(f"{a.requests} results in {run} seconds")
    print(f"Throughput: {a.requests / run} req/s")


if __name__ == "__main__":
    main()
