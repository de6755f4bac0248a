#!/usr/bin/env python3
"""The reference's distributed demo (`test/test.py:1-52`) on this framework.

Same shape of program: a DEFER dispatcher, a ResNet-50, `part_at` cut list,
an input queue fed `task_size` times and a printer thread that reports
"N results in T seconds" and req/s.  Differences: the workers are started
here (one `Node` per entry of `--devices`, all local; the reference expects
`python -m src.node` on each host), the image is synthetic (no network, no
ImageNet checkpoint: random-init weights), and the cut list may be a
multi-tensor frontier or `auto:K`.

    python examples/test.py                                  # 1 worker, whole model
    python examples/test.py --devices cuda:0,cuda:0 --part-at conv3_block1_1_conv
    python examples/test.py --devices cpu,cpu --model resnet_tiny --task-size 4
"""
import argparse
import os
import queue
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.dispatcher import DEFER  # noqa: E402
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.model import resnet  # noqa: E402
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.node import Node  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--devices", default="cuda:0", help="one local worker per entry")
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--part-at", default="", help="comma-separated cut layers, or auto:K")
    ap.add_argument("--task-size", type=int, default=10)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"],
                    help="worker precision: fp32 = the reference's Keras float32 (`src/node.py:177`)")
    ap.add_argument("--transport", default="auto", choices=["auto", "tcp", "rccl", "gloo"],
                    help="stage -> stage hops; auto = RCCL p2p when every stage has its own GPU")
    a = ap.parse_args()
    devices = [d for d in a.devices.split(",") if d]
    image = (32, 32, 3) if a.model == "resnet_tiny" else (224, 224, 3)
    kw = {"input_shape": image, "classes": 10} if a.model == "resnet_tiny" else {}
    model = resnet(a.model, seed=0, **kw)
    part_at = [c for c in a.part_at.split(",") if c]
    defer = DEFER(membership_port=0, result_port=0, batch=a.batch, min_workers=len(devices), worker_wait=60,
                  ordered=True, precision=a.dtype, transport=a.transport)
    defer.membership_server.start()
    nodes = [Node(membership_port=defer.membership_port, data_port=0, config_port=0, device=d, node_id=f"w{i}")
             for i, d in enumerate(devices)]
    for n in nodes:
        n.run(block=False)
    x = np.random.default_rng(0).standard_normal((a.batch,) + image).astype(np.float32)

    start = time.time()
    done = threading.Event()

    def print_result(q):
        res_count = 0
        while res_count < a.task_size:
            res = q.get()
            res_count += 1
            print(res.shape)
        run = time.time() - start
        print(f"{res_count} results in {run} seconds")
        print(f"Throughput: {res_count / run} req/s")
        done.set()

    input_q, output_q = queue.Queue(10), queue.Queue(10)
    t = threading.Thread(target=defer.run_defer, args=(model, part_at, input_q, output_q), daemon=True)
    b = threading.Thread(target=print_result, args=(output_q,), daemon=True)
    t.start()
    b.start()
    for _ in range(a.task_size):
        input_q.put(x)
    done.wait(600)
    defer.shutdown()
    for n in nodes:
        n.stop()


if __name__ == "__main__":
    main()
