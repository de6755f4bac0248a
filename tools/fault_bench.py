#!/usr/bin/env python3
"""Fault-injection benchmark (BASELINE.json config 4): CLI of
`<pkg>.parallel.fault_run` (see its docstring for what is measured).

    python tools/fault_bench.py --workers 4 --device cpu --model resnet_tiny
    python tools/fault_bench.py --workers 4 --device cuda:0 --model resnet50 --image 224 --batch 32
    python tools/fault_bench.py --workers 8 --device each --model resnet50 --image 224 --batch 32   # 8 GPUs
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.parallel.fault_run import main  # noqa: E402

if __name__ == "__main__":
    rc = main()
    sys.stdout.flush()
    sys.stderr.flush()
    os._exit(rc)        # daemon I/O threads may sit in native recv(); skip finalization
