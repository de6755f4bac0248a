#!/usr/bin/env python3
"""After re-tuning other model families, put back ResNet-50's own entries (the
headline model's tuning wins wherever the families share a conv shape with it).
    python tools/merge_r50_keys.py <table-before.json>"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.resnet import init_weights  # noqa: E402
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.zoo import build_model  # noqa: E402
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.runtime import executor as E  # noqa: E402

before = json.load(open(sys.argv[1]))
g = build_model("resnet50")
keys = set()
for bs in (32, 16, 1):
    ex = E.SliceExecutor(g, init_weights(g, 0), bs, precision="bf16")
    for i in ex.cfg:
        B, H, W, C, OH, OW, pc = ex._conv_geom(i)
        keys.add(E.conv_key(B, H, W, C, pc))
now = json.loads(E.TUNING_FILE.read_text())
restored = [k for k in keys if k in before and now.get(k) != before[k]]
for k in keys:
    if k in before:
        now[k] = before[k]
E.TUNING_FILE.write_text(json.dumps(now, indent=1, sort_keys=True))
print(f"restored {len(restored)} ResNet-50 entries: {restored}")
