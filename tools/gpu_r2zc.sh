#!/bin/bash
# Round-2 GPU pass zc: worker kill with device (IPC) stage links, 4 and 8 stages.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r2zc
bash tools/gpu_steps.sh \
  "420|r2zc/fault4|python -u tools/fault_bench.py --workers 4 --device cuda:0 --model resnet50 --image 224 --batch 32 --duration 15 --kill-at 6 --inflight 8 --links dev --json gpurun_out/r2zc/fault_r50_4w_dev.json" \
  "420|r2zc/fault8|python -u tools/fault_bench.py --workers 8 --device cuda:0 --model resnet50 --image 224 --batch 32 --duration 20 --kill-at 8 --inflight 8 --links dev --json gpurun_out/r2zc/fault_r50_8w_dev.json"
