#!/bin/bash
# Round-2 GPU pass b: multi-GPU gated tests (rehearsal on 1 GPU), DEFER GPU
# tests, and the 8-stage / 4-stage SIGKILL fault benches (1-GPU TCP rehearsal).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r2b
bash tools/gpu_steps.sh \
  "600|r2b/pytest_mgpu|python -u -m pytest tests/test_multigpu.py tests/test_defer_gpu.py -x -v --timeout 300 --timeout-method thread" \
  "420|r2b/fault8|python -u tools/fault_bench.py --workers 8 --device cuda:0 --model resnet50 --image 224 --batch 32 --duration 20 --kill-at 8 --inflight 8 --json gpurun_out/r2b/fault_r50_8w.json" \
  "420|r2b/fault4|python -u tools/fault_bench.py --workers 4 --device cuda:0 --model resnet50 --image 224 --batch 32 --duration 20 --kill-at 8 --inflight 8 --json gpurun_out/r2b/fault_r50_4w.json"
