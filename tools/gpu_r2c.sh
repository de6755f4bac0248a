#!/bin/bash
# Round-2 GPU pass c: fp32 path tests + fp32/bf16 bench, 8-stage fault bench with heartbeats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r2c
bash tools/gpu_steps.sh \
  "600|r2c/pytest_fp32|python -u -m pytest tests/test_fp32_gpu.py tests/test_multigpu.py -x -v --timeout 300 --timeout-method thread" \
  "300|r2c/bench_fp32|python -u bench.py --dtype fp32 --steps 20 --warmup 5" \
  "300|r2c/bench_bf16|python -u bench.py --steps 50 --warmup 10" \
  "420|r2c/fault8|python -u tools/fault_bench.py --workers 8 --device cuda:0 --model resnet50 --image 224 --batch 32 --duration 20 --kill-at 8 --inflight 8 --json gpurun_out/r2c/fault_r50_8w.json"
