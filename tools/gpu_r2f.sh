#!/bin/bash
# Round-2 GPU pass f: fused bottleneck tests, bench, per-layer profile, plan check (compute objective).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r2f
bash tools/gpu_steps.sh \
  "300|r2f/pytest_bn|python -u -m pytest tests/test_bottleneck_gpu.py tests/test_fp32_gpu.py::test_resnet50_bf16_logits_and_top1 tests/test_model_gpu.py -x -v --timeout 300 --timeout-method thread" \
  "240|r2f/bench|python -u bench.py --steps 50 --warmup 10" \
  "300|r2f/prof|python -u tools/profile_r50.py --batch 32 --json gpurun_out/r2f/r50_bs32_steps.json" \
  "500|r2f/plan_check|python -u tools/plan_check.py --model resnet50 --batch 32 --stages 2,4,8 --objective compute --json gpurun_out/r2f/plan_check_compute.json"
