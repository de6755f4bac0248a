#!/bin/bash
# Round-2 GPU pass e: GPU zfp tests + codec bench, planner calibration + plan check, rocprof of fp32.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r2e
bash tools/gpu_steps.sh \
  "600|r2e/pytest_codec|python -u -m pytest tests/test_codec_wire_gpu.py -x -v --timeout 300 --timeout-method thread" \
  "400|r2e/codec_bench|python -u tools/codec_bench.py --json gpurun_out/r2e/codec_bench.json" \
  "400|r2e/calib|python -u tools/profile_r50.py --batch 32 --calib --json gpurun_out/r2e/r50_bs32_steps.json && cp adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd/tuning/gfx950_layer_costs.json gpurun_out/r2e/" \
  "500|r2e/plan_check|python -u tools/plan_check.py --model resnet50 --batch 32 --stages 2,4,8 --json gpurun_out/r2e/plan_check_calibrated.json" \
  "500|r2e/plan_check_analytic|python -u tools/plan_check.py --model resnet50 --batch 32 --stages 4,8 --analytic --json gpurun_out/r2e/plan_check_analytic.json" \
  "400|r2e/prof_fp32|python -u tools/profile_r50.py --batch 32 --dtype fp32 --json gpurun_out/r2e/r50_fp32_steps.json"
