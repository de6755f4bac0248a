#!/bin/bash
# Round-2 GPU pass q: fp32 conv kernel (32-wide K tiles, residual prefetch, tap-uniform gather, 6 tiles):
# numerics, autotune, profile, bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r2q
T=adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd/tuning/gfx950_conv.json
bash tools/gpu_steps.sh \
  "400|r2q/pytest_fp32|python -u -m pytest tests/test_fp32_gpu.py -x -q --timeout 120 --timeout-method thread" \
  "900|r2q/tune_fp32|python -u tools/profile_r50.py --batch 32 --dtype fp32 --tune --json gpurun_out/r2q/r50_fp32_tuned.json && cp $T gpurun_out/r2q/" \
  "240|r2q/bench_fp32|python -u bench.py --dtype fp32 --steps 20 --warmup 5"
