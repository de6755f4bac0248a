#!/bin/bash
# Round-2 GPU pass zh: persistent pointwise conv -- numerics, kernel timing, whole-model A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r2zh
bash tools/gpu_steps.sh \
  "300|r2zh/tests|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_pw_gpu.py" \
  "240|r2zh/bench_s3|python -u tools/pw_bench.py --rounds 15 --json gpurun_out/r2zh/pw_s3.json" \
  "240|r2zh/ab_r50|python -u tools/ab_cfg.py --model resnet50 --key 32x28x28x128,1x1s1p0000,512 --cfg 60 --json gpurun_out/r2zh/ab_r50.json" \
  "240|r2zh/ab_r152|python -u tools/ab_cfg.py --model resnet152 --key 32x28x28x128,1x1s1p0000,512 --cfg 60 --json gpurun_out/r2zh/ab_r152.json"
