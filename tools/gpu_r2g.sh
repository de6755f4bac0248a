#!/bin/bash
# Round-2 GPU pass g: fused bottleneck v2 (disjoint weight fragments per wave, hoisted loads).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r2g
bash tools/gpu_steps.sh \
  "300|r2g/pytest_bn|python -u -m pytest tests/test_bottleneck_gpu.py -x -q --timeout 300 --timeout-method thread" \
  "300|r2g/prof|python -u tools/profile_r50.py --batch 32 --json gpurun_out/r2g/r50_bs32_steps.json" \
  "240|r2g/bench|python -u bench.py --steps 50 --warmup 10"
