#!/bin/bash
# Round-2 GPU pass w: write-through conv output stores (sc1) -- numerics, bench, per-step profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r2w
mkdir -p $O
bash tools/gpu_steps.sh \
  "300|r2w/tests|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bottleneck_gpu.py tests/test_model_gpu.py tests/test_fp32_gpu.py" \
  "180|r2w/bench|python -u bench.py --steps 200 --warmup 30" \
  "180|r2w/bench_b|python -u bench.py --steps 200 --warmup 30" \
  "240|r2w/profile|python -u tools/profile_r50.py --batch 32 --json $O/r50_steps.json" \
  "240|r2w/bs16|python -u tools/profile_r50.py --batch 16 --json $O/r50_bs16_steps.json"
