#!/bin/bash
# Round-2 GPU pass zz8: rr3 with two K groups of waves (config 72) -- numerics, isolated timing, whole-model A/B vs 71.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r2zz8
S3=32x28x28x128,3x3s1p1111
bash tools/gpu_steps.sh \
  "240|r2zz8/tests|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_rr3_gpu.py" \
  "120|r2zz8/bench|python -u tools/conv_bench.py --shape 32,28,28,128,128,3,1,1,0 --shape 8,28,28,128,128,3,1,1,0 --only 71,72,22 --ks 1" \
  "200|r2zz8/ab|python -u tools/ab_cfg.py --set $S3@72@1 --rounds 21 --json gpurun_out/r2zz8/ab_72.json"
