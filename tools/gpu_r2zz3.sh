#!/bin/bash
# Round-2 GPU pass zz3: register-resident-filter 3x3 conv (config 71) -- numerics, isolated timing, whole-model A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r2zz3
S3=32x28x28x128,3x3s1p1111
bash tools/gpu_steps.sh \
  "240|r2zz3/tests|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_rr3_gpu.py" \
  "120|r2zz3/bench|python -u tools/conv_bench.py --shape 32,28,28,128,128,3,1,1,0 --only 71,20,65,22 --ks 1" \
  "200|r2zz3/ab|python -u tools/ab_cfg.py --set $S3@71@1 --rounds 21 --json gpurun_out/r2zz3/ab.json" \
  "200|r2zz3/ab_r152|python -u tools/ab_cfg.py --model resnet152 --set $S3@71@1 --rounds 11 --json gpurun_out/r2zz3/ab_r152.json"
