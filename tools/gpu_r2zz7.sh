#!/bin/bash
# Round-2 GPU pass zz7: rr3 with the rotation swizzle -- numerics, isolated timing, PMC conflicts, whole-model A/B vs glds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r2zz7
S3=32x28x28x128,3x3s1p1111
bash tools/gpu_steps.sh \
  "240|r2zz7/tests|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_rr3_gpu.py" \
  "120|r2zz7/bench|python -u tools/conv_bench.py --shape 32,28,28,128,128,3,1,1,0 --shape 8,28,28,128,128,3,1,1,0 --only 71,20,22 --ks 1" \
  "240|r2zz7/pmc|bash tools/pmc_run.sh gpurun_out/r2zz7/pmc tools/conv_bench.py --shape 32,28,28,128,128,3,1,1,0 --only 71 --ks 1" \
  "200|r2zz7/ab|python -u tools/ab_cfg.py --set $S3@22@1 --rounds 21 --json gpurun_out/r2zz7/ab_vs_glds.json" \
  "150|r2zz7/bench_r50|python -u bench.py --steps 300 --warmup 30"
