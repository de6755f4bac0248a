#!/bin/bash
# Round-2 GPU pass zx: persistent pipelined pair kernel v4 -- numerics, isolated timing, whole-model A/B, trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r2zx
bash tools/gpu_steps.sh \
  "240|r2zx/tests|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_pair_gpu.py" \
  "120|r2zx/bench|python -u tools/pair_bench.py" \
  "200|r2zx/ab|python -u tools/ab_cfg.py --env-a 'ADAPT_FUSED_PAIR=0' --env-b 'ADAPT_FUSED_PAIR=1' --rounds 21 --json gpurun_out/r2zx/ab.json" \
  "200|r2zx/ab2|python -u tools/ab_cfg.py --env-a 'ADAPT_FUSED_PAIR=0' --env-b 'ADAPT_FUSED_PAIR=1' --rounds 21 --json gpurun_out/r2zx/ab2.json"
