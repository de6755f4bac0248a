#!/bin/bash
# Round-2 GPU pass zp: fused 1x1 pair v3 (one round of 112-px tiles, early loads) -- numerics, A/B, trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r2zp
bash tools/gpu_steps.sh \
  "240|r2zp/tests|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_pair_gpu.py" \
  "200|r2zp/ab_112|python -u tools/ab_cfg.py --env-a 'ADAPT_FUSED_PAIR=0' --env-b 'ADAPT_FUSED_PAIR=1' --rounds 21 --json gpurun_out/r2zp/ab_112.json" \
  "200|r2zp/ab_64|python -u tools/ab_cfg.py --env-a 'ADAPT_FUSED_PAIR=0' --env-b 'ADAPT_FUSED_PAIR=1;ADAPT_PAIR_BM=128:64' --rounds 21 --json gpurun_out/r2zp/ab_64.json" \
  "200|r2zp/prof|ADAPT_FUSED_PAIR=1 rocprofv3 --kernel-trace --stats -d gpurun_out/r2zp/prof -o run -- python3 bench.py --steps 50 --warmup 10"
