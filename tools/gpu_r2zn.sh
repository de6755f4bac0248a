#!/bin/bash
# Round-2 GPU pass zn: fused 1x1 pair v2 (loads issued ahead of the barriers) -- numerics and whole-model A/B per tile size.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r2zn
bash tools/gpu_steps.sh \
  "240|r2zn/tests|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_pair_gpu.py" \
  "200|r2zn/ab_s3_64|python -u tools/ab_cfg.py --env-a 'ADAPT_FUSED_PAIR=0' --env-b 'ADAPT_PAIR_BM=256:0,128:64' --rounds 21" \
  "200|r2zn/ab_s3_32|python -u tools/ab_cfg.py --env-a 'ADAPT_FUSED_PAIR=0' --env-b 'ADAPT_PAIR_BM=256:0,128:32' --rounds 21" \
  "200|r2zn/ab_s4_16|python -u tools/ab_cfg.py --env-a 'ADAPT_FUSED_PAIR=0' --env-b 'ADAPT_PAIR_BM=128:0,256:16' --rounds 21" \
  "200|r2zn/ab_s4_32|python -u tools/ab_cfg.py --env-a 'ADAPT_FUSED_PAIR=0' --env-b 'ADAPT_PAIR_BM=128:0,256:32' --rounds 21"
