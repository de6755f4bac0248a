#!/bin/bash
# Round-2 GPU pass zm: fused 1x1 pair kernel -- numerics, model numerics, whole-model A/B per tile size, bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r2zm
bash tools/gpu_steps.sh \
  "240|r2zm/tests|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_pair_gpu.py tests/test_model_gpu.py" \
  "200|r2zm/ab_default|python -u tools/ab_cfg.py --env-a ADAPT_FUSED_PAIR=0 --env-b ADAPT_FUSED_PAIR=1 --rounds 21 --json gpurun_out/r2zm/ab_default.json" \
  "200|r2zm/ab_s3only|python -u tools/ab_cfg.py --env-a ADAPT_FUSED_PAIR=0 --env-b ADAPT_PAIR_BM=256:0 --rounds 21 --json gpurun_out/r2zm/ab_s3only.json" \
  "200|r2zm/ab_s3_32|python -u tools/ab_cfg.py --env-a ADAPT_FUSED_PAIR=0 --env-b ADAPT_PAIR_BM=256:0,128:32 --rounds 21 --json gpurun_out/r2zm/ab_s3_32.json" \
  "200|r2zm/ab_s4only|python -u tools/ab_cfg.py --env-a ADAPT_FUSED_PAIR=0 --env-b ADAPT_PAIR_BM=128:0 --rounds 21 --json gpurun_out/r2zm/ab_s4only.json" \
  "200|r2zm/ab_s4_32|python -u tools/ab_cfg.py --env-a ADAPT_FUSED_PAIR=0 --env-b ADAPT_PAIR_BM=128:0,256:32 --rounds 21 --json gpurun_out/r2zm/ab_s4_32.json" \
  "200|r2zm/bench|python -u bench.py --steps 300 --warmup 30"
