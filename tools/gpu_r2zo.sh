#!/bin/bash
# Round-2 GPU pass zo: kernel trace of the bench with the fused 1x1 pairs on (stage 3 BM 64, stage 4 BM 32).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r2zo
export ADAPT_FUSED_PAIR=1 ADAPT_PAIR_BM=128:64,256:32
bash tools/gpu_steps.sh \
  "200|r2zo/prof|rocprofv3 --kernel-trace --stats -d gpurun_out/r2zo/prof -o run -- python3 bench.py --steps 50 --warmup 10"
