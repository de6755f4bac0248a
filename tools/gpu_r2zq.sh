#!/bin/bash
# Round-2 GPU pass zq: fused 1x1 pair -- isolated timing and two PMC passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r2zq
bash tools/gpu_steps.sh \
  "120|r2zq/bench|python -u tools/pair_bench.py" \
  "300|r2zq/pmc|bash tools/pmc_run.sh gpurun_out/r2zq/pmc tools/pair_bench.py --bm 112 --only-pair"
