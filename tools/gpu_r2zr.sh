#!/bin/bash
# Round-2 GPU pass zr: full GPU suite, smoke, headline bench, kernel trace of the committed tree.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r2zr
bash tools/gpu_steps.sh \
  "400|r2zr/pytest_gpu|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "150|r2zr/smoke|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "150|r2zr/bench|python -u bench.py --steps 300 --warmup 30" \
  "150|r2zr/bench_fp32|python -u bench.py --dtype fp32 --steps 100 --warmup 10" \
  "200|r2zr/prof|rocprofv3 --kernel-trace --stats -d gpurun_out/r2zr/prof -o run -- python3 bench.py --steps 50 --warmup 10"
