#!/bin/bash
# Round-2 GPU pass zz2: full GPU suite + smoke + bench on the committed tree (pairs on, calibrated checker).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r2zz2
bash tools/gpu_steps.sh \
  "400|r2zz2/pytest_gpu|python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread" \
  "150|r2zz2/smoke|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "150|r2zz2/bench|python -u bench.py --steps 300 --warmup 30" \
  "150|r2zz2/bench_default|python -u bench.py"
