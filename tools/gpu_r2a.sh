#!/bin/bash
# Round-2 first GPU pass: GPU tests, smoke, 1-GPU bench, kernel-trace stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "900|pytest_gpu|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "240|smoke|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "240|bench1|python -u bench.py --steps 50 --warmup 10" \
  "300|rocprof|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r2a -o run -- python3 bench.py --steps 20 --warmup 5"
