#!/bin/bash
# Round-2 GPU pass zz5: final tree (pairs + register-resident stage-3 3x3) -- GPU suite, smoke, benches, trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r2zz5
bash tools/gpu_steps.sh \
  "400|r2zz5/pytest_gpu|python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread" \
  "150|r2zz5/smoke|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "150|r2zz5/bench|python -u bench.py --steps 300 --warmup 30" \
  "150|r2zz5/bench_default|python -u bench.py" \
  "150|r2zz5/bench_r152|python -u bench.py --model resnet152 --steps 100 --warmup 20" \
  "150|r2zz5/bench_fp32|python -u bench.py --dtype fp32 --steps 100 --warmup 10" \
  "200|r2zz5/prof|rocprofv3 --kernel-trace --stats -d gpurun_out/r2zz5/prof -o run -- python3 bench.py --steps 50 --warmup 10"
