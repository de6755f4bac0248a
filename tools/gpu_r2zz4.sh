#!/bin/bash
# Round-2 GPU pass zz4: register-resident-filter 3x3 -- isolated timing (bs 32 / 64) and trace of the switched model.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r2zz4
bash tools/gpu_steps.sh \
  "120|r2zz4/bench|python -u tools/conv_bench.py --shape 32,28,28,128,128,3,1,1,0 --shape 64,28,28,128,128,3,1,1,0 --shape 8,28,28,128,128,3,1,1,0 --only 71,20,22 --ks 1" \
  "240|r2zz4/pmc|bash tools/pmc_run.sh gpurun_out/r2zz4/pmc tools/conv_bench.py --shape 32,28,28,128,128,3,1,1,0 --only 71 --ks 1"
