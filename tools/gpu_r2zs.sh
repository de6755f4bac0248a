#!/bin/bash
# Round-2 GPU pass zs: in-graph candidate sweep for the heaviest conv groups (stream-K stage 5, K-group configs elsewhere).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r2zs
bash tools/gpu_steps.sh \
  "600|r2zs/sweep|python -u tools/ingraph_sweep.py --adopt --json gpurun_out/r2zs/sweep.json \
     --key 32x7x7x512,3x3s1p1111 --cands 68@-1,62@-1,23@-1,66@-1,68@-2,62@2,64@4,66@2 \
     --key 32x28x28x128,1x1s1p0000,512 --cands 62@1,63@1,65@1,66@1,67@1,68@1,30@1 \
     --key 32x14x14x256,1x1s1p0000,1024 --cands 62@1,63@1,65@1,69@1,70@1,64@1,66@1 \
     --key 32x28x28x128,3x3s1p1111 --cands 66@1,62@1,63@1,65@1,22@1 \
     --key 32x14x14x1024,1x1s1p0000,256 --cands 62@1,66@1,68@1,67@1 \
     --key 32x28x28x512,1x1s1p0000,128 --cands 62@1,66@1,68@1,67@1 \
     && cp adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd/tuning/gfx950_conv.json gpurun_out/r2zs/" \
  "150|r2zs/bench|python -u bench.py --steps 300 --warmup 30"
