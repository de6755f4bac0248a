#!/bin/bash
# Round-2 GPU pass zw: in-graph sweep of many-workgroup tiles for the single-round 1x1 convs of stages 4-5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r2zw
cp adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd/tuning/gfx950_conv.json gpurun_out/r2zw/table_before.json
bash tools/gpu_steps.sh \
  "600|r2zw/sweep|python -u tools/ingraph_sweep.py --adopt --rounds 5 --json gpurun_out/r2zw/sweep.json \
     --key 32x14x14x256,1x1s1p0000,1024 --cands 3@1,10@1,16@1,24@1,34@1,31@1,21@1,8@1,17@1,25@1,32@1 \
     --key 32x7x7x512,1x1s1p0000,2048 --cands 3@1,10@1,16@1,24@1,34@1,31@1,21@1,23@1,54@1 \
     --key 32x7x7x2048,1x1s1p0000,512 --cands 3@1,10@1,16@1,34@1,21@1,22@1,24@2,23@2 \
     --key 32x14x14x1024,1x1s1p0000,256 --cands 3@1,10@1,16@1,24@1,34@1,21@1,31@1 \
     --key 32x28x28x128,1x1s1p0000,512 --cands 10@1,16@1,24@1,34@1,21@1,37@1,39@1 \
     && cp adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd/tuning/gfx950_conv.json gpurun_out/r2zw/" \
  "150|r2zw/bench|python -u bench.py --steps 300 --warmup 30"
