#!/bin/bash
# Round-2 GPU pass zk: re-tune ResNet-50 bs=32 with the K-group configs (6 in-graph
# candidates per problem), bench with the new table, kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r2zk
export ADAPT_TUNE_REFINE=6 ADAPT_TUNE_VERBOSE=1
bash tools/gpu_steps.sh \
  "900|r2zk/tune|python -u tools/profile_r50.py --batch 32 --tune --json gpurun_out/r2zk/r50_bs32_tuned.json && cp adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd/tuning/gfx950_conv.json gpurun_out/r2zk/" \
  "200|r2zk/bench|python -u bench.py --steps 200 --warmup 30" \
  "200|r2zk/prof|rocprofv3 --kernel-trace --stats -d gpurun_out/r2zk/prof -o run -- python3 bench.py --steps 50 --warmup 10"
