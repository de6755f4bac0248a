#!/bin/bash
# Round-2 GPU pass zt: re-tune the other bf16 model families with the K-group configs
# (6 in-graph candidates per problem), keep ResNet-50's entries, re-profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r2zt
mkdir -p $O
T=adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd/tuning/gfx950_conv.json
cp $T $O/table_before.json
export ADAPT_TUNE_REFINE=6 ADAPT_TUNE_VERBOSE=1
steps=()
for m in mobilenet_v2 densenet121 vgg16 efficientnetb0 inception_v3; do
  steps+=("300|r2zt/${m}_tune|python -u tools/profile_r50.py --model $m --batch 32 --tune --json $O/${m}_tuned.json")
done
steps+=("200|r2zt/merge|python -u tools/merge_r50_keys.py $O/table_before.json && cp $T $O/table_after.json")
steps+=("150|r2zt/bench|python -u bench.py --steps 300 --warmup 30")
bash tools/gpu_steps.sh "${steps[@]}"
