#!/bin/bash
# Round-2 GPU pass y: store-policy A/B (plain vs write-through per kernel site), interleaved in one process.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r2y
mkdir -p $O
steps=("240|r2y/r50|python -u tools/store_policy_ab.py --model resnet50 --policies 0,1,4,5,7,13,29,125,127 --json $O/r50.json")
for m in mobilenet_v2 densenet121 efficientnetb0 inception_v3; do
  steps+=("240|r2y/$m|python -u tools/store_policy_ab.py --model $m --policies 0,5,21,37,53,117,127 --rounds 9 --json $O/$m.json")
done
steps+=("240|r2y/r50_fp32|python -u tools/store_policy_ab.py --model resnet50 --dtype fp32 --policies 0,5,127 --rounds 7 --json $O/r50_fp32.json")
bash tools/gpu_steps.sh "${steps[@]}"
