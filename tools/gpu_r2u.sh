#!/bin/bash
# Round-2 GPU pass u: the other model families, bf16 and fp32, bs=32 (per-step profile + graph replay).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r2u
mkdir -p $O
steps=()
for m in mobilenet_v2 densenet121 vgg16 efficientnetb0 inception_v3 resnet152; do
  steps+=("240|r2u/${m}_bf16|python -u tools/profile_r50.py --model $m --batch 32 --json $O/${m}_bf16.json")
  steps+=("240|r2u/${m}_fp32|python -u tools/profile_r50.py --model $m --batch 32 --dtype fp32 --json $O/${m}_fp32.json")
done
bash tools/gpu_steps.sh "${steps[@]}"
