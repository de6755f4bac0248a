#!/bin/bash
# Round-2 GPU pass x: write-through stores in every bf16 kernel -- full GPU suite, bench, families.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r2x
mkdir -p $O
steps=("180|r2x/bench|python -u bench.py --steps 200 --warmup 30"
       "240|r2x/profile|python -u tools/profile_r50.py --batch 32 --json $O/r50_steps.json")
for m in mobilenet_v2 densenet121 efficientnetb0 inception_v3 vgg16 resnet152; do
  steps+=("240|r2x/${m}_bf16|python -u tools/profile_r50.py --model $m --batch 32 --json $O/${m}_bf16.json")
done
steps+=("900|r2x/pytest_gpu|python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/")
bash tools/gpu_steps.sh "${steps[@]}"
