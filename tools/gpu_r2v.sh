#!/bin/bash
# Round-2 GPU pass v: fp32 sliced GAP (tests + EfficientNetB0 / MobileNetV2 / DenseNet121 fp32 re-profile).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r2v
mkdir -p $O
steps=("300|r2v/fp32_tests|python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fp32_gpu.py tests/test_zoo_gpu.py")
for m in efficientnetb0 mobilenet_v2 densenet121 inception_v3; do
  steps+=("240|r2v/${m}_fp32|python -u tools/profile_r50.py --model $m --batch 32 --dtype fp32 --json $O/${m}_fp32.json")
done
bash tools/gpu_steps.sh "${steps[@]}"
