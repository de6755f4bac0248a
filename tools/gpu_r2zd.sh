#!/bin/bash
# Round-2 GPU pass zd: blocking event wait in the stage send loop -- serve 1/2-stage.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r2zd
M="python -u -m adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd"
S="serve --model resnet50 --batch 32 --device cuda:0 --requests 1000 --uint8 --preprocess caffe"
bash tools/gpu_steps.sh \
  "300|r2zd/serve1_u8|$M $S --spawn 1" \
  "300|r2zd/serve2_dev|$M $S --spawn 2 --part-at conv3_block1_1_conv" \
  "300|r2zd/serve1_u8_b|$M $S --spawn 1" \
  "600|r2zd/tests|python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_defer_gpu.py tests/test_ingest_gpu.py"
