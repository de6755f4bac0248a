#!/bin/bash
# Round-2 GPU pass zb: device (IPC) stage links -- tests, then 2/4-stage serve with dev vs host slots.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r2zb
M="python -u -m adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd"
S="serve --model resnet50 --batch 32 --device cuda:0 --requests 800 --uint8 --preprocess caffe"
bash tools/gpu_steps.sh \
  "600|r2zb/tests|python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_defer_gpu.py" \
  "300|r2zb/serve2_dev|$M $S --spawn 2 --part-at conv3_block1_1_conv --links dev" \
  "300|r2zb/serve2_shm|$M $S --spawn 2 --part-at conv3_block1_1_conv --links shm" \
  "400|r2zb/serve4_dev|$M $S --spawn 4 --part-at auto:4 --links dev" \
  "400|r2zb/serve8_dev|$M $S --spawn 8 --part-at auto:8 --links dev"
