#!/bin/bash
# Round-2 GPU pass o: same-host shared-memory stage links: GPU DEFER tests, 2- and 4-stage serving throughput.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r2o
M="python -u -m adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd"
bash tools/gpu_steps.sh \
  "600|r2o/pytest_defer|python -u -m pytest tests/test_defer_gpu.py -x -v --timeout 300 --timeout-method thread" \
  "300|r2o/serve2_u8_links|$M serve --model resnet50 --batch 32 --spawn 2 --device cuda:0 --requests 600 --uint8 --preprocess caffe --part-at conv3_block1_1_conv" \
  "300|r2o/serve2_u8_tcp|$M serve --model resnet50 --batch 32 --spawn 2 --device cuda:0 --requests 300 --uint8 --preprocess caffe --part-at conv3_block1_1_conv --links tcp" \
  "400|r2o/serve4_u8_links|$M serve --model resnet50 --batch 32 --spawn 4 --device cuda:0 --requests 600 --uint8 --preprocess caffe --part-at auto:4"
