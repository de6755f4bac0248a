#!/bin/bash
# Round-2 GPU pass zv: serving and fault path on the final tree -- 1/2/4-stage serve, 4- and 8-stage kill.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r2zv
M="python -u -m adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd"
S="serve --model resnet50 --batch 32 --device cuda:0 --requests 1500 --uint8 --preprocess caffe"
bash tools/gpu_steps.sh \
  "300|r2zv/serve1_u8|$M $S --spawn 1" \
  "300|r2zv/serve2_dev|$M $S --spawn 2 --part-at conv3_block1_1_conv" \
  "400|r2zv/serve4_dev|$M $S --spawn 4 --part-at auto:4" \
  "420|r2zv/fault4|python -u tools/fault_bench.py --workers 4 --device cuda:0 --model resnet50 --image 224 --batch 32 --duration 15 --kill-at 6 --inflight 8 --json gpurun_out/r2zv/fault_r50_4w_dev.json" \
  "420|r2zv/fault8|python -u tools/fault_bench.py --workers 8 --device cuda:0 --model resnet50 --image 224 --batch 32 --duration 15 --kill-at 6 --inflight 8 --json gpurun_out/r2zv/fault_r50_8w_dev.json"
