#!/bin/bash
# Round-2 GPU pass zf: stage streams chosen by the dispatcher (2 alone on a GPU, 1 when shared) -- full suite + serve + fault.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r2zf
M="python -u -m adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd"
S="serve --model resnet50 --batch 32 --device cuda:0 --requests 1500 --uint8 --preprocess caffe"
bash tools/gpu_steps.sh \
  "900|r2zf/pytest_gpu|python -u -m pytest -x -q --timeout 180 --timeout-method thread -m gpu tests/" \
  "300|r2zf/serve1_u8|$M $S --spawn 1" \
  "300|r2zf/serve1_f32|$M serve --model resnet50 --batch 32 --device cuda:0 --requests 1000 --spawn 1" \
  "300|r2zf/serve2_dev|$M $S --spawn 2 --part-at conv3_block1_1_conv" \
  "400|r2zf/serve4_dev|$M $S --spawn 4 --part-at auto:4" \
  "420|r2zf/fault4|python -u tools/fault_bench.py --workers 4 --device cuda:0 --model resnet50 --image 224 --batch 32 --duration 15 --kill-at 6 --inflight 8 --json gpurun_out/r2zf/fault_r50_4w_dev.json" \
  "180|r2zf/bench|python -u bench.py --steps 200 --warmup 30"
