#!/bin/bash
# Round-2 GPU pass d: ingest tests, serving throughput (uint8 + shm ingest vs fp32 inline), fault bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r2d
M="python -u -m adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd"
bash tools/gpu_steps.sh \
  "600|r2d/pytest_ingest|python -u -m pytest tests/test_ingest_gpu.py tests/test_defer_gpu.py -x -v --timeout 300 --timeout-method thread" \
  "300|r2d/serve1_u8_shm|$M serve --model resnet50 --batch 32 --spawn 1 --device cuda:0 --requests 600 --uint8 --preprocess caffe" \
  "300|r2d/serve1_f32_shm|$M serve --model resnet50 --batch 32 --spawn 1 --device cuda:0 --requests 400" \
  "300|r2d/serve1_f32_tcp|$M serve --model resnet50 --batch 32 --spawn 1 --device cuda:0 --requests 300 --ingest tcp" \
  "400|r2d/serve2_u8_shm|$M serve --model resnet50 --batch 32 --spawn 2 --device cuda:0 --requests 400 --uint8 --part-at conv3_block1_1_conv" \
  "420|r2d/fault8|python -u tools/fault_bench.py --workers 8 --device cuda:0 --model resnet50 --image 224 --batch 32 --duration 20 --kill-at 8 --inflight 8 --json gpurun_out/r2d/fault_r50_8w.json"
