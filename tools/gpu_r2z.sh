#!/bin/bash
# Round-2 GPU pass z: serving stage with a separate H2D copy stream -- tests, then 1/2/4-stage serve.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r2z
M="python -u -m adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd"
bash tools/gpu_steps.sh \
  "600|r2z/tests|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ingest_gpu.py tests/test_defer_gpu.py tests/test_pipeline_codec_gpu.py tests/test_model_gpu.py tests/test_codec_wire_gpu.py" \
  "300|r2z/serve1_u8_shm|$M serve --model resnet50 --batch 32 --spawn 1 --device cuda:0 --requests 600 --uint8 --preprocess caffe" \
  "300|r2z/serve1_f32_shm|$M serve --model resnet50 --batch 32 --spawn 1 --device cuda:0 --requests 400" \
  "300|r2z/serve2_u8_links|$M serve --model resnet50 --batch 32 --spawn 2 --device cuda:0 --requests 600 --uint8 --preprocess caffe --part-at conv3_block1_1_conv" \
  "400|r2z/serve4_u8_links|$M serve --model resnet50 --batch 32 --spawn 4 --device cuda:0 --requests 600 --uint8 --preprocess caffe --part-at auto:4"
