#!/bin/bash
# Round-2 GPU pass ze: per-set compute streams in the serving stage -- A/B one vs two streams, tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r2ze
M="python -u -m adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd"
S="serve --model resnet50 --batch 32 --device cuda:0 --requests 1500 --uint8 --preprocess caffe"
bash tools/gpu_steps.sh \
  "600|r2ze/tests|python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_stage_streams_gpu.py tests/test_defer_gpu.py tests/test_ingest_gpu.py tests/test_pipeline_codec_gpu.py" \
  "300|r2ze/serve1_2streams|$M $S --spawn 1" \
  "300|r2ze/serve1_1stream|ADAPT_STAGE_STREAMS=1 $M $S --spawn 1" \
  "300|r2ze/serve1_f32_2streams|$M serve --model resnet50 --batch 32 --device cuda:0 --requests 1000 --spawn 1" \
  "300|r2ze/serve2_dev_2streams|$M $S --spawn 2 --part-at conv3_block1_1_conv" \
  "300|r2ze/serve1_2streams_b|$M $S --spawn 1"
