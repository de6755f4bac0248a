#!/bin/bash
# Round-2 GPU pass zg: threaded ingest copy -- 1-stage serve with fp32 and uint8 pixels.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r2zg
M="python -u -m adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd"
bash tools/gpu_steps.sh \
  "300|r2zg/serve1_f32|$M serve --model resnet50 --batch 32 --device cuda:0 --requests 1500 --spawn 1" \
  "300|r2zg/serve1_u8|$M serve --model resnet50 --batch 32 --device cuda:0 --requests 1500 --uint8 --preprocess caffe --spawn 1" \
  "300|r2zg/serve1_f32_b|$M serve --model resnet50 --batch 32 --device cuda:0 --requests 1500 --spawn 1" \
  "300|r2zg/local_bs1|$M local-infer --model resnet50 --batch 1 --requests 200 --device cuda:0"
