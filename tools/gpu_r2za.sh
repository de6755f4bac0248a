#!/bin/bash
# Round-2 GPU pass za: private capture streams + copy-stream uploads -- full GPU suite, serve 1/2/4 stages, bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r2za
M="python -u -m adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd"
bash tools/gpu_steps.sh \
  "900|r2za/pytest_gpu|python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/" \
  "300|r2za/serve1_u8_shm|$M serve --model resnet50 --batch 32 --spawn 1 --device cuda:0 --requests 800 --uint8 --preprocess caffe" \
  "300|r2za/serve1_f32_shm|$M serve --model resnet50 --batch 32 --spawn 1 --device cuda:0 --requests 600" \
  "300|r2za/serve2_u8_links|$M serve --model resnet50 --batch 32 --spawn 2 --device cuda:0 --requests 800 --uint8 --preprocess caffe --part-at conv3_block1_1_conv" \
  "400|r2za/serve4_u8_links|$M serve --model resnet50 --batch 32 --spawn 4 --device cuda:0 --requests 800 --uint8 --preprocess caffe --part-at auto:4" \
  "180|r2za/bench|python -u bench.py --steps 200 --warmup 30" \
  "180|r2za/smoke|python -u -c 'import __graft_entry__ as g; g.smoke()'"
