#!/bin/bash
# Round-2 GPU pass t: the reference's own protocol (batch 1 req/s): local_infer and 2-stage DEFER with shm links;
# 4-stage kill with shm links.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r2t
M="python -u -m adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd"
bash tools/gpu_steps.sh \
  "200|r2t/local_bs1|$M local-infer --model resnet50 --batch 1 --requests 2000" \
  "300|r2t/serve2_bs1_links|$M serve --model resnet50 --batch 1 --spawn 2 --device cuda:0 --requests 3000 --part-at conv3_block1_1_conv" \
  "300|r2t/serve2_bs1_tcp|$M serve --model resnet50 --batch 1 --spawn 2 --device cuda:0 --requests 2000 --part-at conv3_block1_1_conv --links tcp" \
  "420|r2t/fault4|python -u tools/fault_bench.py --workers 4 --device cuda:0 --model resnet50 --image 224 --batch 32 --duration 15 --kill-at 6 --inflight 8 --json gpurun_out/r2t/fault_r50_4w_links.json"
