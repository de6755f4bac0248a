#!/bin/bash
# Round-2 GPU pass zz: pipeline checker (2 gloo ranks on one GPU) with and without the fused pairs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r2zz
P="python -u -m adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.parallel.check --gpus 2 --backend gloo --part-at conv3_block1_1_conv --batch 4"
bash tools/gpu_steps.sh \
  "200|r2zz/check_pairs|$P" \
  "200|r2zz/check_nopairs|ADAPT_FUSED_PAIR=0 $P" \
  "200|r2zz/check_pairs_b1|python -u -m adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.parallel.check --gpus 2 --backend gloo --part-at conv4_block1_1_conv --batch 4"
