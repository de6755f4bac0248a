#!/bin/bash
# Round-2 GPU pass j: re-tune conv tiles with the 32-row configs, profile, bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r2j
T=adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd/tuning/gfx950_conv.json
bash tools/gpu_steps.sh \
  "900|r2j/tune|python -u tools/profile_r50.py --batch 32 --tune --json gpurun_out/r2j/r50_bs32_tuned.json && cp $T gpurun_out/r2j/" \
  "240|r2j/bench|python -u bench.py --steps 50 --warmup 10"
