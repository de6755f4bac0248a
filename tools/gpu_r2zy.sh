#!/bin/bash
# Round-2 GPU pass zy: stage-3 1x1 pairs fused by default -- full GPU suite, smoke, bench, R152 bench, trace, serve.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r2zy
M="python -u -m adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd"
bash tools/gpu_steps.sh \
  "400|r2zy/pytest_gpu|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "150|r2zy/smoke|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "150|r2zy/bench|python -u bench.py --steps 300 --warmup 30" \
  "150|r2zy/bench_b|python -u bench.py --steps 300 --warmup 30" \
  "150|r2zy/bench_r152|python -u bench.py --model resnet152 --steps 100 --warmup 20" \
  "200|r2zy/prof|rocprofv3 --kernel-trace --stats -d gpurun_out/r2zy/prof -o run -- python3 bench.py --steps 50 --warmup 10" \
  "300|r2zy/serve1_u8|$M serve --model resnet50 --batch 32 --device cuda:0 --requests 1500 --uint8 --preprocess caffe --spawn 1"
