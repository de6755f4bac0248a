#!/bin/bash
# Round-2 GPU pass zi: two-K-group LDS-DMA conv configs (62-70) -- numerics, isolated timing, whole-model A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r2zi
bash tools/gpu_steps.sh \
  "300|r2zi/tests|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k 'conv_vs_torch or stream_k'" \
  "300|r2zi/bench3x3|python -u tools/conv_bench.py --shape 32,28,28,128,128,3,1,1,0 --shape 32,14,14,256,256,3,1,1,0 --shape 32,7,7,512,512,3,1,1,0 --only 20,23,27,62,63,64,65,66,67,68,69,70 --ks 1,2,4,-1" \
  "240|r2zi/ab_s4|python -u tools/ab_cfg.py --model resnet50 --key 32x14x14x256,3x3s1p1111 --cfg 62 --json gpurun_out/r2zi/ab_s4.json" \
  "240|r2zi/ab_s3|python -u tools/ab_cfg.py --model resnet50 --key 32x28x28x128,3x3s1p1111 --cfg 63 --json gpurun_out/r2zi/ab_s3.json" \
  "240|r2zi/ab_s5|python -u tools/ab_cfg.py --model resnet50 --key 32x7x7x512,3x3s1p1111 --cfg 64 --ksplit 4 --json gpurun_out/r2zi/ab_s5.json"
