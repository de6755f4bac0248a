#!/bin/bash
# Per-block fixed cost of the fp32 Winograd v2 kernel: time vs input channels (K chunks) at fixed
# spatial shape / output channels; the intercept of the linear fit is the prologue + epilogue + launch.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/r4w
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/conv_bench_f32.py --only 103 --ks 1 \
  --shape 32,56,56,16,64,3,1,1,0 --shape 32,56,56,32,64,3,1,1,0 --shape 32,56,56,64,64,3,1,1,0 \
  --shape 32,56,56,128,64,3,1,1,0 --shape 32,56,56,256,64,3,1,1,0 \
  --shape 32,28,28,16,128,3,1,1,0 --shape 32,28,28,32,128,3,1,1,0 --shape 32,28,28,64,128,3,1,1,0 \
  --shape 32,28,28,128,128,3,1,1,0 --shape 32,28,28,256,128,3,1,1,0 > gpurun_out/r4w/wino_vs_c.log 2>&1
# the same for the 1x1 tile GEMM (conv_f32g cfg 18, stream-K 2) and the persistent pointwise kernel (cfg 120)
timeout -k 10 200 python -u tools/conv_bench_f32.py --only 18,38,120 --ks 1,-2 \
  --shape 32,14,14,128,256,1,1,0,0 --shape 32,14,14,256,256,1,1,0,0 --shape 32,14,14,512,256,1,1,0,0 \
  --shape 32,14,14,1024,256,1,1,0,0 --shape 32,14,14,2048,256,1,1,0,0 > gpurun_out/r4w/gemm_vs_k.log 2>&1
