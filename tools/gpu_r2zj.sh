#!/bin/bash
# Round-2 GPU pass zj: whole-model A/B of the K-group conv configs per 3x3 group and combined.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r2zj
S3=32x28x28x128,3x3s1p1111; S4=32x14x14x256,3x3s1p1111; S5=32x7x7x512,3x3s1p1111
bash tools/gpu_steps.sh \
  "200|r2zj/s3_65|python -u tools/ab_cfg.py --set $S3@65@1 --json gpurun_out/r2zj/s3_65.json" \
  "200|r2zj/s5_68|python -u tools/ab_cfg.py --set $S5@68@1 --json gpurun_out/r2zj/s5_68.json" \
  "200|r2zj/s5_62|python -u tools/ab_cfg.py --set $S5@62@2 --json gpurun_out/r2zj/s5_62.json" \
  "200|r2zj/s4_62|python -u tools/ab_cfg.py --set $S4@62@1 --json gpurun_out/r2zj/s4_62.json" \
  "200|r2zj/s4_66|python -u tools/ab_cfg.py --set $S4@66@1 --json gpurun_out/r2zj/s4_66.json" \
  "200|r2zj/all|python -u tools/ab_cfg.py --set $S3@65@1 --set $S4@62@1 --set $S5@62@2 --rounds 21 --json gpurun_out/r2zj/all.json"
