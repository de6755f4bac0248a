set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6ab
timeout -k 10 240 python tools/ab_cfg.py --precision fp32 --rounds 21 --set "32x28x28x128,1x1s1p0000,512@120@1" > gpurun_out/r6ab/ab_s3out_120.log 2>&1 &&
timeout -k 10 240 python tools/ab_cfg.py --precision fp32 --rounds 21 --set "32x28x28x128,1x1s1p0000,512@120@1" > gpurun_out/r6ab/ab_s3out_120_b.log 2>&1
