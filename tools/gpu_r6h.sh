set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6h
S2="32x56x56x64,3x3s1p1111"; S3="32x28x28x128,3x3s1p1111"; S4="32x14x14x256,3x3s1p1111"; S5="32x7x7x512,3x3s1p1111"
timeout -k 10 300 python tools/ab_cfg.py --precision fp32 --rounds 10 --set "$S2@227@1" --set "$S3@221@2" --set "$S4@221@4" --set "$S5@221@8" --json gpurun_out/r6h/ab_all.json > gpurun_out/r6h/ab_all.log 2>&1 &&
timeout -k 10 200 python tools/ab_cfg.py --precision fp32 --rounds 10 --set "$S2@227@1" > gpurun_out/r6h/ab_s2.log 2>&1 &&
timeout -k 10 200 python tools/ab_cfg.py --precision fp32 --rounds 10 --set "$S3@221@2" > gpurun_out/r6h/ab_s3.log 2>&1 &&
timeout -k 10 200 python tools/ab_cfg.py --precision fp32 --rounds 10 --set "$S4@221@4" > gpurun_out/r6h/ab_s4.log 2>&1 &&
timeout -k 10 200 python tools/ab_cfg.py --precision fp32 --rounds 10 --set "$S5@221@8" > gpurun_out/r6h/ab_s5.log 2>&1
