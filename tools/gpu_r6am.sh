set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6am
timeout -k 10 240 python tools/ab_cfg.py --precision bf16 --rounds 21 --set "32x14x14x256,1x1s1p0000,1024@76@2" > gpurun_out/r6am/ab_bf16_s4out_76.log 2>&1 &&
timeout -k 10 240 python tools/ab_cfg.py --precision bf16 --rounds 21 --set "32x14x14x256,1x1s1p0000,1024@76@2" > gpurun_out/r6am/ab_bf16_s4out_76_b.log 2>&1
