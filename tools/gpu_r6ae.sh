set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6ae
timeout -k 10 240 python tools/ab_cfg.py --precision fp32 --rounds 21 --env-a "ADAPT_STEM_F32_VARIANT=2" --env-b "ADAPT_STEM_F32_VARIANT=6" > gpurun_out/r6ae/ab_stem6.log 2>&1 &&
timeout -k 10 240 python tools/ab_cfg.py --precision fp32 --rounds 21 --env-a "ADAPT_STEM_F32_VARIANT=2" --env-b "ADAPT_STEM_F32_VARIANT=6" > gpurun_out/r6ae/ab_stem6_b.log 2>&1
