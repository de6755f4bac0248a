set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6s
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_pw_f32_gpu.py > gpurun_out/r6s/pytest_pw.log 2>&1 &&
timeout -k 10 240 python tools/ab_cfg.py --precision fp32 --rounds 21 --env-a "ADAPT_PW_NOSHARE=1" --env-b "ADAPT_PW_NOSHARE=0" > gpurun_out/r6s/ab_pwshare.log 2>&1 &&
timeout -k 10 240 python tools/ab_cfg.py --precision fp32 --rounds 21 --env-a "ADAPT_PW_NOSHARE=1" --env-b "ADAPT_PW_NOSHARE=0" > gpurun_out/r6s/ab_pwshare2.log 2>&1
