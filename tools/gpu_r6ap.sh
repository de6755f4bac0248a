set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6ap
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_pw_f32_gpu.py tests/test_fp32_gpu.py > gpurun_out/r6ap/pytest.log 2>&1 &&
timeout -k 10 240 python tools/ab_cfg.py --precision fp32 --rounds 21 --env-a "ADAPT_PW_ACT_GENERIC=1" --env-b "ADAPT_PW_ACT_GENERIC=0" > gpurun_out/r6ap/ab_act.log 2>&1 &&
timeout -k 10 240 python tools/ab_cfg.py --precision fp32 --rounds 21 --env-a "ADAPT_PW_ACT_GENERIC=1" --env-b "ADAPT_PW_ACT_GENERIC=0" > gpurun_out/r6ap/ab_act_b.log 2>&1
