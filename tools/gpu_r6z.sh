set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6z
ADAPT_PW_RESPF=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_pw_f32_gpu.py > gpurun_out/r6z/pytest_pw_respf.log 2>&1 &&
timeout -k 10 240 python tools/ab_cfg.py --precision fp32 --rounds 21 --env-a "ADAPT_PW_RESPF=0" --env-b "ADAPT_PW_RESPF=1" > gpurun_out/r6z/ab_respf.log 2>&1 &&
timeout -k 10 240 python tools/ab_cfg.py --precision fp32 --rounds 21 --env-a "ADAPT_PW_RESPF=0" --env-b "ADAPT_PW_RESPF=1" > gpurun_out/r6z/ab_respf2.log 2>&1
