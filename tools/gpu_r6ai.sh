set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6ai
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wino4s_gpu.py > gpurun_out/r6ai/pytest_w4s.log 2>&1 &&
timeout -k 10 240 python tools/ab_cfg.py --precision fp32 --rounds 21 --env-a "ADAPT_W4S_REDUCE=0" --env-b "ADAPT_W4S_REDUCE=1" > gpurun_out/r6ai/ab_reduce.log 2>&1 &&
timeout -k 10 240 python tools/ab_cfg.py --precision fp32 --rounds 21 --env-a "ADAPT_W4S_REDUCE=0" --env-b "ADAPT_W4S_REDUCE=1" > gpurun_out/r6ai/ab_reduce_b.log 2>&1
