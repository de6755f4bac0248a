set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6y
ADAPT_PAIR_F32_DEPTH=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_pair_f32_gpu.py > gpurun_out/r6y/pytest_pair.log 2>&1 &&
timeout -k 10 240 python tools/ab_cfg.py --precision fp32 --rounds 21 --env-a "ADAPT_PAIR_F32_DEPTH=1" --env-b "ADAPT_PAIR_F32_DEPTH=2" > gpurun_out/r6y/ab_pair_depth.log 2>&1
