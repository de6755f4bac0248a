set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6ak
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py > gpurun_out/r6ak/pytest.log 2>&1 &&
timeout -k 10 240 python tools/ab_cfg.py --precision bf16 --rounds 21 --env-a "ADAPT_SPLITK_GENERIC=1" --env-b "ADAPT_SPLITK_GENERIC=0" > gpurun_out/r6ak/ab_splitk.log 2>&1 &&
timeout -k 10 240 python tools/ab_cfg.py --precision bf16 --rounds 21 --env-a "ADAPT_SPLITK_GENERIC=1" --env-b "ADAPT_SPLITK_GENERIC=0" > gpurun_out/r6ak/ab_splitk_b.log 2>&1
