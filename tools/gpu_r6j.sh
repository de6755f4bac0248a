set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6j
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fp32_gpu.py tests/test_model_gpu.py tests/test_wino4s_gpu.py > gpurun_out/r6j/pytest_model.log 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_rccl_loopback_gpu.py -k hang > gpurun_out/r6j/pytest_loopback_hang.log 2>&1
