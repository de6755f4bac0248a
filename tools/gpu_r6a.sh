set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6a
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_rccl_native_gpu.py -s > gpurun_out/r6a/pytest_rccl.log 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r6a/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/r6a/bench.log 2>&1
