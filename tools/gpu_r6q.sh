set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6q
timeout -k 10 1000 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r6q/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/r6q/smoke.log 2>&1
