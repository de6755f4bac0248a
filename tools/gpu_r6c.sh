set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6c
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_wino4s_gpu.py > gpurun_out/r6c/pytest_wino4s.log 2>&1 &&
timeout -k 10 300 python tools/wino4s_bench.py --json gpurun_out/r6c/wino4s_bench.json > gpurun_out/r6c/wino4s_bench.log 2>&1
