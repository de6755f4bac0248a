set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6f
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wino4s_gpu.py > gpurun_out/r6f/pytest_wino4s.log 2>&1 &&
timeout -k 10 300 python tools/wino4s_bench.py --cfgs 220,221,223,227,228,230 > gpurun_out/r6f/wino4s_bench.log 2>&1 &&
bash tools/gpu_r6e.sh
