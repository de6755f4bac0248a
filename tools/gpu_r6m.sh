set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6m
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wino4s_gpu.py > gpurun_out/r6m/pytest_wino4s.log 2>&1 &&
timeout -k 10 200 python tools/wino4s_timeline.py --json gpurun_out/r6m/timeline.json > gpurun_out/r6m/timeline.log 2>&1 &&
timeout -k 10 300 python tools/wino4s_bench.py --cfgs 221,227,236,237 --ks 1,2,4,8 > gpurun_out/r6m/bench.log 2>&1
