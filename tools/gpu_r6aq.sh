set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6aq
timeout -k 10 1000 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r6aq/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/r6aq/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/r6aq/bench.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r6aq/bench_driver_style.log 2>&1 &&
timeout -k 10 300 python -u bench.py --model resnet152 --steps 50 --warmup 10 > gpurun_out/r6aq/bench_r152.log 2>&1
