set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6ad
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fp32_gpu.py -k stem_f32 > gpurun_out/r6ad/pytest_stem.log 2>&1 &&
timeout -k 10 200 python tools/stem_bench.py --iters 100 > gpurun_out/r6ad/stem_bench.log 2>&1 &&
timeout -k 10 200 python tools/stem_bench.py --iters 100 > gpurun_out/r6ad/stem_bench_b.log 2>&1
