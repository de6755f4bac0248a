set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6aj
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fp32_gpu.py tests/test_kernels_gpu.py -k "dense or head or softmax or finish" > gpurun_out/r6aj/pytest_head.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6aj/prof -o fp32 -- python3 bench.py --steps 20 --warmup 5 --no-bf16 > gpurun_out/r6aj/prof.log 2>&1 &&
python tools/rocpd_kernels.py gpurun_out/r6aj/prof/fp32_results.db --grid > gpurun_out/r6aj/kernels_fp32.txt 2>&1
