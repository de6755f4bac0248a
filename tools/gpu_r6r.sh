set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6r
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_pw_f32_gpu.py tests/test_fp32_gpu.py > gpurun_out/r6r/pytest_pw.log 2>&1 &&
timeout -k 10 120 python tools/pw_timeline.py --shape 32,14,14,256,1024 --cfg 123 --res --json gpurun_out/r6r/tl.jsonl > gpurun_out/r6r/tl.log 2>&1 &&
timeout -k 10 120 python tools/pw_timeline.py --shape 32,28,28,512,128 --cfg 123 --json gpurun_out/r6r/tl.jsonl >> gpurun_out/r6r/tl.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/r6r/bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6r/prof -o fp32 -- python3 bench.py --steps 20 --warmup 5 --no-bf16 > gpurun_out/r6r/prof.log 2>&1 &&
python tools/rocpd_kernels.py gpurun_out/r6r/prof/fp32_results.db --grid > gpurun_out/r6r/kernels_fp32.txt 2>&1
