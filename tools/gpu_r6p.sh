set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6p
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > gpurun_out/r6p/bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6p/prof -o fp32 -- python3 bench.py --steps 20 --warmup 5 --no-bf16 > gpurun_out/r6p/prof.log 2>&1 &&
python tools/rocpd_kernels.py $(ls gpurun_out/r6p/prof/*/fp32_results.db gpurun_out/r6p/prof/fp32_results.db 2>/dev/null | head -1) --grid > gpurun_out/r6p/kernels_fp32.txt 2>&1
