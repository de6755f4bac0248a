cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/r4c
export TMPDIR=/tmp
timeout -k 10 120 python -u bench.py --no-bf16 --steps 50 --warmup 10 > gpurun_out/r4c/b32.log 2>&1 || exit $?
timeout -k 10 120 python -u bench.py --no-bf16 --steps 50 --warmup 10 --batch 16 --streams 2 > gpurun_out/r4c/b16x2.log 2>&1 || exit $?
timeout -k 10 120 python -u bench.py --no-bf16 --steps 50 --warmup 10 --batch 8 --streams 4 > gpurun_out/r4c/b8x4.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --no-bf16 --steps 50 --warmup 10 --batch 16 --streams 2 --tune > gpurun_out/r4c/b16x2_tune.log 2>&1 || exit $?
timeout -k 10 120 python -u bench.py --dtype bf16 --steps 50 --warmup 10 --batch 16 --streams 2 > gpurun_out/r4c/bf16_b16x2.log 2>&1 || exit $?
tail -n 2 gpurun_out/r4c/*.log
