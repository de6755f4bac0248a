set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6g
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wino4s_gpu.py > gpurun_out/r6g/pytest_wino4s.log 2>&1 &&
for cpt in 0; do
timeout -k 10 300 python tools/wino4s_bench.py --cfgs 221,227,232,233,234,235 --no-tuned > gpurun_out/r6g/bench_cpt$cpt.log 2>&1 || exit 1
done
