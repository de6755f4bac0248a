set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6x
timeout -k 10 400 python tools/codec_bench.py --json gpurun_out/r6x/codec.json > gpurun_out/r6x/codec.log 2>&1 &&
ADAPT_TEST_NORMAL_EXIT=1 timeout -k 10 1000 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r6x/pytest_gpu_normal_exit.log 2>&1
rc=$?
echo "suite rc=$rc" > gpurun_out/r6x/rc.txt
exit $rc
