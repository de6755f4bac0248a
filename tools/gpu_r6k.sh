set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6k
cd $R && timeout -k 10 400 rocprofv3 --kernel-trace -d $R/gpurun_out/r6k/prof -o hang -- python3 -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_rccl_loopback_gpu.py -k hang > $R/gpurun_out/r6k/pytest_hang.log 2>&1
