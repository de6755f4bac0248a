set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6d
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6d/prof -o w4s -- python3 tools/wino4s_bench.py --cfgs 221,223 > gpurun_out/r6d/bench.log 2>&1
