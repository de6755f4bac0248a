set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6l
timeout -k 10 200 python tools/wino4s_timeline.py --json gpurun_out/r6l/timeline.json > gpurun_out/r6l/timeline.log 2>&1 &&
bash tools/gpu_r6k.sh
