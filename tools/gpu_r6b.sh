set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6b
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --steps 20 --warmup 5 > gpurun_out/r6b/bench_gloo2.log 2>&1 &&
timeout -k 10 400 python bench.py --gpus 4 --backend gloo --steps 20 --warmup 5 > gpurun_out/r6b/bench_gloo4.log 2>&1 &&
timeout -k 10 200 python examples/local_infer.py --device cpu --requests 20 > gpurun_out/r6b/local_infer_cpu_bs1.log 2>&1
