set -o pipefail
mkdir -p gpurun_out/g1
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/g1/smoke.log 2>&1 &&
timeout -k 10 240 python -u bench.py --steps 50 --warmup 10 > gpurun_out/g1/bench1.log 2>&1 &&
timeout -k 10 300 python -u bench.py --gpus 2 --mode pp --backend gloo --part-at conv3_block1_1_conv --steps 10 --warmup 3 > gpurun_out/g1/bench_pp2.log 2>&1 &&
timeout -k 10 300 python -u bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/g1/bench_dp2.log 2>&1
