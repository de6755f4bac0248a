set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6ac
ADAPT_W4S_IN=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wino4s_gpu.py > gpurun_out/r6ac/pytest_in2.log 2>&1 &&
timeout -k 10 200 python tools/wino4s_bench.py --cfgs 221 --ks 1,4,8 --no-tuned > gpurun_out/r6ac/bench_in1.log 2>&1 &&
ADAPT_W4S_IN=2 timeout -k 10 200 python tools/wino4s_bench.py --cfgs 221 --ks 1,4,8 --no-tuned > gpurun_out/r6ac/bench_in2.log 2>&1 &&
timeout -k 10 240 python tools/ab_cfg.py --precision fp32 --rounds 21 --env-a "ADAPT_W4S_IN=1" --env-b "ADAPT_W4S_IN=2" > gpurun_out/r6ac/ab_in2.log 2>&1 &&
timeout -k 10 240 python tools/ab_cfg.py --precision fp32 --rounds 21 --env-a "ADAPT_W4S_IN=1" --env-b "ADAPT_W4S_IN=2" > gpurun_out/r6ac/ab_in2_b.log 2>&1
