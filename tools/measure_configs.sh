#!/bin/bash
# One-GPU measurement campaign for the BASELINE.json configs that fit a single
# MI355X (the driver runs the 2/4/8-GPU scaling bench itself).  Each step runs
# under its own timeout; the script stops at the first abnormal exit.
#   tools/measure_configs.sh [outdir]
out="${1:-gpurun_out/meas}"
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$root" && mkdir -p "$out"
M="python -m adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd"
run() {   # secs name cmd...
  local secs="$1" name="$2"; shift 2
  echo "=== [$name] $*"
  timeout -k 10 "$secs" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "=== [$name] rc=$rc"; tail -4 "$out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
[ -n "$SKIP_LOCAL" ] || run 300 local_cpu_bs1 $M local-infer --model resnet50 --batch 1 --requests 10 --device cpu
[ -n "$SKIP_LOCAL" ] || run 300 local_gpu_bs1 $M local-infer --model resnet50 --batch 1 --requests 200 --device cuda
[ -n "$SKIP_LOCAL" ] || run 300 local_gpu_bs32 $M local-infer --model resnet50 --batch 32 --requests 200 --device cuda
[ -n "$SKIP_LOCAL" ] || run 300 bench_r152 python bench.py --model resnet152 --steps 50 --warmup 10
run 400 serve_2stage_tcp $M serve --model resnet50 --batch 32 --part-at conv3_block1_1_conv --spawn 2 --device cuda:0 --codec none --requests 300
run 300 serve_2stage_bs1 $M serve --model resnet50 --batch 1 --part-at conv3_block1_1_conv --spawn 2 --device cuda:0 --codec none --requests 500
run 400 serve_2stage_zvc $M serve --model resnet50 --batch 32 --part-at conv3_block1_1_conv --spawn 2 --device cuda:0 --codec zvc --requests 300
run 500 serve_4stage_r152 $M serve --model resnet152 --batch 32 --part-at auto:4 --spawn 4 --device cuda:0 --codec none --requests 200
run 500 fault_r50_4w python tools/fault_bench.py --workers 4 --device cuda:0 --model resnet50 --image 224 --batch 32 --duration 25 --kill-at 10 --codec zvc --inflight 8 --json "$out/fault_r50_4w.json"
run 400 pp2_gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --mode pp --backend gloo --part-at conv3_block1_1_conv --steps 30 --warmup 5
