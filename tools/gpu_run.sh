#!/bin/bash
# One parameterised GPU pass for gpurun (replaces the per-pass lease scripts).
#   usage: tools/gpu_run.sh <outdir> <preset>[,<preset>...]
#   e.g.   gpurun --timeout 1100 -- bash tools/gpu_run.sh r3a suite,smoke,bench,prof
# Presets (each step has its own time limit; a fault stops the pass, see gpu_steps.sh):
#   suite     the GPU test suite
#   rccl      the native RCCL layer tests only + RCCL self-p2p under rocprofv3
#   smoke     __graft_entry__.smoke()
#   bench     default bench.py (fp32 headline + bf16 companion), then a longer run
#   bench152  ResNet-152 (bf16 and fp32)
#   rehearse  bench.py --gpus 2 --backend gloo (the multi-GPU record, ranks sharing one GPU, with its
#             pp / fault sub-runs); rehearse4 the same at --gpus 4 (adds the ResNet-152 4-stage sub-run)
#   queues    compute stream vs spinning link / side streams (tests/test_stream_queues_gpu.py)
#   prof      rocprofv3 kernel trace + stats of the fp32 and bf16 benches
#   fp32t     the fp32 kernel / model tests only
#   models    model numerics + multi-GPU link twins + DEFER GPU tests
#   peak      fp32 MFMA ceiling under full load (tools/mfma_f32_peak.hip, prebuilt .bin)
#   tune32    fp32 conv autotune of ResNet-50 bs=32 (entries to gpurun_out/<outdir>/tune_f32.json)
#   fault     4-stage SIGKILL recovery bench (device links)
#   pmc32     two rocprofv3 PMC passes over the fp32 bench (tools/pmc_summary.py reads them)
#   hang      4-stage wedged-stage (alive, no progress) recovery bench (device links)
#   roof32    per-layer fp32 roofline table (two PMC passes over tools/roofline_r50.py --dtype fp32)
#   roof16    the same for bf16
#   cs3       channel-split 3x3 (stage 4/5) numerics, isolated timings vs the tile kernels, whole-model A/B
#   wino      fp32 Winograd numerics + isolated timings of the v2 configs on the four ResNet-50 3x3 shapes
#   pmcw      PMC passes over the fp32 Winograd kernel (tools/pmc_f32.sh), stage 2-5 shapes
#   faultd    config 4 at the shipped DEFER defaults (fp32, transport auto, 0.25 s heartbeat): 4- and
#             8-worker SIGKILL and a 4-worker hang, all workers on cuda:0 (parallel/fault_run.py)
#   wino4     fp32 Winograd numerics + isolated timings incl. the v3 cfgs 116/117
#   stem      fp32 stem numerics + isolated timing (tools/stem_bench.py)
#   stem16    bf16 stem numerics (v1-v4) + isolated timing
#   wino5     Winograd numerics + isolated timings of 118/119 vs the front-loaded DMA cfgs 150-153
#   wino6     Winograd numerics + isolated timings of 118 vs the stagger / priority cfgs 154-156
#   wtl       per-block phase timelines of the Winograd kernel on the four ResNet-50 3x3 shapes
#   skp       stream-K Winograd probe (tools/debug/sk_probe.py) + the Winograd tests + v3 stream-K timings
#   wino7     Winograd numerics + isolated timings of 118 / 155 vs the half-prefetch cfgs 160 / 161
#   pw5       pointwise numerics + isolated timings incl. the deep-ring streaming cfg 124
#   wino8     Winograd numerics + isolated timings: 118 / 155 / 116 / 117 vs early patch read (162/163)
#             and the DMA hidden from the wait model (164-167)
#   wino9     Winograd numerics + timings of 118 / 155 / 167 vs the counter-synchronised cfg 171, and the
#             in-loop timelines of 170 (barrier) vs 172 (counters)
#   pwtl      pointwise numerics, timings and per-wave timelines (tools/pw_timeline.py)
#   pw6       pointwise numerics + isolated timings incl. the K-split tail configs 125 / 126
#   pmcstem   two PMC passes over the fp32 stem (tools/stem_bench.py)
#   pmc1x1    PMC passes over the tuned fp32 1x1 convs of ResNet-50 (stage 2/4 GEMMs, stage-3 shortcut)
#   w4        Winograd F(4x4, 3x3) numerics (fp64 oracle) + isolated timings vs the tuned F(2x2) configs
#   rehearse8 bench.py --gpus 8 --backend gloo (8 ranks sharing one GPU: config-3 lz4 pipeline + 8-worker fault)
#   w4t       per-wave phase timelines of the F(4x4) kernel (tools/wino4_timeline.py)
#   loop      the RCCL branch of the stage data plane over the test-only loopback communicator (steady,
#             SIGKILL, hang; tests/test_rccl_loopback_gpu.py)
#   ab4       whole-model fp32 A/B: the tuned 3x3s vs F(4x4) cfg 200 on stages 3-5 (tools/ab_cfg.py)
#   li        the reference's local_infer protocol at fp32: ResNet-50 bs=1, 10 and 1000 requests
#   codec     activation-codec table on the ResNet-50 bs=32 frontiers, fp32 (tools/codec_bench.py)
#   w4x / w4pc / w4pcx  F(4x4) measurement variants / producer-consumer tests + timelines / its variants
# Extra steps: GPU_EXTRA="secs|name|cmd" (one step; quoted as for gpu_steps.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
out="$1"; presets="$2"
[ -n "$out" ] && [ -n "$presets" ] || { echo "usage: $0 <outdir> <preset>[,...]"; exit 2; }
mkdir -p "gpurun_out/$out"
steps=()
IFS=',' read -ra P <<< "$presets"
for p in "${P[@]}"; do
  case "$p" in
    suite)    steps+=("600|$out/pytest_gpu|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread") ;;
    rccl)     steps+=("180|$out/pytest_rccl|python -u -m pytest tests/test_rccl_native_gpu.py -m gpu -v --timeout 60 --timeout-method thread")
              steps+=("120|$out/rccl_prof|rocprofv3 --kernel-trace --stats -d gpurun_out/$out/rccl_prof -o run -- python3 tools/rccl_selftest.py") ;;
    smoke)    steps+=("180|$out/smoke|python -u -c 'import __graft_entry__ as g; g.smoke()'") ;;
    bench)    steps+=("240|$out/bench_default|python -u bench.py")
              steps+=("240|$out/bench_long|python -u bench.py --steps 200 --warmup 20") ;;
    bench152) steps+=("240|$out/bench_r152|python -u bench.py --model resnet152 --steps 50 --warmup 10") ;;
    rehearse) steps+=("500|$out/bench_gloo2|python -u bench.py --gpus 2 --backend gloo --steps 10 --warmup 3") ;;
    rehearse4) steps+=("600|$out/bench_gloo4|python -u bench.py --gpus 4 --backend gloo --steps 10 --warmup 3") ;;
    rehearse8) steps+=("600|$out/bench_gloo8|python -u bench.py --gpus 8 --backend gloo --steps 10 --warmup 3") ;;
    w4)       steps+=("300|$out/pytest_wino4|python -u -m pytest tests/test_wino4_gpu.py -v -s -x --timeout 120 --timeout-method thread")
              steps+=("300|$out/wino4_bench|python -u tools/wino4_bench.py") ;;
    w4t)      steps+=("200|$out/wino4_timeline|python -u tools/wino4_timeline.py --json gpurun_out/$out/wino4_timeline.json") ;;
    w4pc)     steps+=("300|$out/pytest_wino4|python -u -m pytest tests/test_wino4_gpu.py -v -s -x --timeout 120 --timeout-method thread")
              steps+=("120|$out/wino4pc_timeline|python -u tools/wino4_timeline.py --cfg 210 --json gpurun_out/$out/wino4pc_timeline.json")
              steps+=("300|$out/wino4_bench|python -u tools/wino4_bench.py") ;;
    ab4)      steps+=("300|$out/ab_wino4|python -u tools/ab_cfg.py --precision fp32 --set 32x28x28x128,3x3s1p1111@200@1 --set 32x14x14x256,3x3s1p1111@200@2 --set 32x7x7x512,3x3s1p1111@200@4 --json gpurun_out/$out/ab_wino4.json") ;;
    li)       steps+=("180|$out/local_infer_bs1_10|python -u -m adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd local-infer --model resnet50 --batch 1 --requests 10 --device cuda")
              steps+=("180|$out/local_infer_bs1_1000|python -u -m adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd local-infer --model resnet50 --batch 1 --requests 1000 --device cuda") ;;
    gemm1x1)  steps+=("300|$out/gemm1x1_bigtiles|python -u tools/conv_bench_f32.py --only 10,11,12,13,14,15,16,17,18,30,31,32,33,34,37,38 --ks 1,2,-1,-2 --top 8 --shape 32,14,14,1024,256,1,1,0,0 --shape 32,14,14,256,1024,1,1,0,1 --shape 32,7,7,2048,512,1,1,0,0 --shape 32,28,28,512,128,1,1,0,0 --shape 32,28,28,128,512,1,1,0,1") ;;
    bf3x3)    steps+=("300|$out/bf16_3x3_s45|python -u tools/conv_bench.py --shape 32,14,14,256,256,3,1,1,0 --shape 32,7,7,512,512,3,1,1,0 --ks 1,2,3,4,-1,-2") ;;
    gs)       steps+=("300|$out/pytest_gemm_f32s|python -u -m pytest tests/test_gemm_f32s_gpu.py -v -x --timeout 120 --timeout-method thread")
              steps+=("300|$out/gemm_f32s_bench|python -u tools/conv_bench_f32.py --only 300,301,302,303,304,305,306,18,38,122,123,125,126 --ks 1,-1,-2 --top 10 --shape 32,14,14,1024,256,1,1,0,0 --shape 32,14,14,256,1024,1,1,0,1 --shape 32,7,7,2048,512,1,1,0,0 --shape 32,7,7,512,2048,1,1,0,1 --shape 32,28,28,512,128,1,1,0,0 --shape 32,28,28,128,512,1,1,0,1 --shape 32,56,56,256,64,1,1,0,0 --shape 32,56,56,64,256,1,1,0,1") ;;
    gst)      steps+=("200|$out/gemm_f32s_timeline|python -u tools/gemm_f32s_timeline.py --json gpurun_out/$out/gemm_f32s_timeline.json") ;;
    codec)    steps+=("300|$out/codec_fp32|python -u tools/codec_bench.py --precision fp32 --json gpurun_out/$out/codec_fp32.json") ;;
    w4pcx)    steps+=("200|$out/wino4pc_exp|python -u tools/wino4_timeline.py --cfg 210 --exp 0,1,4,5,12,13,14,17,21 --json gpurun_out/$out/wino4pc_exp.json") ;;
    w4x)      steps+=("200|$out/wino4_exp|python -u tools/wino4_timeline.py --exp 0,8,4,1,2 --json gpurun_out/$out/wino4_exp.json") ;;
    loop)     steps+=("600|$out/pytest_loop|python -u -m pytest tests/test_rccl_loopback_gpu.py -v -s -x --timeout 300 --timeout-method thread") ;;
    qprobe)   for q in 4 8 16; do steps+=("90|$out/qprobe_$q|GPU_MAX_HW_QUEUES=$q python -u tools/queue_probe.py"); done ;;
    queues)   steps+=("180|$out/pytest_queues|python -u -m pytest tests/test_stream_queues_gpu.py -m gpu -v -s --timeout 120 --timeout-method thread") ;;
    prof)     steps+=("240|$out/prof_fp32|rocprofv3 --kernel-trace --stats -d gpurun_out/$out/prof_fp32 -o run -- python3 bench.py --no-bf16 --steps 30 --warmup 5")
              steps+=("240|$out/prof_bf16|rocprofv3 --kernel-trace --stats -d gpurun_out/$out/prof_bf16 -o run -- python3 bench.py --dtype bf16 --steps 50 --warmup 10") ;;
    fp32t)    steps+=("400|$out/pytest_fp32|python -u -m pytest tests/test_fp32_gpu.py -m gpu -v -x --timeout 120 --timeout-method thread") ;;
    models)   steps+=("600|$out/pytest_models|python -u -m pytest tests/test_model_gpu.py tests/test_multigpu_links.py tests/test_defer_gpu.py -m gpu -v --timeout 300 --timeout-method thread") ;;
    peak)     steps+=("60|$out/mfma_f32_peak|./tools/mfma_f32_peak.bin") ;;
    ab62)     steps+=("300|$out/ab_s5_3x3_62|python -u tools/ab_cfg.py --model resnet50 --key 32x7x7x512,3x3s1p1111,512 --cfg 62 --ksplit 2 --rounds 25 --json gpurun_out/$out/ab_s5_3x3_62.json")
              steps+=("300|$out/ab_s5_3x3_64|python -u tools/ab_cfg.py --model resnet50 --key 32x7x7x512,3x3s1p1111,512 --cfg 64 --ksplit 4 --rounds 25 --json gpurun_out/$out/ab_s5_3x3_64.json") ;;
    tune16w)  steps+=("900|$out/tune_bf16|env ADAPT_TUNE_REFINE=8 python -u tools/tune_f32.py --precision bf16 --models resnet50 --batch 32 --out gpurun_out/$out/tune_bf16.json")
              steps+=("900|$out/tune_f32|env ADAPT_TUNE_REFINE=8 python -u tools/tune_f32.py --precision fp32 --models resnet50 --batch 32 --out gpurun_out/$out/tune_f32.json") ;;
    tune16)   steps+=("900|$out/tune_bf16|python -u tools/tune_f32.py --precision bf16 --models resnet50 --batch 32 --out gpurun_out/$out/tune_bf16.json") ;;
    tune32)   steps+=("600|$out/tune_f32|python -u tools/tune_f32.py --models resnet50 --batch 32 --out gpurun_out/$out/tune_f32.json") ;;
    pmc32)    steps+=("500|$out/pmc32|bash tools/pmc_run.sh gpurun_out/$out/pmc32 bench.py --no-bf16 --steps 2 --warmup 1") ;;
    hang)     steps+=("300|$out/hang4_dev|python -u tools/fault_bench.py --workers 4 --device cuda:0 --model resnet50 --image 224 --batch 32 --duration 25 --kill-at 10 --links dev --inflight 8 --fault hang --json gpurun_out/$out/hang_r50_4w_dev.json") ;;
    fault)    steps+=("300|$out/fault4_dev|python -u tools/fault_bench.py --workers 4 --device cuda:0 --model resnet50 --image 224 --batch 32 --duration 25 --kill-at 10 --links dev --inflight 8 --json gpurun_out/$out/fault_r50_4w_dev.json") ;;
    cs3)      steps+=("300|$out/pytest_cs3|python -u -m pytest tests/test_cs3_gpu.py tests/test_rr3_gpu.py -m gpu -v -x --timeout 120 --timeout-method thread")
              steps+=("240|$out/cs3_bench|python -u tools/conv_bench.py --shape 32,14,14,256,256,3,1,1 --shape 32,7,7,512,512,3,1,1 --only 73,0,1,2,3,4,5,6,7,8,9 --ks 1,2,4,-1")
              steps+=("240|$out/cs3_ab|python -u tools/ab_cfg.py --model resnet50 --set 32x14x14x256,3x3s1p1111@73@1 --set 32x7x7x512,3x3s1p1111@73@1 --json gpurun_out/$out/cs3_ab.json") ;;
    roof32)   steps+=("200|$out/roof32_meta|mkdir -p gpurun_out/$out/roof32 && python -u tools/roofline_r50.py --run --dtype fp32 --meta gpurun_out/$out/roof32/meta.json")
              steps+=("400|$out/roof32_pmc|bash tools/pmc_groups.sh gpurun_out/$out/roof32 'SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT' 'TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum' -- tools/roofline_r50.py --run --dtype fp32")
              steps+=("60|$out/roof32_table|python tools/roofline_r50.py --table gpurun_out/$out/roof32 --meta gpurun_out/$out/roof32/meta.json --json gpurun_out/$out/roof32/roofline_fp32.json") ;;
    roof16)   steps+=("200|$out/roof16_meta|mkdir -p gpurun_out/$out/roof16 && python -u tools/roofline_r50.py --run --dtype bf16 --meta gpurun_out/$out/roof16/meta.json")
              steps+=("400|$out/roof16_pmc|bash tools/pmc_groups.sh gpurun_out/$out/roof16 'SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT' 'TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum' -- tools/roofline_r50.py --run --dtype bf16")
              steps+=("60|$out/roof16_table|python tools/roofline_r50.py --table gpurun_out/$out/roof16 --meta gpurun_out/$out/roof16/meta.json --json gpurun_out/$out/roof16/roofline_bf16.json") ;;
    wino)     steps+=("200|$out/pytest_wino|python -u -m pytest tests/test_wino_gpu.py tests/test_wino.py -v -x --timeout 120 --timeout-method thread")
              steps+=("300|$out/wino_bench|python -u tools/conv_bench_f32.py --shape 32,56,56,64,64,3,1,1,0 --shape 32,28,28,128,128,3,1,1,0 --shape 32,14,14,256,256,3,1,1,0 --shape 32,7,7,512,512,3,1,1,0 --only 103,104,105,106,107,108 --ks 1,2,4,-2,-4") ;;
    wino4)    steps+=("200|$out/pytest_wino|python -u -m pytest tests/test_wino_gpu.py tests/test_wino.py -v -x --timeout 120 --timeout-method thread")
              steps+=("300|$out/wino_bench|python -u tools/conv_bench_f32.py --shape 32,56,56,64,64,3,1,1,0 --shape 32,28,28,128,128,3,1,1,0 --shape 32,14,14,256,256,3,1,1,0 --shape 32,7,7,512,512,3,1,1,0 --only 103,104,105,106,107,108,116,117,130,131,132,140,141 --ks 1,2,-2,-4") ;;
    wino23)   steps+=("200|$out/pytest_wino|python -u -m pytest tests/test_wino_gpu.py -v -x --timeout 120 --timeout-method thread")
              steps+=("300|$out/wino23_bench|python -u tools/conv_bench_f32.py --shape 32,56,56,64,64,3,1,1,0 --shape 32,28,28,128,128,3,1,1,0 --only 103,106,131,118,119 --ks 1")
              steps+=("300|$out/wino23_bench_b|python -u tools/conv_bench_f32.py --shape 32,56,56,64,64,3,1,1,0 --shape 32,28,28,128,128,3,1,1,0 --only 103,106,131,118,119 --ks 1") ;;
    pw4)      steps+=("200|$out/pytest_pw|python -u -m pytest tests/test_pw_f32_gpu.py -v -x --timeout 120 --timeout-method thread")
              steps+=("300|$out/pw_bench|python -u tools/conv_bench_f32.py --only 18,38,120,121,122,123 --ks 1,-2 --shape 32,28,28,128,512,1,1,0,1 --shape 32,28,28,512,128,1,1,0,0 --shape 32,14,14,256,1024,1,1,0,1 --shape 32,14,14,1024,256,1,1,0,0 --shape 32,7,7,512,2048,1,1,0,1 --shape 32,7,7,2048,512,1,1,0,0 --shape 32,56,56,64,256,1,1,0,1 --shape 32,56,56,256,64,1,1,0,0") ;;
    faultd)   for w in 4 8; do steps+=("300|$out/fault${w}_defaults|python -u -m adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.parallel.fault_run --workers $w --devices cuda:0 --model resnet50 --image 224 --batch 32 --duration 20 --kill-at 8 --json gpurun_out/$out/fault_r50_${w}w_defaults.json"); done
              steps+=("300|$out/hang4_defaults|python -u -m adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.parallel.fault_run --workers 4 --devices cuda:0 --model resnet50 --image 224 --batch 32 --duration 20 --kill-at 8 --fault hang --json gpurun_out/$out/hang_r50_4w_defaults.json") ;;
    pmcw)     steps+=("500|$out/pmcw|bash tools/pmc_f32.sh gpurun_out/$out/pmcw 32,56,56,64,64,3,1,1,0:106:1 32,56,56,64,64,3,1,1,0:103:1 32,28,28,128,128,3,1,1,0:106:1 32,28,28,128,128,3,1,1,0:103:1 32,14,14,256,256,3,1,1,0:108:1 32,14,14,256,256,3,1,1,0:105:1") ;;
    pmc1x1)   steps+=("500|$out/pmc1x1|bash tools/pmc_f32.sh gpurun_out/$out/pmc1x1 32,14,14,1024,256,1,1,0,0:18:-2 32,14,14,256,1024,1,1,0,1:38:1 32,56,56,64,256,1,1,0,1:3:1 32,28,28,512,1024,1,2,0,0:20:-1") ;;
    ps)       steps+=("300|$out/pytest_ps|python -u -m pytest tests/test_pw_slice_gpu.py -v -x --timeout 120 --timeout-method thread")
              steps+=("300|$out/ps_bench|python -u tools/ps_bench.py --json gpurun_out/$out/ps_bench.json") ;;
    psab)     steps+=("300|$out/ab_ps_s4out|python -u tools/ab_cfg.py --model resnet50 --key 32x14x14x256,1x1s1p0000,1024 --cfg 75 --ksplit 2 --json gpurun_out/$out/ab_ps_s4out.json")
              steps+=("300|$out/ab_ps_s3one|python -u tools/ab_cfg.py --model resnet50 --key 32x28x28x512,1x1s1p0000,128 --cfg 76 --ksplit 1 --json gpurun_out/$out/ab_ps_s3one.json") ;;
    gstm)     steps+=("300|$out/pytest_gemm_f32s|python -u -m pytest tests/test_gemm_f32s_gpu.py -v -x --timeout 120 --timeout-method thread")
              steps+=("300|$out/gemm_f32s_tm_bench|python -u tools/conv_bench_f32.py --only 307,308,18,38,122,123,125,126 --ks 1,-1,-2 --top 8 --shape 32,14,14,1024,256,1,1,0,0 --shape 32,7,7,512,2048,1,1,0,1")
              steps+=("300|$out/ab_f32s_307|python -u tools/ab_cfg.py --precision fp32 --model resnet50 --key 32x14x14x1024,1x1s1p0000,256 --cfg 307 --ksplit 1 --json gpurun_out/$out/ab_f32s_307.json")
              steps+=("300|$out/ab_f32s_308|python -u tools/ab_cfg.py --precision fp32 --model resnet50 --key 32x7x7x512,1x1s1p0000,2048 --cfg 308 --ksplit 1 --json gpurun_out/$out/ab_f32s_308.json") ;;
    gstm2)    steps+=("300|$out/pytest_gemm_f32s|python -u -m pytest tests/test_gemm_f32s_gpu.py -v -x --timeout 120 --timeout-method thread")
              steps+=("300|$out/ab_f32s_307|python -u tools/ab_cfg.py --precision fp32 --model resnet50 --key 32x14x14x1024,1x1s1p0000,256 --cfg 307 --ksplit 1 --rounds 25 --json gpurun_out/$out/ab_f32s_307.json")
              steps+=("300|$out/ab_f32s_309|python -u tools/ab_cfg.py --precision fp32 --model resnet50 --key 32x7x7x2048,1x1s1p0000,512 --cfg 309 --ksplit 1 --rounds 25 --json gpurun_out/$out/ab_f32s_309.json") ;;
    ps3)      steps+=("300|$out/pytest_ps|python -u -m pytest tests/test_pw_slice_gpu.py -v -x --timeout 120 --timeout-method thread")
              steps+=("300|$out/ps_bench|python -u tools/ps_bench.py --shape 25088,128,512,1 --json gpurun_out/$out/ps_bench.json")
              steps+=("300|$out/ab_ps_s3out_74|python -u tools/ab_cfg.py --model resnet50 --key 32x28x28x128,1x1s1p0000,512 --cfg 74 --ksplit 1 --rounds 25")
              steps+=("300|$out/ab_ps_s3out_75|python -u tools/ab_cfg.py --model resnet50 --key 32x28x28x128,1x1s1p0000,512 --cfg 75 --ksplit 2 --rounds 25") ;;
    ab4s)     steps+=("300|$out/ab_w4_s5|python -u tools/ab_cfg.py --precision fp32 --model resnet50 --key 32x7x7x512,3x3s1p1111 --cfg 200 --ksplit 4 --rounds 25")
              steps+=("300|$out/ab_w4_s4|python -u tools/ab_cfg.py --precision fp32 --model resnet50 --key 32x14x14x256,3x3s1p1111 --cfg 200 --ksplit 2 --rounds 25")
              steps+=("300|$out/ab_w4_s3|python -u tools/ab_cfg.py --precision fp32 --model resnet50 --key 32x28x28x128,3x3s1p1111 --cfg 200 --ksplit 1 --rounds 25") ;;
    psab2)    steps+=("300|$out/ab_ps_s4one|python -u tools/ab_cfg.py --model resnet50 --key 32x14x14x1024,1x1s1p0000,256 --cfg 76 --ksplit 1 --rounds 25")
              steps+=("300|$out/ab_ps_s5out|python -u tools/ab_cfg.py --model resnet50 --key 32x7x7x512,1x1s1p0000,2048 --cfg 75 --ksplit 1 --rounds 25") ;;
    abs4)     steps+=("5|$out/abs4_start|true")
              steps+=("300|$out/ab_s4_3x3_62_2|python -u tools/ab_cfg.py --model resnet50 --key 32x14x14x256,3x3s1p1111,256 --cfg 62 --ksplit 2 --rounds 25")
              steps+=("300|$out/ab_s4_3x3_62_-2|python -u tools/ab_cfg.py --model resnet50 --key 32x14x14x256,3x3s1p1111,256 --cfg 62 --ksplit -2 --rounds 25")
              steps+=("300|$out/ab_s4_3x3_63_2|python -u tools/ab_cfg.py --model resnet50 --key 32x14x14x256,3x3s1p1111,256 --cfg 63 --ksplit 2 --rounds 25")
              steps+=("300|$out/ab_s4_3x3_64_2|python -u tools/ab_cfg.py --model resnet50 --key 32x14x14x256,3x3s1p1111,256 --cfg 64 --ksplit 2 --rounds 25") ;;
    stemt)    steps+=("120|$out/stem_timeline|python -u tools/stem_timeline.py --json gpurun_out/$out/stem_timeline.json") ;;
    stemt67)  steps+=("120|$out/stem_timeline6|python -u tools/stem_timeline.py --version 6 --json gpurun_out/$out/stem_timeline6.json")
              steps+=("120|$out/stem_timeline7|python -u tools/stem_timeline.py --version 7 --json gpurun_out/$out/stem_timeline7.json") ;;
    stemx)    steps+=("120|$out/stem_exp|python -u tools/stem_timeline.py --version 4 --exp 0,1,2,4,8,3,13,15 --json gpurun_out/$out/stem_exp.json") ;;
    stem16)   steps+=("200|$out/pytest_stem16|python -u -m pytest tests/test_kernels_gpu.py -k stem -v -x --timeout 120 --timeout-method thread")
              steps+=("120|$out/stem_bench|python -u tools/stem_bench.py") ;;
    stem)     steps+=("200|$out/pytest_stem|python -u -m pytest tests/test_fp32_gpu.py -k stem -v -x --timeout 120 --timeout-method thread")
              steps+=("120|$out/stem_bench|python -u tools/stem_bench.py")
              steps+=("120|$out/stem_bench_b|python -u tools/stem_bench.py") ;;
    wino5)    steps+=("200|$out/pytest_wino|python -u -m pytest tests/test_wino_gpu.py -v -x --timeout 120 --timeout-method thread")
              steps+=("300|$out/wino5_bench|python -u tools/conv_bench_f32.py --shape 32,56,56,64,64,3,1,1,0 --shape 32,28,28,128,128,3,1,1,0 --shape 32,14,14,256,256,3,1,1,0 --shape 32,7,7,512,512,3,1,1,0 --only 118,119,150,151,152,153 --ks 1,-2,-4") ;;
    wino6)    steps+=("200|$out/pytest_wino|python -u -m pytest tests/test_wino_gpu.py -v -x --timeout 120 --timeout-method thread")
              for rep in a b; do steps+=("300|$out/wino6_bench_$rep|python -u tools/conv_bench_f32.py --shape 32,56,56,64,64,3,1,1,0 --shape 32,28,28,128,128,3,1,1,0 --shape 32,14,14,256,256,3,1,1,0 --shape 32,7,7,512,512,3,1,1,0 --only 118,154,155,156 --ks 1,-2,-4"); done ;;
    wtl)      for spec in "32,56,56,64,64:118:1" "32,56,56,64,64:170:1" "32,28,28,128,128:170:1" "32,14,14,256,256:170:-2" "32,7,7,512,512:170:-4"; do
                IFS=':' read -r shp cfg ks <<< "$spec"
                steps+=("120|$out/wtl_${cfg}_${shp//,/x}|python -u tools/wino_timeline.py --shape $shp --cfg $cfg --ks $ks --json gpurun_out/$out/wtl_${cfg}_${shp//,/x}.json")
              done ;;
    skp)      steps+=("120|$out/sk_probe|python -u tools/debug/sk_probe.py 2,56,56,64,64 110,157,158")
              steps+=("200|$out/pytest_wino|python -u -m pytest tests/test_wino_gpu.py -v --timeout 120 --timeout-method thread")
              steps+=("300|$out/wino_sk_bench|python -u tools/conv_bench_f32.py --shape 32,28,28,128,128,3,1,1,0 --shape 32,14,14,256,256,3,1,1,0 --shape 32,7,7,512,512,3,1,1,0 --only 118,155,157,158 --ks 1,-2,-4,-101,-102") ;;
    wino7)    steps+=("200|$out/pytest_wino|python -u -m pytest tests/test_wino_gpu.py -v -x --timeout 120 --timeout-method thread")
              for rep in a b; do steps+=("300|$out/wino7_bench_$rep|python -u tools/conv_bench_f32.py --shape 32,56,56,64,64,3,1,1,0 --shape 32,28,28,128,128,3,1,1,0 --shape 32,14,14,256,256,3,1,1,0 --shape 32,7,7,512,512,3,1,1,0 --only 118,155,160,161 --ks 1,-2,-4"); done ;;
    pw5)      steps+=("200|$out/pytest_pw|python -u -m pytest tests/test_pw_f32_gpu.py -v -x --timeout 120 --timeout-method thread")
              steps+=("300|$out/pw5_bench|python -u tools/conv_bench_f32.py --only 18,20,38,120,122,123,124 --ks 1,-1,-2 --shape 32,28,28,512,128,1,1,0,0 --shape 32,14,14,256,1024,1,1,0,1 --shape 32,14,14,1024,256,1,1,0,0 --shape 32,7,7,512,2048,1,1,0,1 --shape 32,7,7,2048,512,1,1,0,0 --shape 32,28,28,512,1280,1,2,0,0 --shape 32,14,14,1024,2560,1,2,0,0") ;;
    pw6)      steps+=("200|$out/pytest_pw|python -u -m pytest tests/test_pw_f32_gpu.py -v -x --timeout 120 --timeout-method thread")
              for rep in a b; do steps+=("300|$out/pw6_bench_$rep|python -u tools/conv_bench_f32.py --only 18,38,122,123,124,125,126 --ks 1,-2 --shape 32,28,28,512,128,1,1,0,0 --shape 32,28,28,128,512,1,1,0,1 --shape 32,14,14,256,1024,1,1,0,1 --shape 32,14,14,1024,256,1,1,0,0 --shape 32,56,56,64,256,1,1,0,1 --shape 32,56,56,256,64,1,1,0,0"); done ;;
    pwtl)     steps+=("200|$out/pytest_pw|python -u -m pytest tests/test_pw_f32_gpu.py -v -x --timeout 120 --timeout-method thread")
              steps+=("300|$out/pw_bench|python -u tools/conv_bench_f32.py --only 18,38,122,123,124,125,126 --ks 1,-2 --shape 32,28,28,512,128,1,1,0,0 --shape 32,14,14,256,1024,1,1,0,1 --shape 32,56,56,256,64,1,1,0,0 --shape 32,28,28,128,512,1,1,0,1 --shape 32,56,56,64,256,1,1,0,1 --shape 32,14,14,1024,256,1,1,0,0 --shape 32,7,7,512,2048,1,1,0,1")
              for spec in "32,28,28,512,128:123" "32,14,14,256,1024:123" "32,56,56,256,64:123" "32,28,28,512,128:126" "32,14,14,256,1024:126"; do
                IFS=':' read -r shp cfg <<< "$spec"
                steps+=("120|$out/pwtl_${cfg}_${shp//,/x}|python -u tools/pw_timeline.py --shape $shp --cfg $cfg --json gpurun_out/$out/pwtl_${cfg}_${shp//,/x}.json")
              done ;;
    wino8)    steps+=("200|$out/pytest_wino|python -u -m pytest tests/test_wino_gpu.py -v -x --timeout 120 --timeout-method thread")
              for rep in a b; do steps+=("300|$out/wino8_bench_$rep|python -u tools/conv_bench_f32.py --shape 32,56,56,64,64,3,1,1,0 --shape 32,28,28,128,128,3,1,1,0 --shape 32,14,14,256,256,3,1,1,0 --shape 32,7,7,512,512,3,1,1,0 --only 116,117,118,155,162,163,164,165,166,167 --ks 1,-2,-4"); done ;;
    wino9)    steps+=("200|$out/pytest_wino|python -u -m pytest tests/test_wino_gpu.py -v -x --timeout 120 --timeout-method thread")
              for rep in a b; do steps+=("300|$out/wino9_bench_$rep|python -u tools/conv_bench_f32.py --shape 32,56,56,64,64,3,1,1,0 --shape 32,28,28,128,128,3,1,1,0 --shape 32,14,14,256,256,3,1,1,0 --shape 32,7,7,512,512,3,1,1,0 --only 118,155,167,171 --ks 1,-2,-4"); done
              for spec in "32,56,56,64,64:170:1" "32,56,56,64,64:172:1" "32,28,28,128,128:170:1" "32,28,28,128,128:172:1" "32,14,14,256,256:172:-2"; do
                IFS=':' read -r shp cfg ks <<< "$spec"
                steps+=("120|$out/wtl_${cfg}_${shp//,/x}|python -u tools/wino_timeline.py --shape $shp --cfg $cfg --ks $ks")
              done ;;
    pmcstem)  steps+=("120|$out/pmcstem1|cd /tmp && rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/$out/pmcstem/g1 -o run -- python3 \$GRAFT_REPO_ROOT/tools/stem_bench.py --iters 20")
              steps+=("120|$out/pmcstem2|cd /tmp && rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/$out/pmcstem/g2 -o run -- python3 \$GRAFT_REPO_ROOT/tools/stem_bench.py --iters 20") ;;
    *) echo "unknown preset $p"; exit 2 ;;
  esac
done
[ -n "$GPU_EXTRA" ] && steps+=("$GPU_EXTRA")
exec bash tools/gpu_steps.sh "${steps[@]}"
