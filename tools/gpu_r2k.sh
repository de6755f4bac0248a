#!/bin/bash
# Round-2 GPU pass k: planner calibration refresh for the fused plan, plan check,
# per-layer roofline counters (two PMC passes), kernel-trace stats of the bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r2k
mkdir -p $O/roof
R="$PWD"
C1="TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA"
C2="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE TCC_HIT_sum TCC_MISS_sum"
bash tools/gpu_steps.sh \
  "240|r2k/calib|python -u tools/profile_r50.py --batch 32 --calib --json $O/r50_bs32_steps.json && cp adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd/tuning/gfx950_layer_costs.json $O/" \
  "300|r2k/plan_check|python -u tools/plan_check.py --stages 2,4,8 --json $O/plan_check.json" \
  "180|r2k/roof_meta|python -u tools/roofline_r50.py --run --meta $O/roof/meta.json" \
  "60|r2k/list|rocprofv3 -L > $O/counters_list.txt 2>&1" \
  "90|r2k/pmc1|cd /tmp && rocprofv3 --pmc $C1 --output-format csv -d $R/$O/roof/g1 -o run -- python3 $R/tools/roofline_r50.py --run" \
  "90|r2k/pmc2|cd /tmp && rocprofv3 --pmc $C2 --output-format csv -d $R/$O/roof/g2 -o run -- python3 $R/tools/roofline_r50.py --run" \
  "120|r2k/trace|cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace -o bench -- python3 $R/bench.py --steps 50 --warmup 10"
