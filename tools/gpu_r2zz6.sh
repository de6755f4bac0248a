#!/bin/bash
# Round-2 GPU pass zz6: per-layer roofline counters of the final plan (two PMC passes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r2zz6
mkdir -p $O/roof
R="$PWD"
C1="TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA"
C2="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE TCC_HIT_sum TCC_MISS_sum"
bash tools/gpu_steps.sh \
  "180|r2zz6/roof_meta|python -u tools/roofline_r50.py --run --meta $O/roof/meta.json" \
  "90|r2zz6/pmc1|cd /tmp && timeout -s KILL 80 rocprofv3 --pmc $C1 --output-format csv -d $R/$O/roof/g1 -o run -- python3 $R/tools/roofline_r50.py --run" \
  "90|r2zz6/pmc2|cd /tmp && timeout -s KILL 80 rocprofv3 --pmc $C2 --output-format csv -d $R/$O/roof/g2 -o run -- python3 $R/tools/roofline_r50.py --run"
