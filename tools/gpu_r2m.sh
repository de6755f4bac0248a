#!/bin/bash
# Round-2 GPU pass m: roofline counters (two PMC passes), the GPU test suite, smoke.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r2m
mkdir -p $O/roof
R="$PWD"
C1="TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA"
C2="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE TCC_HIT_sum TCC_MISS_sum"
bash tools/gpu_steps.sh \
  "180|r2m/roof_meta|python -u tools/roofline_r50.py --run --meta $O/roof/meta.json" \
  "90|r2m/pmc1|cd /tmp && rocprofv3 --pmc $C1 --output-format csv -d $R/$O/roof/g1 -o run -- python3 $R/tools/roofline_r50.py --run" \
  "90|r2m/pmc2|cd /tmp && rocprofv3 --pmc $C2 --output-format csv -d $R/$O/roof/g2 -o run -- python3 $R/tools/roofline_r50.py --run" \
  "900|r2m/pytest_gpu|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "120|r2m/smoke|python -u -c 'import __graft_entry__ as g; g.smoke()'"
