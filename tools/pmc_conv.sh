#!/bin/bash
# PMC counters for the conv kernels on one ResNet-50 problem (run on the GPU box).
#   tools/pmc_conv.sh "<shape>" "<cfgs>" <outdir>
shape="${1:-32,28,28,128,128,3,1,1}"; cfgs="${2:-6,2}"; out="${3:-gpurun_out/pmc}"
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$root/$out"; cd /tmp && export TMPDIR=/tmp
set -e
timeout -k 10 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
  --output-format csv -d "$root/$out/p1" -o run -- python3 "$root/tools/conv_bench.py" --shape "$shape" --only "$cfgs"
timeout -k 10 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE \
  --output-format csv -d "$root/$out/p2" -o run -- python3 "$root/tools/conv_bench.py" --shape "$shape" --only "$cfgs"
