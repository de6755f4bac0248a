#!/bin/bash
# Two PMC passes (rocprofv3 --pmc, csv) over any python tool; run on the GPU box.
#   tools/pmc_run.sh <outdir> <python script> [args...]
out="$1"; shift
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$root/$out"; cd /tmp && export TMPDIR=/tmp
set -e
script="$1"; shift
timeout -k 10 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
  --output-format csv -d "$root/$out/p1" -o run -- python3 "$root/$script" "$@"
timeout -k 10 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_WAVES \
  --output-format csv -d "$root/$out/p2" -o run -- python3 "$root/$script" "$@"
