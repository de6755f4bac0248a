#!/bin/bash
# PMC counters of one fp32 conv launch per pass (tools/conv_bench_f32.py, one shape x cfg x split each),
# run on the GPU box.
#   tools/pmc_f32.sh <outdir> "<B,H,W,C,N,k,stride,pad,res>:<cfg>:<ks>" ...
# Two counter groups per spec (MI355X one-pass limits); summarise with
#   python tools/pmc_summary.py <outdir>/<tag>
out="$1"; shift
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
set -e
for spec in "$@"; do
  IFS=':' read -r shp cfg ks <<< "$spec"
  IFS=',' read -r B H W C N K S P R <<< "$shp"
  tag="h${H}_c${C}_n${N}_k${K}s${S}_cfg${cfg}_ks${ks}"
  mkdir -p "$root/$out/$tag"
  timeout -s KILL 100 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
    --output-format csv -d "$root/$out/$tag/g1" -o run -- python3 "$root/tools/conv_bench_f32.py" --shape "$shp" --only "$cfg" --ks "$ks"
  timeout -s KILL 100 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS TCC_HIT_sum TCC_MISS_sum \
    --output-format csv -d "$root/$out/$tag/g2" -o run -- python3 "$root/tools/conv_bench_f32.py" --shape "$shp" --only "$cfg" --ks "$ks"
done
