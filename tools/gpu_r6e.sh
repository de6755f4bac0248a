set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6f/pmc
for spec in "56:221:1" "7:221:-8" "14:221:-4"; do
  IFS=':' read -r H cfg ks <<< "$spec"
  tag=h${H}_${cfg}_${ks}
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
    --output-format csv -d $R/gpurun_out/r6f/pmc/$tag/g1 -o run -- python3 $R/tools/wino4s_bench.py --cfgs $cfg --ks $ks --shapes $H --no-tuned --reps 5 || exit 1
  timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS TCC_HIT_sum TCC_MISS_sum \
    --output-format csv -d $R/gpurun_out/r6f/pmc/$tag/g2 -o run -- python3 $R/tools/wino4s_bench.py --cfgs $cfg --ks $ks --shapes $H --no-tuned --reps 5 || exit 1
done
