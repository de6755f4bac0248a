set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6ah
for c in 1 2 4; do
  timeout -k 10 240 python tools/ab_cfg.py --precision fp32 --rounds 21 --env-b "ADAPT_W4S_CPT=$c" > gpurun_out/r6ah/ab_cpt$c.log 2>&1 || exit $?
done
