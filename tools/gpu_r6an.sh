set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6an
AB="timeout -k 10 240 python tools/ab_cfg.py --precision fp32 --rounds 15"
$AB --set "32x7x7x512,3x3s1p1111@221@4" > gpurun_out/r6an/ab_s5_221_4.log 2>&1 &&
$AB --set "32x56x56x64,3x3s1p1111@223@1" > gpurun_out/r6an/ab_s2_223_1.log 2>&1 &&
$AB --set "32x56x56x64,3x3s1p1111@228@1" > gpurun_out/r6an/ab_s2_228_1.log 2>&1 &&
$AB --set "32x14x14x256,3x3s1p1111@227@4" > gpurun_out/r6an/ab_s4_227_4.log 2>&1
