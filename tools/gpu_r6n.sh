set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6n
AB="timeout -k 10 240 python tools/ab_cfg.py --precision fp32 --rounds 15"
$AB --set "32x56x56x64,3x3s1p1111@221@1" > gpurun_out/r6n/ab_s2_221_1.log 2>&1 &&
$AB --set "32x28x28x128,3x3s1p1111@221@1" > gpurun_out/r6n/ab_s3_221_1.log 2>&1 &&
$AB --set "32x28x28x128,3x3s1p1111@221@2" > gpurun_out/r6n/ab_s3_221_2.log 2>&1 &&
$AB --set "32x14x14x256,3x3s1p1111@221@2" > gpurun_out/r6n/ab_s4_221_2.log 2>&1 &&
$AB --set "32x7x7x512,3x3s1p1111@236@8" > gpurun_out/r6n/ab_s5_236_8.log 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_rccl_loopback_gpu.py -k hang -s > gpurun_out/r6n/pytest_loopback_hang.log 2>&1
