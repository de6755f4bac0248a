set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6w
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_codec_wire_gpu.py tests/test_pipeline_codec_gpu.py tests/test_kernels_gpu.py tests/test_gemm_f32s_gpu.py > gpurun_out/r6w/pytest.log 2>&1 &&
timeout -k 10 400 python tools/codec_bench.py --json gpurun_out/r6w/codec.json > gpurun_out/r6w/codec.log 2>&1 &&
bash tools/gpu_r6u.sh
