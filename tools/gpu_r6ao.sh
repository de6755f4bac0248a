set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6ao
bash tools/pmc_groups.sh gpurun_out/r6ao/pmc 'SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES' 'SQ_WAIT_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MFMA TCC_HIT_sum TCC_MISS_sum' -- bench.py --steps 3 --warmup 2 --no-bf16 > gpurun_out/r6ao/pmc.log 2>&1 &&
python tools/pmc_kernels.py gpurun_out/r6ao/pmc pw_stream > gpurun_out/r6ao/pw_stream_pmc.txt 2>&1 &&
python tools/pmc_kernels.py gpurun_out/r6ao/pmc wino4s > gpurun_out/r6ao/wino4s_pmc.txt 2>&1 &&
python tools/pmc_kernels.py gpurun_out/r6ao/pmc pair > gpurun_out/r6ao/pair_pmc.txt 2>&1
