set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6aa
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS --output-format csv -d $R/gpurun_out/r6aa/p1 -o run -- python3 $R/tools/stem_bench.py --iters 20 > $R/gpurun_out/r6aa/p1.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_INST_CYCLES_VMEM --output-format csv -d $R/gpurun_out/r6aa/p2 -o run -- python3 $R/tools/stem_bench.py --iters 20 > $R/gpurun_out/r6aa/p2.log 2>&1 &&
cd $R && python tools/pmc_kernels.py gpurun_out/r6aa stem_pool_f32 > gpurun_out/r6aa/summary.txt 2>&1; python tools/pmc_kernels.py gpurun_out/r6aa stem_hpool >> gpurun_out/r6aa/summary.txt 2>&1
