# Round 3: counters of the L1 3x3 weight gradient (row-tile LDS-DMA kernel + its reduction).
mkdir -p gpurun_out/pmc_wgrad
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pmc_wgrad/t -o run -- python3 $R/tools/wgrad_one.py > $R/gpurun_out/pmc_wgrad/t.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $R/gpurun_out/pmc_wgrad/p -o run -- python3 $R/tools/wgrad_one.py > $R/gpurun_out/pmc_wgrad/p.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_INSTS_SMEM -d $R/gpurun_out/pmc_wgrad/q -o run -- python3 $R/tools/wgrad_one.py > $R/gpurun_out/pmc_wgrad/q.log 2>&1 || exit 1
echo pmc wgrad done
