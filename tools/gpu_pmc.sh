set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for cfg in 14; do
rm -rf $R/gpurun_out/pmc_g$cfg $R/gpurun_out/pmc2_g$cfg
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc_g$cfg -o run --output-format csv -- python3 $R/tools/one_gemm.py 112 128 2 9 128 $cfg 5 > $R/gpurun_out/pmc_g$cfg.log 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS -d $R/gpurun_out/pmc2_g$cfg -o run --output-format csv -- python3 $R/tools/one_gemm.py 112 128 2 9 128 $cfg 5 > $R/gpurun_out/pmc2_g$cfg.log 2>&1
done
