# Stall / pipe counters of the implicit-GEMM conv kernel on one shape (two SQ passes each)
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for spec in "112 128 2 9 128 14" "28 512 2 9 512 14" "224 64 2 9 64 0"; do
  tag=$(echo $spec | tr ' ' '_')
  rm -rf $R/gpurun_out/pg1_$tag $R/gpurun_out/pg2_$tag
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/pg1_$tag -o run -- python3 $R/tools/one_gemm.py $spec 5 > $R/gpurun_out/pg1_$tag.log 2>&1
  timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d $R/gpurun_out/pg2_$tag -o run -- python3 $R/tools/one_gemm.py $spec 5 > $R/gpurun_out/pg2_$tag.log 2>&1
done
