# Round 6: P = 16, B = 2 flash-path gradient deviation -- stream ordering vs memory reuse
mkdir -p gpurun_out
: > gpurun_out/r06f_diag.log
for v in "FLASH=1 DFCSA_SIDE_STREAM=0 DFCSA_BRANCH_STREAM=0" "FLASH=1 DFCSA_BRANCH_STREAM=0" "FLASH=1 DFCSA_SIDE_STREAM=0" "FLASH=1 PYTORCH_NO_CUDA_MEMORY_CACHING=1" "FLASH=1 FLASH_MIN_N=100000 PYTORCH_NO_CUDA_MEMORY_CACHING=1" "FLASH=1 AMD_SERIALIZE_KERNEL=3"; do
  echo "== $v" >> gpurun_out/r06f_diag.log
  env $v timeout -k 10 150 python -u tools/lsa_bmm_diag.py >> gpurun_out/r06f_diag.log 2>&1 || { rc=$?; echo "diag rc=$rc" >> gpurun_out/r06f_diag.log; exit $rc; }
done
