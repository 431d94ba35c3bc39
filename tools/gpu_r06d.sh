# Round 6: uninitialised-read probe of the pooled-attention paths (every torch.empty poisoned with NaN)
mkdir -p gpurun_out
: > gpurun_out/r06d_diag.log
for v in "POISON=1 FLASH=1 FLASH_MIN_N=100000" "POISON=1 FLASH=1" "POISON=0 FLASH=1 FLASH_MIN_N=100000 B=3" "POISON=0 FLASH=1 B=3"; do
  echo "== $v" >> gpurun_out/r06d_diag.log
  env $v timeout -k 10 150 python -u tools/lsa_bmm_diag.py >> gpurun_out/r06d_diag.log 2>&1 || { rc=$?; echo "diag rc=$rc" >> gpurun_out/r06d_diag.log; exit $rc; }
done
