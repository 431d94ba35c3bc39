# Round 6: max-pool argmax flips between the per-row and the flash pooled attention (P = 16, B = 2),
# the flash-path error budget, the standalone odd-width tests
mkdir -p gpurun_out
: > gpurun_out/r06e_diag.log
for v in "TIES=1 FLASH=1 FLASH_MIN_N=100000 SAVE=/tmp/g_row.pt" "TIES=1 FLASH=1 SAVE=/tmp/g_fl.pt CMP=/tmp/g_row.pt"; do
  env $v timeout -k 10 150 python -u tools/lsa_bmm_diag.py >> gpurun_out/r06e_diag.log 2>&1 || { rc=$?; echo "diag rc=$rc" >> gpurun_out/r06e_diag.log; exit $rc; }
done
: > gpurun_out/r06e_err.log
for a in "64 16 28 2 2" "64 16 28 2 1" "256 32 14 2 2" "1024 32 14 1 2" "512 16 7 2 2"; do
  timeout -k 10 120 python -u tools/lsa_flash_err.py $a >> gpurun_out/r06e_err.log 2>&1 || { rc=$?; echo "err rc=$rc" >> gpurun_out/r06e_err.log; exit $rc; }
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_oddwidth.py tests/test_gpu_model.py::test_lsa_fp32 -q -p no:cacheprovider > gpurun_out/r06e_odd.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r06e_odd.log
exit $rc
