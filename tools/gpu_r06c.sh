# Round 6: pooled-attention diagnostics (GEMM-path cause; flash vs per-row at model level), the flash
# tests, and the driver's -m gpu command line.
mkdir -p gpurun_out
: > gpurun_out/r06c_diag.log
for v in "USE_F=bmm USE_B=row" "USE_F=row USE_B=bmm" "FLASH=1 FLASH_MIN_N=100000 SAVE=/tmp/g_row.pt" "FLASH=1 SAVE=/tmp/g_fl.pt CMP=/tmp/g_row.pt"; do
  env $v timeout -k 10 150 python -u tools/lsa_bmm_diag.py >> gpurun_out/r06c_diag.log 2>&1 || { rc=$?; echo "diag rc=$rc" >> gpurun_out/r06c_diag.log; exit $rc; }
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_lsa_flash.py tests/test_gpu_qk_ratio.py "tests/test_gpu_kernels.py::test_wgrad_cooperative_reduction" -q -p no:cacheprovider > gpurun_out/r06c_flash.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r06c_flash.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python3 -m pytest tests/ -q -m gpu -p no:cacheprovider > gpurun_out/r06c_suite.log 2>&1
rc=$?; echo "suite rc=$rc" >> gpurun_out/r06c_suite.log
exit $rc
