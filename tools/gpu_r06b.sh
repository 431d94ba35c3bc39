# Round 6: the pooled-attention flash path's tests + the round-5 GEMM-path diagnostic, then the
# whole -m gpu suite with the driver's exact command line.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_lsa_flash.py tests/test_gpu_model.py::test_lsa_fp32 tests/test_gpu_qk_ratio.py -q -p no:cacheprovider > gpurun_out/r06b_flash.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r06b_flash.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for v in "USE=row" "USE=bmm" "USE=bmm SYNC=1"; do
  env $v timeout -k 10 150 python -u tools/lsa_bmm_diag.py >> gpurun_out/r06b_diag.log 2>&1 || { rc=$?; echo "diag rc=$rc" >> gpurun_out/r06b_diag.log; exit $rc; }
done
timeout -k 10 900 python3 -m pytest tests/ -x -q -m gpu -p no:cacheprovider > gpurun_out/r06b_suite.log 2>&1
rc=$?; echo "suite rc=$rc" >> gpurun_out/r06b_suite.log
exit $rc
