# Model/block tests, then the per-kernel trace A/B (tools/gpu_ab_ktrace.sh) of the working tree against _ab_base/.
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_parity2.py tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -k "model or block or cfg2 or first_layer or streaming or dgrad or gate or apply or lsa" > gpurun_out/pk_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/pk_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_ktrace.sh
