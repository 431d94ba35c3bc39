mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_parity2.py -k "lsa or model or block or cfg2 or step" -x -q -rs --timeout 200 --timeout-method thread > gpurun_out/lsa_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/lsa_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_ab_envs.sh "fused:DFCSA_LSA_CORE_BWD=1" "three:DFCSA_LSA_CORE_BWD=0"
