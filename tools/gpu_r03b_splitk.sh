mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_transunet.py -k "splitk or reduce_layouts or pair_layout3 or dropout" -x -q -rs --timeout 120 --timeout-method thread > gpurun_out/sk_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/sk_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
GEMM_SHAPES=BN,L4 GEMM_CHECK=1 timeout -k 10 300 python3 tools/gemm_bench.py 0,19,15,14 > gpurun_out/splitk_gemm.jsonl 2> gpurun_out/splitk_gemm.err || exit 1
cat gpurun_out/splitk_gemm.jsonl
timeout -k 10 900 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_parity2.py -x -q --timeout 240 --timeout-method thread > gpurun_out/sk_model.log 2>&1
rc=$?; echo "model rc=$rc"; tail -3 gpurun_out/sk_model.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_ab_envs.sh "new:DFCSA_TUNE=25=1" "nosplit:DFCSA_TUNE=25=0" "nopair:DFCSA_PAIR_WGRAD=0"
