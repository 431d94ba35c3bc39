mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity2.py -m gpu -q --timeout 200 --timeout-method thread -k "maxpool or rccl" > gpurun_out/rccl_test.log 2>&1
echo "rccl test rc=$?"
timeout -k 10 300 python -u tools/step_breakdown.py > gpurun_out/step_breakdown.log 2>&1
