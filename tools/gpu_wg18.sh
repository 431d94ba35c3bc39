mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x --timeout 100 --timeout-method thread -k "wide_tile" > gpurun_out/wg18_test.log 2>&1 || { tail -20 gpurun_out/wg18_test.log; exit 1; }
tail -1 gpurun_out/wg18_test.log
WGRAD_MODES=default,wide192,t1024,t256 timeout -k 10 300 python -u tools/wgrad_shapes.py > gpurun_out/wg18_shapes.jsonl 2>&1
