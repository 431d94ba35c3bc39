mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q --timeout 100 --timeout-method thread -k "big_tiles" > gpurun_out/wgbig_test.log 2>&1 || exit 1
WGRAD_MODES=default,big1,big1_t256,big1_t1024,big2,big2_t256,big3,big3_t256,big1_f16 timeout -k 10 400 python -u tools/wgrad_shapes.py > gpurun_out/wgbig_shapes.jsonl 2>&1
