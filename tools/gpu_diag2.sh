mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x --timeout 200 --timeout-method thread -k "dgrad_gate" > gpurun_out/diag_tests.log 2>&1
echo "tests rc=$?"; tail -5 gpurun_out/diag_tests.log
AMD_SERIALIZE_KERNEL=3 DFCSA_DEBUG=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-graph --no-cpu-baseline --no-val-dice --no-trainer-faithful --no-kernel-timing > gpurun_out/diag_bench.json 2> gpurun_out/diag_bench.err
echo "bench rc=$?"
