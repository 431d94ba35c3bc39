mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
echo "tests rc=$?"
