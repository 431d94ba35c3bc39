set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_small_gemm.py -x -q --timeout 100 --timeout-method thread > gpurun_out/sg_tests.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
AB_BASE_ENV=DFCSA_SIDE_STREAM=0 AB_NEW_ENV=DFCSA_SIDE_STREAM=0 bash tools/gpu_ab_tree.sh
