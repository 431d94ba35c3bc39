# Block/model tests with the late gate weight gradients, then an env A/B of DFCSA_WGRAD_LATE.
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
DFCSA_WGRAD_LATE=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_parity2.py -k "block or model or cfg2" > gpurun_out/t_ab5.log 2>&1 || { tail -30 gpurun_out/t_ab5.log; exit 1; }
tail -1 gpurun_out/t_ab5.log
bash tools/gpu_ab_envs.sh "base:X=0" "late:DFCSA_WGRAD_LATE=1"
