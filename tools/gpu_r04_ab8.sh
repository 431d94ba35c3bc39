# Block/model tests with the deferred input-side weight gradients, then its env A/B.
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
DFCSA_DEFER_WGRAD=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_parity2.py tests/test_gpu_trainer.py -k "block or model or cfg2 or trainer" > gpurun_out/t_ab8.log 2>&1 || { tail -30 gpurun_out/t_ab8.log; exit 1; }
tail -1 gpurun_out/t_ab8.log
bash tools/gpu_ab_envs.sh "base:X=0" "defer:DFCSA_DEFER_WGRAD=1"
