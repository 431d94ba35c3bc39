# Model tests with the last block's early conv1 weight gradient, then its env A/B.
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
DFCSA_LAST_EARLY=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_parity2.py -k "model or cfg2" > gpurun_out/t_ab9.log 2>&1 || { tail -30 gpurun_out/t_ab9.log; exit 1; }
tail -1 gpurun_out/t_ab9.log
bash tools/gpu_ab_envs.sh "base:X=0" "lastearly:DFCSA_LAST_EARLY=1" "lastearly2:DFCSA_LAST_EARLY=2"
