# Env A/B of the forward's attention-entry conv placement (DFCSA_ENTRY_ON_BRANCH_HW).
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
DFCSA_ENTRY_ON_BRANCH_HW=3136 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_model.py -k "block or model" > gpurun_out/t_ab7.log 2>&1 || { tail -30 gpurun_out/t_ab7.log; exit 1; }
tail -1 gpurun_out/t_ab7.log
bash tools/gpu_ab_envs.sh "base:X=0" "hw3136:DFCSA_ENTRY_ON_BRANCH_HW=3136" "hw12544:DFCSA_ENTRY_ON_BRANCH_HW=12544" "hw784:DFCSA_ENTRY_ON_BRANCH_HW=784"
