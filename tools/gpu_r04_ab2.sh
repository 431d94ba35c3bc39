# Tests of the changed block path, the tree A/B against _ab_prev/, then an env A/B of the weight-gradient
# workgroup target (knob 2).
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_model.py -k "entry_window or block or model" > gpurun_out/t_ab.log 2>&1 || { tail -30 gpurun_out/t_ab.log; exit 1; }
tail -1 gpurun_out/t_ab.log
bash tools/gpu_ab_tree3.sh || exit 1
bash tools/gpu_ab_envs.sh "base:X=0" "t256:DFCSA_TUNE=2=256" "t128:DFCSA_TUNE=2=128"
