# Quick round-4 check: the changed GPU tests, then the per-kernel trace A/B and the tree A/B against _ab_prev/.
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_model.py -k "entry_window or block or model" > gpurun_out/t_ab.log 2>&1 || { tail -30 gpurun_out/t_ab.log; exit 1; }
tail -1 gpurun_out/t_ab.log
AB_BASE=_ab_prev bash tools/gpu_ab_ktrace.sh || exit 1
cd $R && bash tools/gpu_ab_tree3.sh
