# Block/model/parity tests and the pack test, then the tree A/B against _ab_prev/ and an env A/B of the
# split block-input gradient (DFCSA_SPLIT_DX).
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "pack or lsa" > gpurun_out/t_ab4a.log 2>&1 || { tail -30 gpurun_out/t_ab4a.log; exit 1; }
tail -1 gpurun_out/t_ab4a.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_parity2.py tests/test_gpu_trainer.py tests/test_gpu_zoo.py -k "not rccl and not bench_ddp" > gpurun_out/t_ab4b.log 2>&1 || { tail -30 gpurun_out/t_ab4b.log; exit 1; }
tail -1 gpurun_out/t_ab4b.log
bash tools/gpu_ab_tree3.sh || exit 1
bash tools/gpu_ab_envs.sh "base:X=0" "nosplit:DFCSA_SPLIT_DX=0"
