# Tests of the attention kernels and the block path, the tree A/B against _ab_prev/, then env A/Bs
# (knob 35: column-kernel threads; knob 2: weight-gradient workgroup target).
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "lsa" > gpurun_out/t_ab3a.log 2>&1 || { tail -30 gpurun_out/t_ab3a.log; exit 1; }
tail -1 gpurun_out/t_ab3a.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_parity2.py -k "not rccl and not bench_ddp" > gpurun_out/t_ab3b.log 2>&1 || { tail -30 gpurun_out/t_ab3b.log; exit 1; }
tail -1 gpurun_out/t_ab3b.log
bash tools/gpu_ab_tree3.sh || exit 1
bash tools/gpu_ab_envs.sh "base:X=0" "cols256:DFCSA_TUNE=35=256" "t768:DFCSA_TUNE=2=768"
