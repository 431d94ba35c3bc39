# The fused local/attention gate forward at C = 128: its kernel test, block/model tests, then an env A/B.
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fused_ref.py -k "local_attn_gate" > gpurun_out/t_ab10a.log 2>&1 || { tail -40 gpurun_out/t_ab10a.log; exit 1; }
tail -1 gpurun_out/t_ab10a.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_parity2.py -k "block or model or cfg2 or cfg3" > gpurun_out/t_ab10b.log 2>&1 || { tail -30 gpurun_out/t_ab10b.log; exit 1; }
tail -1 gpurun_out/t_ab10b.log
bash tools/gpu_ab_envs.sh "base:X=0" "la64:DFCSA_LOCAL_ATTN_WIDTHS=64"
