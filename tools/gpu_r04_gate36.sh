# Knob 36 (fused gate dgrad grid: column blocks share the resident slots): correctness with the knob
# on, then a per-kernel trace A/B and a same-box step A/B.
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd $R
DFCSA_TUNE=36=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py tests/test_gpu_fused_ref.py -k "gate or acc_relu or fused" > gpurun_out/g36_tests.log 2>&1 || { tail -30 gpurun_out/g36_tests.log; exit 1; }
tail -2 gpurun_out/g36_tests.log
bash tools/gpu_ab_knob_ktrace.sh 36=1 || exit 1
cd $R
python3 tools/kt_compare.py gpurun_out/kt_A/*/run_results.db gpurun_out/kt_B/*/run_results.db 25 > gpurun_out/g36_ktc.txt 2>&1 || python3 tools/kt_compare.py gpurun_out/kt_A/run_results.db gpurun_out/kt_B/run_results.db 25 > gpurun_out/g36_ktc.txt 2>&1
bash tools/gpu_ab_envs.sh "base:DFCSA_X=0" "g36:DFCSA_TUNE=36=1"
