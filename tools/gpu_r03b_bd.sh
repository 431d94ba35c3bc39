mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -k "wgrad" -x -q -rs --timeout 120 --timeout-method thread > gpurun_out/bd_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/bd_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 500 python3 tools/wgrad_bench.py "warm:" "bd:26=1" "ptr:26=0" "bd2:26=1" > gpurun_out/wgb_bd.jsonl 2> gpurun_out/wgb_bd.err || exit 1
cat gpurun_out/wgb_bd.jsonl
bash tools/gpu_ab_envs.sh "bd:DFCSA_TUNE=26=1" "ptr:DFCSA_TUNE=26=0"
