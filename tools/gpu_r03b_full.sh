# Full evidence on the current build: -m gpu suite, smoke, default bench (with CPU leg), kernel
# trace + stats, FETCH/WRITE/SQ passes (tools/gpu_profile_r03.sh), per-launch shape table.
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rs --timeout 240 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "gpu_tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_profile_r03.sh || exit 1
cd $R
DB=$(ls gpurun_out/p_trace/*/run_results.db gpurun_out/p_trace/run_results.db 2>/dev/null | head -1)
python3 tools/step_kernels.py $DB 80 > gpurun_out/step_kernels.txt 2>&1
cat gpurun_out/bench_default.json
