# Round 3: the whole -m gpu suite on the current build, then the profile set (tools/gpu_profile_r03.sh).
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rs --timeout 240 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "gpu_tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_profile_r03.sh
