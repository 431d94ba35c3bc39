# Full -m gpu suite, then a same-box A/B of environment arms on the default bench (gpu_ab_envs.sh
# arguments).  Test failures (rc 1) do not stop the A/B; any other non-zero status ends the script.
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r04_suite.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/r04_suite.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_ab_envs.sh "$@"
