# Full -m gpu suite, then a kernel trace of the default bench step (tools/kt_classes.py,
# tools/kt_launch_compare.py read gpurun_out/kt_S/*/run_results.db).  Test failures (rc 1) do not stop
# the trace; any other non-zero status ends the script.
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r04_suite.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/r04_suite.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/kt_S
B="--steps 20 --warmup 5 --no-cpu-baseline --no-val-dice --no-trainer-faithful --no-kernel-timing"
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/kt_S -o run -- python3 $R/bench.py $B > $R/gpurun_out/kt_S.log 2>&1 || exit 1
grep '"value"' $R/gpurun_out/kt_S.log | head -c 300
