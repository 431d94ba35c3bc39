# Round 6: closing check on the final tree -- the default bench line (live replay trace), smoke, and the
# driver's exact -m gpu command line
mkdir -p gpurun_out
T=${TAG:-r06final}
timeout -k 10 400 python bench.py > gpurun_out/${T}_bench_default.json 2> gpurun_out/${T}_bench_default.err || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 || exit 1
timeout -k 10 900 python3 -m pytest tests/ -x -q -m gpu -p no:cacheprovider > gpurun_out/${T}_gpu_suite.log 2>&1
rc=$?; echo "suite rc=$rc" >> gpurun_out/${T}_gpu_suite.log; tail -3 gpurun_out/${T}_gpu_suite.log
exit $rc
