# Round-5 record: the whole -m gpu suite with the tests' printouts (-s: the bf16 step tests' per-tensor
# tables), then the smoke entry point.
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests/ -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/${TAG:-r05}_gpu_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
tail -3 gpurun_out/${TAG:-r05}_gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG:-r05}_smoke.log 2>&1 || exit 1
exit $rc
