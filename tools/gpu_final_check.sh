# final HEAD check: all GPU tests, smoke, default bench line (as the driver runs them)
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/final_tests.log 2>&1
echo "tests rc=$?"; tail -1 gpurun_out/final_tests.log
set -e
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1
tail -1 gpurun_out/final_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err
head -c 300 gpurun_out/final_bench.json
