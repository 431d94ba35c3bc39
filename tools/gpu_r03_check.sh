# Round-3 checks on one box.  Each GPU step has its own time limit; a test FAILURE (rc 1) lets the
# next step run, a crash / fault / time-out (any other non-zero rc) ends the script there.
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd $R
step() {  # step <name> <timeout> <cmd...>
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step halo_tests 300 python -u -m pytest tests/test_gpu_halo.py -v -rs --timeout 120 --timeout-method thread
step gpu_tests_nohalo 900 env DFCSA_TUNE=19=0 python -u -m pytest tests -m gpu -q -rs --timeout 240 --timeout-method thread
step gpu_tests 900 python -u -m pytest tests -m gpu -q -rs --timeout 240 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
timeout -k 10 400 env DFCSA_TUNE=19=0 python bench.py --no-cpu-baseline > gpurun_out/bench_nohalo.json 2> gpurun_out/bench_nohalo.err; echo "bench_nohalo rc=$?"
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err; echo "bench rc=$?"
