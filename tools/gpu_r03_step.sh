# Round-3: whole -m gpu suite, smoke, bench line and a kernel-trace profile of the bench on one box.
# A test FAILURE (rc 1) lets the next step run; a crash / fault / time-out ends the script there.
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
step gpu_tests 900 python -u -m pytest tests -m gpu -q -rs --timeout 240 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 400 python bench.py --no-cpu-baseline
export TMPDIR=/tmp
step prof 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_step -o run -- python3 bench.py --no-cpu-baseline --steps 10 --warmup 5
echo done
