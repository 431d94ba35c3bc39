# A/B of tuning knobs on the bench (same box): gpu_r03b_ab.sh "<label>=<DFCSA_TUNE value>" ...
# plus an optional test selection in $TESTS run first.
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd $R
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q -rs --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/ab_tests.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
B="--no-cpu-baseline --no-val-dice --no-trainer-faithful"
for rep in 1 2; do
  for kv in "$@"; do
    lab=${kv%%=*}; tune=${kv#*=}
    DFCSA_TUNE=$tune timeout -k 10 300 python bench.py $B > gpurun_out/ab_${lab}_$rep.json 2> gpurun_out/ab_${lab}_$rep.err || { echo "bench $lab failed"; exit 1; }
    python3 -c "import json,sys;d=json.load(open('gpurun_out/ab_${lab}_$rep.json'));print('$lab', $rep, d['value'], d['ms_per_step'])"
  done
done
