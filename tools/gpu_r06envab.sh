# Round 6: targeted tests, then a same-box A/B of the default against one environment setting (ENVOFF,
# e.g. DFCSA_LSA_DP16=0) at the pool sizes in POOLS (default 8 16 32), two rounds
mkdir -p gpurun_out
T=${TAG:-r06env2}
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -q -p no:cacheprovider > gpurun_out/${T}_targeted.log 2>&1
  rc=$?; echo "targeted rc=$rc" >> gpurun_out/${T}_targeted.log; tail -3 gpurun_out/${T}_targeted.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
S="--no-cpu-baseline --no-val-dice --no-trainer-faithful --no-live-trace --steps 40 --warmup 5"
: > gpurun_out/${T}_ab.txt
for round in 1 2; do
  for v in "X=0" "${ENVOFF}"; do
    for p in ${POOLS:-8 16 32}; do
      out=$(env $v timeout -k 10 300 python bench.py --pool $p $S 2>> gpurun_out/${T}_ab.err) || exit 1
      echo "$round $v P=$p $(echo "$out" | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> gpurun_out/${T}_ab.txt
    done
  done
done
cat gpurun_out/${T}_ab.txt
