# Round 6: config 5 A/B of the in-tree library against ab_lib/libdfcsa_base.so (DFCSA_LIB), three rounds
mkdir -p gpurun_out
T=${TAG:-r06c5b}
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -q -p no:cacheprovider > gpurun_out/${T}_targeted.log 2>&1
  rc=$?; echo "targeted rc=$rc" >> gpurun_out/${T}_targeted.log; tail -3 gpurun_out/${T}_targeted.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
S="--no-cpu-baseline --no-val-dice --no-trainer-faithful --no-live-trace --model fullres --img 512 --batch 2 --steps 4 --warmup 2"
: > gpurun_out/${T}_ab.txt
for round in 1 2 3; do
  for v in new base; do
    if [ $v = new ]; then L=X=0; else L=DFCSA_LIB=$GRAFT_REPO_ROOT/ab_lib/libdfcsa_base.so; fi
    out=$(env $L timeout -k 10 300 python bench.py $S 2>> gpurun_out/${T}_ab.err) || exit 1
    echo "$round $v cfg5 $(echo "$out" | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"])')" >> gpurun_out/${T}_ab.txt
  done
done
cat gpurun_out/${T}_ab.txt
