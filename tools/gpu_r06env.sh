# Round 6: the default bench step under the remaining opt-in switches, interleaved, three rounds
mkdir -p gpurun_out
T=${TAG:-r06env}
S="--no-cpu-baseline --no-val-dice --no-trainer-faithful --no-live-trace --steps 40 --warmup 5"
: > gpurun_out/${T}_ab.txt
for round in 1 2 3; do
  for v in "X=0" "DFCSA_SPLIT_DX=1" "DFCSA_DEFER_WGRAD=1" "DFCSA_LSA_CORE_BWD=1"; do
    out=$(env $v timeout -k 10 300 python bench.py $S 2>> gpurun_out/${T}_ab.err) || exit 1
    echo "$round $v $(echo "$out" | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> gpurun_out/${T}_ab.txt
  done
done
cat gpurun_out/${T}_ab.txt
