# same-box A/B of tuning knobs: default vs each DFCSA_TUNE setting in $KNOBS (space-separated), 2 runs each, interleaved
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT; cd $R
B="--no-cpu-baseline --no-val-dice --no-trainer-faithful"
: > gpurun_out/knob_ab.txt
for i in 1 2; do
  v=$(timeout -k 10 300 python bench.py $B 2>/dev/null | python -c "import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])['value'])") || exit 1
  echo "default $v" >> gpurun_out/knob_ab.txt
  for k in $KNOBS; do
    v=$(env $k timeout -k 10 300 python bench.py $B 2>/dev/null | python -c "import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])['value'])") || exit 1
    echo "$k $v" >> gpurun_out/knob_ab.txt
  done
done
cat gpurun_out/knob_ab.txt
