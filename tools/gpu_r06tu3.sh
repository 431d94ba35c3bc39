# Round 6: TransUNet bf16 step under the side stream for its weight gradients and the split-K knobs
mkdir -p gpurun_out
T=${TAG:-r06tu3}
S="--no-cpu-baseline --no-val-dice --no-trainer-faithful --no-live-trace --model transunet --batch 8 --steps 20 --warmup 3 --precision bf16"
: > gpurun_out/${T}_ab.txt
for round in 1 2; do
  for v in "X=0" "DFCSA_SIDE_STREAM_TU=1" "DFCSA_TUNE=37=12" "DFCSA_TUNE=38=1200"; do
    out=$(env $v timeout -k 10 300 python bench.py $S 2>> gpurun_out/${T}_ab.err) || exit 1
    echo "$round $v $(echo "$out" | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> gpurun_out/${T}_ab.txt
  done
done
cat gpurun_out/${T}_ab.txt
