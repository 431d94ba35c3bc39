# Round 6: TransUNet bf16 step under weight-gradient reduction settings (knob 13: most splits reduced
# in-kernel; knob 2: workgroups per weight-gradient launch)
mkdir -p gpurun_out
T=${TAG:-r06tu2}
S="--no-cpu-baseline --no-val-dice --no-trainer-faithful --no-live-trace --model transunet --batch 8 --steps 20 --warmup 3 --precision bf16"
: > gpurun_out/${T}_ab.txt
for round in 1 2; do
  for v in "X=0" "DFCSA_TUNE=13=8" "DFCSA_TUNE=13=64" "DFCSA_TUNE=2=256" "DFCSA_TUNE=2=1024"; do
    out=$(env $v timeout -k 10 300 python bench.py $S 2>> gpurun_out/${T}_ab.err) || exit 1
    echo "$round $v $(echo "$out" | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> gpurun_out/${T}_ab.txt
  done
done
cat gpurun_out/${T}_ab.txt
