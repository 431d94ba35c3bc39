# Round 6: config 5 (full-resolution attention, 512^2) under the flash kernels' waves-per-SIMD budgets
# (knob 10 bits: 1 forward, 2 dK/dV, 4 dQ, 8 forward at 4 waves for C = 64; default 15)
mkdir -p gpurun_out
T=${TAG:-r06c5}
S="--no-cpu-baseline --no-val-dice --no-trainer-faithful --no-live-trace --model fullres --img 512 --batch 2 --steps 4 --warmup 2"
: > gpurun_out/${T}_ab.txt
for round in 1 2; do
  for v in "X=0" "DFCSA_TUNE=10=13" "DFCSA_TUNE=10=7" "DFCSA_TUNE=10=14" "DFCSA_TUNE=10=6"; do
    out=$(env $v timeout -k 10 300 python bench.py $S 2>> gpurun_out/${T}_ab.err) || exit 1
    echo "$round $v $(echo "$out" | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"])')" >> gpurun_out/${T}_ab.txt
  done
done
cat gpurun_out/${T}_ab.txt
