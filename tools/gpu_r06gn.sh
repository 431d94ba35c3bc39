# Round 6: channel-chunked fused GroupNorm reductions (knob 50): TransUNet tests, then A/B on the
# TransUNet bf16 / fp32 step
mkdir -p gpurun_out
T=${TAG:-r06gn}
timeout -k 10 600 python -u -m pytest tests/test_gpu_transunet.py -q -p no:cacheprovider > gpurun_out/${T}_targeted.log 2>&1
rc=$?; echo "targeted rc=$rc" >> gpurun_out/${T}_targeted.log; tail -3 gpurun_out/${T}_targeted.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
S="--no-cpu-baseline --no-val-dice --no-trainer-faithful --no-live-trace --model transunet --batch 8 --steps 20 --warmup 3"
: > gpurun_out/${T}_ab.txt
for round in 1 2 3; do
  for v in "X=0" "DFCSA_TUNE=50=0"; do
    out=$(env $v timeout -k 10 300 python bench.py --precision bf16 $S 2>> gpurun_out/${T}_ab.err) || exit 1
    echo "$round $v bf16 $(echo "$out" | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> gpurun_out/${T}_ab.txt
  done
done
cat gpurun_out/${T}_ab.txt
