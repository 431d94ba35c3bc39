# Round 6: the one-wave-per-window pool also for windows of <= 8 x 8 pixels (P = 4 / 8 below 224^2):
# targeted tests, then A/B (knob 47 = 0: the sliced pool everywhere) at P = 4 / 8 / 16
mkdir -p gpurun_out
T=${TAG:-r06z}
timeout -k 10 900 python -u -m pytest tests/test_gpu_lsa_flash.py tests/test_gpu_parity2.py tests/test_gpu_qk_ratio.py tests/test_gpu_model.py "tests/test_gpu_kernels.py::test_lsa_pool_direct_matches_sliced_pool" tests/test_gpu_oddwidth.py -q -p no:cacheprovider > gpurun_out/${T}_targeted.log 2>&1
rc=$?; echo "targeted rc=$rc" >> gpurun_out/${T}_targeted.log; tail -3 gpurun_out/${T}_targeted.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
S="--no-cpu-baseline --no-val-dice --no-trainer-faithful --no-live-trace --steps 40 --warmup 5"
: > gpurun_out/${T}_ab.txt
for round in 1 2; do
  for v in "X=0" "DFCSA_TUNE=47=0"; do
    for p in 4 8 16; do
      out=$(env $v timeout -k 10 300 python bench.py --pool $p $S 2>> gpurun_out/${T}_ab.err) || exit 1
      echo "$round $v P=$p $(echo "$out" | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> gpurun_out/${T}_ab.txt
    done
  done
done
cat gpurun_out/${T}_ab.txt
