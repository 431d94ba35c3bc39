# Round 6: fused column pass + flash prep for the bf16 flash layers (knob 49): targeted tests, then A/B
# at P = 8 / 16 / 32
mkdir -p gpurun_out
T=${TAG:-r06x}
timeout -k 10 600 python -u -m pytest tests/test_gpu_lsa_flash.py tests/test_gpu_parity2.py tests/test_gpu_qk_ratio.py "tests/test_gpu_kernels.py::test_lsa_pool_direct_matches_sliced_pool" -q -s -p no:cacheprovider > gpurun_out/${T}_targeted.log 2>&1
rc=$?; echo "targeted rc=$rc" >> gpurun_out/${T}_targeted.log; tail -3 gpurun_out/${T}_targeted.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
S="--no-cpu-baseline --no-val-dice --no-trainer-faithful --no-live-trace --steps 40 --warmup 5"
: > gpurun_out/${T}_ab.txt
for round in 1 2; do
  for v in "X=0" "DFCSA_TUNE=49=0"; do
    for p in 8 16 32; do
      out=$(env $v timeout -k 10 300 python bench.py --pool $p $S 2>> gpurun_out/${T}_ab.err) || exit 1
      echo "$round $v P=$p $(echo "$out" | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> gpurun_out/${T}_ab.txt
    done
  done
done
cat gpurun_out/${T}_ab.txt
