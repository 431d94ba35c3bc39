# Round 6: pooled-attention flash path with bf16 projections -- targeted tests, pool-size benches,
# then the driver's -m gpu command line
mkdir -p gpurun_out
T=${TAG:-r06k}
timeout -k 10 500 python -u -m pytest tests/test_gpu_lsa_flash.py tests/test_gpu_qk_ratio.py tests/test_gpu_oddwidth.py "tests/test_gpu_model.py::test_lsa_fp32" tests/test_gpu_parity2.py -q -p no:cacheprovider > gpurun_out/${T}_targeted.log 2>&1
rc=$?; echo "targeted rc=$rc" >> gpurun_out/${T}_targeted.log; tail -3 gpurun_out/${T}_targeted.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
S="--no-cpu-baseline --no-val-dice --no-trainer-faithful --no-live-trace --steps 30 --warmup 5"
: > gpurun_out/${T}_pools.jsonl
for p in 4 8 16 32; do
  timeout -k 10 300 python bench.py --pool $p $S >> gpurun_out/${T}_pools.jsonl 2>> gpurun_out/${T}_pools.err || exit 1
done
python -c "
import json
for l in open('gpurun_out/${T}_pools.jsonl'):
    d = json.loads(l); print(d['config']['pool_size'], d['value'], d['ms_per_step'])
"
timeout -k 10 900 python3 -m pytest tests/ -q -m gpu -p no:cacheprovider > gpurun_out/${T}_suite.log 2>&1
rc=$?; echo "suite rc=$rc" >> gpurun_out/${T}_suite.log; tail -3 gpurun_out/${T}_suite.log
exit $rc
