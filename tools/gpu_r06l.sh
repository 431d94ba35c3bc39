# Round 6: flash bwd with r from the rounded dO -- flash tests, the config-3 bf16 step test, pool benches
mkdir -p gpurun_out
T=${TAG:-r06l}
timeout -k 10 500 python -u -m pytest tests/test_gpu_lsa_flash.py "tests/test_gpu_parity2.py::test_cfg3_geometry_bf16_train_step_vs_reference_autocast" -q -s -p no:cacheprovider > gpurun_out/${T}_targeted.log 2>&1
rc=$?; echo "targeted rc=$rc" >> gpurun_out/${T}_targeted.log; tail -3 gpurun_out/${T}_targeted.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
DFCSA_LSA_FLASH_MIN_N=64 timeout -k 10 300 python -u -m pytest "tests/test_gpu_parity2.py::test_cfg3_geometry_bf16_train_step_vs_reference_autocast" -q -s -p no:cacheprovider > gpurun_out/${T}_cfg3_rowpath.log 2>&1
echo "rc=$?" >> gpurun_out/${T}_cfg3_rowpath.log
S="--no-cpu-baseline --no-val-dice --no-trainer-faithful --no-live-trace --steps 30 --warmup 5"
: > gpurun_out/${T}_pools.jsonl
for p in 8 16 32; do
  timeout -k 10 300 python bench.py --pool $p $S >> gpurun_out/${T}_pools.jsonl 2>> gpurun_out/${T}_pools.err || exit 1
done
DFCSA_LSA_FLASH_MIN_N=64 timeout -k 10 300 python bench.py --pool 8 $S >> gpurun_out/${T}_pools.jsonl 2>> gpurun_out/${T}_pools.err || exit 1
python -c "
import json
for l in open('gpurun_out/${T}_pools.jsonl'):
    d = json.loads(l); print(d['config']['pool_size'], d['value'], d['ms_per_step'])
"
