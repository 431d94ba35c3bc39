# Round 6: per-chunk r on the value-chunked LSA backward -- flash tests, the config-3 bf16 step test,
# FRA (config 5) tests unchanged, P = 16 / 32 benches
mkdir -p gpurun_out
T=${TAG:-r06m}
timeout -k 10 500 python -u -m pytest tests/test_gpu_lsa_flash.py "tests/test_gpu_parity2.py::test_cfg3_geometry_bf16_train_step_vs_reference_autocast" tests/test_gpu_fra_unet.py tests/test_gpu_fra_longn.py -q -p no:cacheprovider > gpurun_out/${T}_targeted.log 2>&1
rc=$?; echo "targeted rc=$rc" >> gpurun_out/${T}_targeted.log; tail -3 gpurun_out/${T}_targeted.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
S="--no-cpu-baseline --no-val-dice --no-trainer-faithful --no-live-trace --steps 30 --warmup 5"
: > gpurun_out/${T}_pools.jsonl
for p in 16 32; do
  timeout -k 10 300 python bench.py --pool $p $S >> gpurun_out/${T}_pools.jsonl 2>> gpurun_out/${T}_pools.err || exit 1
done
python -c "
import json
for l in open('gpurun_out/${T}_pools.jsonl'):
    d = json.loads(l); print(d['config']['pool_size'], d['value'], d['ms_per_step'])
"
